#!/bin/bash
# skewed buckets split over workgroups: multi-pass parity, then C5 / C3 configs
source tools/gpu_lib.sh r02o
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benched.py -x -q --timeout 300 --timeout-method thread -k "tiny or multipass or power_law or zipf or C5 or c5 or C3 or c3 or skew or mixed"
step c5 300 python -u tools/cfg_one.py C5_power_law_bounded
step c3 300 python -u tools/cfg_one.py C3_zipf_fanout
step c3t 300 python -u tools/cfg_one.py C3_zipf_tree
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
