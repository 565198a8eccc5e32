#!/bin/bash
source tools/gpu_lib.sh r02l
step tiny 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "tiny or multipass or power_law or zipf"
step c3 300 python -u tools/cfg_one.py C3_zipf_fanout
AGX_TINY=0 step c3_off 300 python -u tools/cfg_one.py C3_zipf_fanout
step c3t 300 python -u tools/cfg_one.py C3_zipf_tree
step c5 300 python -u tools/cfg_one.py C5_power_law_bounded
AGX_TINY=0 step c5_off 300 python -u tools/cfg_one.py C5_power_law_bounded
step ring100m 300 python -u bench.py --steps 8 --warmup 2 --no-configs --no-cpu-baseline --large-steps 24
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
