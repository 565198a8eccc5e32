#!/bin/bash
source tools/gpu_lib.sh r02j
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step c3 300 python -u tools/cfg_one.py C3_zipf_fanout
step c5 300 python -u tools/cfg_one.py C5_power_law_bounded
step c4d_orset 300 python -u tools/cfg_one.py C4_orset_delta_gossip
step c4d_gc 300 python -u tools/cfg_one.py C4_gcounter_delta_gossip
