#!/bin/bash
# skew split v2 (backlog parts streamed, single-pass drain in the skew launch): parity, C5/C3, kernel times
source tools/gpu_lib.sh r02q
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benched.py -x -q --timeout 300 --timeout-method thread
step c5 300 python -u tools/cfg_one.py C5_power_law_bounded
step c3 300 python -u tools/cfg_one.py C3_zipf_fanout
step c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02q/prof -o c5 -- python3 -u tools/cfg_one.py C5_power_law_bounded
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
