#!/bin/bash
# multi-rank per-superstep cost (loopback group, 1M actors per rank), kernel stats
source tools/gpu_lib.sh r02w
step g2 300 python -u tools/perf_group.py --ranks 2 --n 1000000 --steps 20
step g8 300 python -u tools/perf_group.py --ranks 8 --n 1000000 --steps 10
step g2prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02w/prof -o g2 -- python3 -u tools/perf_group.py --ranks 2 --n 1000000 --steps 20
step rccl 300 python -u -m pytest tests/test_rccl_ranks.py -x -q --timeout 280 --timeout-method thread
