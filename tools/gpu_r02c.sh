#!/bin/bash
source tools/gpu_lib.sh r02c
step bench20 240 python -u bench.py --steps 20 --warmup 5 --no-configs --large-actors 0 --no-cpu-baseline
step bench200 240 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
step rccl 600 python -u -m pytest tests/test_rccl_ranks.py -x -v --timeout 300 --timeout-method thread
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "strict or ring or zipf"
