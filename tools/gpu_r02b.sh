#!/bin/bash
source tools/gpu_lib.sh r02b
step bench20 240 python -u bench.py --steps 20 --warmup 5 --no-configs --large-actors 0 --no-cpu-baseline
step bench200 240 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
