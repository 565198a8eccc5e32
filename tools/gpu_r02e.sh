#!/bin/bash
source tools/gpu_lib.sh r02e
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --large-actors 0
