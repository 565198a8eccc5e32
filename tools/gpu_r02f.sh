#!/bin/bash
source tools/gpu_lib.sh r02f
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench20 300 python -u bench.py --steps 20 --warmup 5
