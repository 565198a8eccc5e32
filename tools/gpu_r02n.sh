#!/bin/bash
# round-2 (session 3) baseline on a fresh box: GPU parity suite, the driver's bench command
source tools/gpu_lib.sh r02n
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 600 python -u bench.py --steps 20 --warmup 5
