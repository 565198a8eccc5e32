#!/bin/bash
source tools/gpu_lib.sh r02g
step delta 600 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_typed.py -x -v --timeout 300 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
