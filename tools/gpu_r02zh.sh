#!/bin/bash
# create-time memsets synchronized before the first upload: the failing case, then the full GPU suite
source tools/gpu_lib.sh r02zh
step one 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bucket_width_multipass"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
