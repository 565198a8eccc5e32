#!/bin/bash
# packed (key, src, payload) send per peer: RCCL multi-process parity, then the full GPU suite
source tools/gpu_lib.sh r02zl
step rccl 600 python -u -m pytest tests/test_rccl_ranks.py -x -v --timeout 280 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
