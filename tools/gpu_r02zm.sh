#!/bin/bash
# packed exchange build (branch packed-exchange) through AKKA_AMD_LIB: RCCL multi-process parity + loopback
source tools/gpu_lib.sh r02zm
export AKKA_AMD_LIB=akka_amd/lib/packed.so
step rccl 600 python -u -m pytest tests/test_rccl_ranks.py -x -v --timeout 280 --timeout-method thread
step shard 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread -k "shard or loopback or group"
