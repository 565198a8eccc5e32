#!/bin/bash
# Round 6: delta-CRDT parity with ORSet delta replicas in 2048-replica buckets (the workload default).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_fullsize.py tests/test_gpu_benched.py tests/test_rccl_ranks.py -q -k "delta" $T > gpurun_out/r06d3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06d3_tests.log; exit 1; }
tail -1 gpurun_out/r06d3_tests.log
