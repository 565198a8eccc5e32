#!/bin/bash
# Round 6: owner-mode dense launch with direct owner-class placement + the dense_left shortcut in owner
# mode -- the sharded dense tests, the RCCL ranks, then the single-queue R = 8 loopback profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06j}
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -q -k "sharded or loopback" $T > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
AGX_DENSE_OWNER=1 timeout -k 10 400 python -u -m pytest tests/test_rccl_ranks.py -q $T > gpurun_out/${TAG}_rccl.log 2>&1 || { echo "rccl tests failed"; tail -40 gpurun_out/${TAG}_rccl.log; exit 1; }
tail -1 gpurun_out/${TAG}_rccl.log
bash tools/gpu_r06i.sh ${TAG}p
