#!/bin/bash
# Round 6: void priming launch of freshly captured strict replays -- dense / recovery / parity tests,
# then the first-run timing (tools/first_run2.py) with and without it (AGX_NO_PRIME=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_tellq.py -q $T > gpurun_out/r06x_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06x_tests.log; exit 1; }
tail -1 gpurun_out/r06x_tests.log
timeout -k 10 200 python tools/first_run2.py > gpurun_out/r06x_fr.log 2>&1 || { tail -5 gpurun_out/r06x_fr.log; exit 1; }
grep run gpurun_out/r06x_fr.log
AGX_NO_PRIME=1 timeout -k 10 200 python tools/first_run2.py > gpurun_out/r06x_fr0.log 2>&1 || { tail -5 gpurun_out/r06x_fr0.log; exit 1; }
sed 's/^/noprime /' gpurun_out/r06x_fr0.log | grep run
