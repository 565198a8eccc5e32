#!/bin/bash
# Round 6: persistent fused supersteps -- dense tests first (persist on / off), the boundary tests,
# then a same-box A/B of the 1M ring (AGX_PERSIST=1 / 0, three alternations), then the sparse-serial
# shadow experiment.  Each GPU step has its own limit; a crash or timeout ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_dense.log 2>&1 || { echo "dense tests failed"; tail -40 gpurun_out/${TAG}_dense.log; exit 1; }
tail -1 gpurun_out/${TAG}_dense.log
for i in 1 2 3; do
  for p in 1 0; do
    AGX_PERSIST=$p timeout -k 10 120 python tools/perf.py --n 1000000 --steps 200 --reps 5 > gpurun_out/${TAG}_perf_p${p}_${i}.json 2>&1 || { echo "perf failed"; tail -5 gpurun_out/${TAG}_perf_p${p}_${i}.json; exit 1; }
    echo "persist=$p $(tail -1 gpurun_out/${TAG}_perf_p${p}_${i}.json)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tellq.py tests/test_abi_c.py tests/test_rccl_ranks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_boundary.log 2>&1 || { echo "boundary tests failed"; tail -40 gpurun_out/${TAG}_boundary.log; exit 1; }
tail -1 gpurun_out/${TAG}_boundary.log
bash tools/gpu_r06b.sh
