#!/bin/bash
# Round 6 A/B: branch-free RING apply in k_dense_fused (the tree) vs HEAD (var/r06base.so): dense
# tests first, then 1M ring medians (three alternations) and rocprofv3 kernel stats of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q $T > gpurun_out/r06q_dense.log 2>&1 || { echo "dense tests failed"; tail -30 gpurun_out/r06q_dense.log; exit 1; }
tail -1 gpurun_out/r06q_dense.log
sed -i 's/^  for lib in akka_amd\/lib\/var\/r06base.so akka_amd\/lib\/libakka_gpu.so; do$/  for lib in akka_amd\/lib\/var\/r06base.so akka_amd\/lib\/libakka_gpu.so; do/' tools/gpu_r06o.sh
bash tools/gpu_r06o.sh
