#!/bin/bash
# FANOUT Zipf lookups hoisted out of the drain: GPU tests, then same-box A/B vs the HEAD build on C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03l}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "zipf or fanout or tiny or multipass or benched" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for c in C3_zipf_fanout C3_zipf_tree; do
  AB_REPS=2 bash tools/ab_cfg.sh $c $L akka_amd/lib/var/headfan.so >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
