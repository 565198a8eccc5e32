#!/bin/bash
# Alive flags stored to LDS after the inbox loads (AGX_LATE_ALIVE): parity, then same-box A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03y}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
PERF_NS="1000000 100000000" AB_REPS=2 bash tools/ab.sh ${TAG} $L akka_amd/lib/var/nola.so || exit 1
for c in C5_power_law_bounded C3_zipf_fanout C3_zipf_tree; do
  AB_REPS=2 bash tools/ab_cfg.sh $c $L akka_amd/lib/var/nola.so >> gpurun_out/${TAG}_abc.log 2>&1 || { cat gpurun_out/${TAG}_abc.log; exit 1; }
done
cat gpurun_out/${TAG}_abc.log
