#!/bin/bash
# Row copies (wave for long rows, lane for short) and the FORWARD_RR edge prefetch: GPU tests, then
# same-box A/B on C4 (vs HEAD) and C5 (vs the build without the prefetch).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03q}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
AB_REPS=2 bash tools/ab_cfg.sh C5_power_law_bounded $L akka_amd/lib/var/nofwdpre.so > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
for c in C4_gcounter_gossip C4_orset_gossip; do
  bash tools/ab_cfg.sh $c $L akka_amd/lib/var/headrow.so >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
