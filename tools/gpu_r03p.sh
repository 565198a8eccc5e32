#!/bin/bash
# Queued-gossip row copies by the whole wave: CRDT / RCCL GPU tests, then same-box A/B vs HEAD on C4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03p}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "crdt or orset or gossip or rccl or delta or sharded" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for c in C4_orset_gossip C4_orset_delta_gossip C4_gcounter_gossip; do
  AB_REPS=2 bash tools/ab_cfg.sh $c $L akka_amd/lib/var/headrow.so >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
