#!/bin/bash
# Skew-path CRDT descriptor loads batched kPF at a time: CRDT GPU tests, then same-box A/B vs HEAD on C4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03t}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "crdt or delta or orset or gossip or skew" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for c in C4_orset_delta_gossip C4_gcounter_delta_gossip C4_orset_gossip; do
  AB_REPS=2 bash tools/ab_cfg.sh $c $L akka_amd/lib/var/headpf.so >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
