#!/bin/bash
# ORSet merge software pipeline: CRDT GPU tests, then same-box A/B on C4 ORSet vs the HEAD build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03g}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "crdt or orset or gossip" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
AB_REPS=2 bash tools/ab_cfg.sh C4_orset_gossip $L akka_amd/lib/var/headorset.so > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
