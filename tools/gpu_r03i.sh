#!/bin/bash
# Delta-CRDT state layout A/B: actor-major rows (default) vs word-major (AGX_CRDT_WORDMAJOR=1);
# the delta parity tests under both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03i}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "delta" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
AGX_CRDT_WORDMAJOR=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "delta" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest_wm.log 2>&1 || { echo "pytest (word-major) failed"; tail -40 gpurun_out/${TAG}_pytest_wm.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_wm.log
AB_REPS=2 bash tools/ab_cfg.sh C4_orset_delta_gossip $L $L:AGX_CRDT_WORDMAJOR=1 > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
bash tools/ab_cfg.sh C4_gcounter_delta_gossip $L $L:AGX_CRDT_WORDMAJOR=1 >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
