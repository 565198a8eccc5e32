#!/bin/bash
# Paired state layout + ring drain batching: GPU tests, then same-box A/B on C5 / C3 / mixed configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03b}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
AB_REPS=2 bash tools/ab_cfg.sh C5_power_law_bounded $L $L:AGX_STATE_SOA=1 $L:AGX_RING_SLOTS=0 > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
bash tools/ab_cfg.sh C3_zipf_fanout $L $L:AGX_STATE_SOA=1 $L:AGX_RING_SLOTS=0 >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
bash tools/ab_cfg.sh C3_zipf_tree $L $L:AGX_STATE_SOA=1 $L:AGX_RING_SLOTS=0 >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
AB_REPS=2 bash tools/ab.sh ${TAG}ring $L akka_amd/lib/var/noearly.so > gpurun_out/${TAG}_abring.log 2>&1 || { cat gpurun_out/${TAG}_abring.log; exit 1; }
cat gpurun_out/${TAG}_abring.log
