#!/bin/bash
# Wave path of up to 256 messages (4 per lane): multi-pass GPU tests, then same-box A/B vs the
# 128-message build (AGX_TINY_IPL=2) on C5 / C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03k}
L=akka_amd/lib/libakka_gpu.so
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for c in C5_power_law_bounded C3_zipf_fanout C3_zipf_tree; do
  AB_REPS=2 bash tools/ab_cfg.sh $c $L akka_amd/lib/var/ipl2.so >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
