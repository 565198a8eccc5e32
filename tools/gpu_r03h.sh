#!/bin/bash
# Diagnostics: phase stamps of the fast and the skew apply launches on the C4 delta configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03h}
for w in c4od c4gd; do
  AGX_STAMPS=1 timeout -k 10 200 python tools/diag_c5.py --workload $w --steps 3 > gpurun_out/${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/${TAG}_$w.log; exit 1; }
  AGX_STAMPS=1 AGX_STAMPS_SKEW=1 timeout -k 10 200 python tools/diag_c5.py --workload $w --steps 3 > gpurun_out/${TAG}_${w}_skew.log 2>&1 || { tail -20 gpurun_out/${TAG}_${w}_skew.log; exit 1; }
  echo "== $w"; grep -E "^step|agx stamps" gpurun_out/${TAG}_$w.log | tail -4; grep -E "agx stamps" gpurun_out/${TAG}_${w}_skew.log | tail -2
done
