#!/bin/bash
# Diagnostics: phase stamps of the C4 full-state ORSet / GCounter applies and of C5 / C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03o}
for w in c4o c4g c5 c3; do
  AGX_STAMPS=1 timeout -k 10 300 python tools/diag_c5.py --workload $w --steps 3 > gpurun_out/${TAG}_$w.log 2>&1 || { tail -20 gpurun_out/${TAG}_$w.log; exit 1; }
  echo "== $w"; grep -E "^step|agx stamps" gpurun_out/${TAG}_$w.log | tail -3
done
