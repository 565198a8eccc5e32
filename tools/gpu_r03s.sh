#!/bin/bash
# Diagnostics after the row copies: phase stamps of C4 ORSet full state and delta (fast and skew).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03s}
AGX_STAMPS=1 timeout -k 10 300 python tools/diag_c5.py --workload c4o --steps 3 > gpurun_out/${TAG}_c4o.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4o.log; exit 1; }
echo "== c4o"; grep -E "^step|agx stamps" gpurun_out/${TAG}_c4o.log | tail -3
AGX_STAMPS=1 timeout -k 10 300 python tools/diag_c5.py --workload c4od --steps 3 > gpurun_out/${TAG}_c4od.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4od.log; exit 1; }
AGX_STAMPS=1 AGX_STAMPS_SKEW=1 timeout -k 10 300 python tools/diag_c5.py --workload c4od --steps 4 > gpurun_out/${TAG}_c4od_skew.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4od_skew.log; exit 1; }
echo "== c4od"; grep -E "^step|agx stamps" gpurun_out/${TAG}_c4od.log | tail -5; grep -E "agx stamps" gpurun_out/${TAG}_c4od_skew.log | tail -4
