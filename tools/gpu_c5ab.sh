#!/bin/bash
# C5 / C3: bounded-mailbox rings on vs off (same box), then the C5 kernel trace summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c5ab}
L=akka_amd/lib/libakka_gpu.so
AB_REPS=2 bash tools/ab_cfg.sh C5_power_law_bounded $L $L:AGX_RING_SLOTS=0 > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
bash tools/ab_cfg.sh C3_zipf_fanout $L $L:AGX_RING_SLOTS=0 >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/cfg_one.py C5_power_law_bounded > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cut -d, -f1-8 {} \; | head -30
