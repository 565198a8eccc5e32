#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/pg -o pg --output-format csv -- python3 tools/perf_group.py --ranks 2 --steps 20 > gpurun_out/pg.log 2>&1 || { tail -30 gpurun_out/pg.log; exit 1; }
find gpurun_out/pg -name "*stats*" | head
