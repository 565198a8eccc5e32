#!/bin/bash
# Round 6: multi-rank owner apply -- rocprofv3 kernel stats of the R = 8 loopback group with the
# dense owner launch (AGX_DENSE_OWNER=1) against the block launch (default); one hardware queue, so the
# eight engines' kernels do not overlap and each duration is one rank's own.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06i}
for d in 1 0; do
  GPU_MAX_HW_QUEUES=1 AGX_DENSE_OWNER=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_d$d -o pg --output-format csv -- python3 tools/perf_group.py --ranks 8 --steps 20 > gpurun_out/${TAG}_d$d.log 2>&1 || { tail -30 gpurun_out/${TAG}_d$d.log; exit 1; }
  tail -1 gpurun_out/${TAG}_d$d.log
  f=$(find gpurun_out/${TAG}_d$d -name "*kernel_stats.csv" | head -1); python3 -c "import csv,sys; [print(\"  %-60s %5s min %7.1f avg %7.1f\" % (x[\"Name\"][:60], x[\"Calls\"], float(x[\"MinNs\"])/1e3, float(x[\"AverageNs\"])/1e3)) for x in list(csv.DictReader(open(sys.argv[1])))[:12]]" "$f"
done
