#!/bin/bash
# PMC passes over tools/perf.py (each counter group in its own rocprofv3 run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmcp}
i=0
for grp in ${GROUPS_LIST}; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc ${grp//,/ } --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 tools/perf.py --steps 20 --reps 1 ${PERF_ARGS} > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py "gpurun_out/${TAG}_p*/run_counter_collection.csv"
