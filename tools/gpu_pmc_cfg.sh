#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 --pmc run per counter, no trace domains) over single
# BASELINE configs (tools/cfg_one.py) -- tools/gpu_pmc_cfg.sh TAG CONFIG...
# Summaries: python3 tools/pmc_summary.py 'gpurun_out/TAG_*_p*/**/*counter_collection.csv'
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmccfg}
shift
for cfg in "$@"; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${cfg}_p$i -o run -- \
      python3 tools/cfg_one.py $cfg > gpurun_out/${TAG}_${cfg}_p$i.log 2>&1 || { echo "pmc $cfg $grp failed"; tail -20 gpurun_out/${TAG}_${cfg}_p$i.log; exit 1; }
    echo "pmc $cfg $grp ok"
  done
done
