#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run; --pmc never combined with trace domains).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
ARGS="--steps 40 --warmup 4 --no-cpu-baseline --no-configs ${BENCH_ARGS}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc ${grp//,/ } --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 gpurun_out/${TAG}_p$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
