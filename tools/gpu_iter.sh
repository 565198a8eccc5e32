#!/bin/bash
# Iteration: GPU parity tests, then A/B perf at 1M and 100M ring (per-kernel breakdown).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-it}
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for n in ${PERF_NS:-1000000 100000000}; do
  timeout -k 10 200 python tools/perf.py --n $n --steps ${PERF_STEPS:-40} --reps 5 --prof ${PERF_ARGS} >> gpurun_out/${TAG}_perf.jsonl 2>gpurun_out/${TAG}_perf.err || { echo "perf failed"; tail -20 gpurun_out/${TAG}_perf.err; exit 1; }
done
cat gpurun_out/${TAG}_perf.jsonl
