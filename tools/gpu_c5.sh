#!/bin/bash
# Multi-pass iteration: full GPU parity tests, then C5 / C3 per-step kernel breakdown and the 100M ring.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c5}
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for w in ${C5_WORKLOADS:-c5 c3}; do
  timeout -k 10 300 python tools/diag_c5.py --workload $w --steps 3 > gpurun_out/${TAG}_diag_$w.log 2>&1 || { echo "diag $w failed"; tail -20 gpurun_out/${TAG}_diag_$w.log; exit 1; }
  cat gpurun_out/${TAG}_diag_$w.log
done
if [ -n "$C5_RING" ]; then
  timeout -k 10 200 python tools/perf.py --n 100000000 --steps 20 --reps 3 --prof > gpurun_out/${TAG}_ring100m.jsonl 2>gpurun_out/${TAG}_ring100m.err || { tail -20 gpurun_out/${TAG}_ring100m.err; exit 1; }
  cat gpurun_out/${TAG}_ring100m.jsonl
fi
