#!/bin/bash
# GPU iteration: parity tests, bench, rocprofv3 kernel stats.  Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 100 --warmup 8 --no-cpu-baseline --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
  cat gpurun_out/${TAG}_prof/run_kernel_stats.csv
fi
