#!/bin/bash
# Round deliverables on one MI355X: GPU parity tests, PMC traffic passes,
# the bench line (with CPU baseline), rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
B1M="--no-cpu-baseline --large-actors 0 --no-configs"
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }

if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || fail pytest gpurun_out/${TAG}_pytest.log
  tail -2 gpurun_out/${TAG}_pytest.log
fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py $B1M --steps 40 --warmup 4 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || fail pmc_fetch gpurun_out/${TAG}_pmc_fetch.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py $B1M --steps 40 --warmup 4 > gpurun_out/${TAG}_pmc_write.log 2>&1 || fail pmc_write gpurun_out/${TAG}_pmc_write.log
python3 tools/pmc_to_json.py gpurun_out/pmc_${TAG}.json gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write \
  --note "bench.py $B1M --steps 40 --warmup 4 (C2 ring, 1M actors)" > /dev/null || exit 1
timeout -k 10 900 python bench.py --pmc gpurun_out/pmc_${TAG}.json ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || fail bench gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py $B1M --pmc gpurun_out/pmc_${TAG}.json > gpurun_out/${TAG}_prof.log 2>&1 || fail rocprof gpurun_out/${TAG}_prof.log
cat gpurun_out/${TAG}_prof/run_kernel_stats.csv
