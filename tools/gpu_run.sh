#!/bin/bash
# One GPU session on an MI355X box (tools/gpu_run.sh TAG).  Steps are chosen by environment:
#   BUILD=1   rebuild libakka_gpu.so on the box from the sources (proves build() there; logs time)
#   TESTS=1   pytest -m gpu (TEST_ARGS: extra pytest arguments, e.g. -k expr)
#   BENCH=1   bench.py ${BENCH_ARGS} -> TAG_bench.json
#   PROF=1    rocprofv3 --kernel-trace --stats of bench.py ${PROF_ARGS}
#   PMC="FETCH_SIZE WRITE_SIZE"  one rocprofv3 --pmc pass per group (PMC_ARGS = bench.py arguments)
#   CMD="..." any extra command (run last, under its own time limit)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
fail() { echo "$1 failed"; tail -40 "$2"; exit 1; }
if [ -n "$BUILD" ]; then
  t0=$(date +%s)
  timeout -k 10 600 python -c "import __graft_entry__ as g; g.build_native(force=True)" > gpurun_out/${TAG}_build.log 2>&1 || fail build gpurun_out/${TAG}_build.log
  echo "build on the box: $(( $(date +%s) - t0 )) s" | tee -a gpurun_out/${TAG}_build.log
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 280 --timeout-method thread ${TEST_ARGS} > gpurun_out/${TAG}_pytest.log 2>&1 || fail pytest gpurun_out/${TAG}_pytest.log
  tail -3 gpurun_out/${TAG}_pytest.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || fail bench gpurun_out/${TAG}_bench.err
  tail -c 3000 gpurun_out/${TAG}_bench.json
fi
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py ${PROF_ARGS:---no-cpu-baseline --no-configs} > gpurun_out/${TAG}_prof.log 2>&1 || fail rocprof gpurun_out/${TAG}_prof.log
  head -30 gpurun_out/${TAG}_prof/run_kernel_stats.csv
fi
i=0
for grp in ${PMC}; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc ${grp//,/ } --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- python3 bench.py ${PMC_ARGS:---no-cpu-baseline --no-configs --steps 40 --warmup 4} > gpurun_out/${TAG}_pmc$i.log 2>&1 || fail "pmc pass $i ($grp)" gpurun_out/${TAG}_pmc$i.log
  echo "pmc pass $i ok: $grp"
done
if [ -n "$CMD" ]; then
  timeout -k 10 ${CMD_TIMEOUT:-600} bash -c "$CMD" > gpurun_out/${TAG}_cmd.log 2>&1 || fail cmd gpurun_out/${TAG}_cmd.log
  tail -30 gpurun_out/${TAG}_cmd.log
fi
echo "gpu_run $TAG done"
