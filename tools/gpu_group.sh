#!/bin/bash
# Multi-rank iteration: loopback/sharded GPU parity tests, then tools/perf_group.py at R=2,4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-grp}
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "${GROUP_K:-loopback or sharded or multipass}" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for r in ${GROUP_RS:-2 4}; do
  timeout -k 10 200 python tools/perf_group.py --ranks $r --n ${GROUP_N:-1000000} >> gpurun_out/${TAG}_group.jsonl 2>gpurun_out/${TAG}_group.err || { echo "perf_group failed"; tail -20 gpurun_out/${TAG}_group.err; exit 1; }
done
cat gpurun_out/${TAG}_group.jsonl
