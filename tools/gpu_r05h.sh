#!/bin/bash
# A/B of the tree's build against variant libs on the 1M / 100M ring (tools/perf.py medians); dense parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -q -x --timeout 110 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05h_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r05h_pytest.log; [ $rc -eq 0 ] || exit 1
for n in ${NS:-1000000}; do
  st=60; [ $n -gt 1000000 ] && st=8
  for rep in 1 2; do
    for lib in akka_amd/lib/libakka_gpu.so $VARS; do
      AKKA_AMD_LIB=$lib timeout -k 10 200 python tools/perf.py --n $n --steps $st --reps 5 > gpurun_out/r05h.json 2> gpurun_out/r05h.err \
        || { tail -5 gpurun_out/r05h.err; exit 1; }
      echo "$n $(basename $lib): $(python -c "import json;d=json.loads(open('gpurun_out/r05h.json').read().strip().splitlines()[-1]);print(round(d['us_per_step_median'],2), 'us')")"
    done
  done
done
