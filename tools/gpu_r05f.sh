#!/bin/bash
# Round 5: k_dense_apply with the next bucket's bounds loaded one bucket ahead -- dense tests, then
# 100M ring A/B (tools/perf.py medians, graph-replayed supersteps), 3 alternations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_dense.py} > gpurun_out/f_tests.log 2>&1 || { tail -30 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
for rep in 1 2 3; do
  for lib in ${BASE:-akka_amd/lib/var/dhead.so} akka_amd/lib/libakka_gpu.so; do
    AKKA_AMD_LIB=$lib timeout -k 10 200 python tools/perf.py --n 100000000 --steps 20 --reps 5 > gpurun_out/f_tmp.json 2>gpurun_out/f_ab.err || { tail -20 gpurun_out/f_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/f_tmp.json')); print('$lib', d['n'], round(d['us_per_step_median'],1))" | tee -a gpurun_out/f_ab.txt
  done
done
