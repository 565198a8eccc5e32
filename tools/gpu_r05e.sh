#!/bin/bash
# Round 5: k_dense_fused prologue (one bucket outside a loop, loads back to back) -- dense tests, then
# 1M ring A/B without per-class events (graph-replayed supersteps), 3 alternations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_dense.py tests/test_gpu_parity.py} > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
for rep in 1 2 3; do
  for lib in ${BASE:-akka_amd/lib/var/dold.so} akka_amd/lib/libakka_gpu.so; do
    AKKA_AMD_LIB=$lib timeout -k 10 200 python tools/perf.py --n 1000000 --steps 100 --reps 7 > gpurun_out/e_tmp.json 2>gpurun_out/e_ab.err || { tail -20 gpurun_out/e_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/e_tmp.json')); print('$lib', d['n'], round(d['us_per_step_median'],2))" | tee -a gpurun_out/e_ab.txt
  done
done
