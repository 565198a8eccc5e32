#!/bin/bash
# Round 6 A/B: k_dense_apply with a branch-free RING apply (the tree) vs HEAD (var/r06base3.so); the earlier
# variant that also loaded a full bucket's actor state in the items' round trip spilled (1.91 ms) or, at 4 waves
# per SIMD, lost occupancy (0.82 ms) -- reverted --
# tests, then the 10^8 ring (tools/perf.py medians, three alternations).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -q $T > gpurun_out/r06t_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06t_tests.log; exit 1; }
tail -1 gpurun_out/r06t_tests.log
for i in 1 2 3; do
  for lib in akka_amd/lib/var/r06base3.so akka_amd/lib/libakka_gpu.so; do
    AKKA_AMD_LIB=$lib timeout -k 10 200 python tools/perf.py --n 100000000 --steps 24 --reps 3 > gpurun_out/r06t_perf.json 2>&1 || { tail -5 gpurun_out/r06t_perf.json; exit 1; }
    echo "$(basename $lib) $(tail -1 gpurun_out/r06t_perf.json | cut -c1-200)"
  done
done
