#!/bin/bash
# apply counters flushed once per block (multi-pass / fused fast path), per bucket elsewhere: parity + A/B
source tools/gpu_lib.sh r02zc
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
AB_REPS=2 PERF_STEPS=40 step ab 600 bash tools/ab.sh r02zc akka_amd/lib/ab_prev.so akka_amd/lib/libakka_gpu.so
for lib in ab_prev libakka_gpu; do
  AKKA_AMD_LIB=akka_amd/lib/$lib.so step c5_$lib 300 python -u tools/cfg_one.py C5_power_law_bounded
done
