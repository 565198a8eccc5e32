#!/bin/bash
# apply counters flushed once per block: parity + same-box A/B (ring 1M/100M, C5, C3)
source tools/gpu_lib.sh r02zb
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
AB_REPS=2 PERF_STEPS=40 step ab 600 bash tools/ab.sh r02zb akka_amd/lib/ab_prev.so akka_amd/lib/libakka_gpu.so
for lib in ab_prev libakka_gpu; do
  AKKA_AMD_LIB=akka_amd/lib/$lib.so step c5_$lib 300 python -u tools/cfg_one.py C5_power_law_bounded
  AKKA_AMD_LIB=akka_amd/lib/$lib.so step c3_$lib 300 python -u tools/cfg_one.py C3_zipf_fanout
done
