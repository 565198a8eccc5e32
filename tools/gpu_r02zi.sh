#!/bin/bash
# multi-pass apply grid = one wave-per-bucket group per block: parity + C3/C5 A/B
source tools/gpu_lib.sh r02zi
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for lib in ab_prev libakka_gpu; do
  for c in C3_zipf_fanout C3_zipf_tree C5_power_law_bounded; do
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step ${c}_$lib 300 python -u tools/cfg_one.py $c
  done
done
