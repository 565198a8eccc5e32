#!/bin/bash
# tiny path: batched loads + readlane rank loop; skew grid 512: parity + same-box A/B on C5 / C3
source tools/gpu_lib.sh r02x
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  for lib in ab_prev libakka_gpu; do
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step c5_${lib}_$rep 300 python -u tools/cfg_one.py C5_power_law_bounded
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step c3_${lib}_$rep 300 python -u tools/cfg_one.py C3_zipf_fanout
  done
done
