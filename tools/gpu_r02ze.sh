#!/bin/bash
# replay rows written to the host ring by the graph's last kernel (no D2H copy per replay):
# strict-replay recovery + full parity, then headline A/B at the driver's step counts
source tools/gpu_lib.sh r02ze
step strict 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "strict or ring or mixed"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  for lib in ab_prev libakka_gpu; do
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step b20_${lib}_$rep 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step b200_${lib}_$rep 300 python -u bench.py --steps 200 --warmup 16 --no-configs --no-cpu-baseline --large-actors 0
  done
done
