#!/bin/bash
# budget end spin-waited on an event: strict/replay parity + headline A/B
source tools/gpu_lib.sh r02zk
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benched.py -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  for lib in ab_prev libakka_gpu; do
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step b20_${lib}_$rep 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --large-actors 0
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step b200_${lib}_$rep 300 python -u bench.py --steps 200 --warmup 16 --no-configs --no-cpu-baseline --large-actors 0
  done
done
