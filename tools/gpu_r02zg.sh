#!/bin/bash
# ORSet runs: vvector re-read per batch (spills 34 -> 27): CRDT parity + C4 ORSet A/B
source tools/gpu_lib.sh r02zg
step par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_benched.py tests/test_gpu_delta_crdt.py -x -q --timeout 300 --timeout-method thread -k "crdt or orset or ORSet or C4 or gossip or counter"
for rep in 1 2; do
  for lib in ab_prev libakka_gpu; do
    AKKA_AMD_LIB=akka_amd/lib/$lib.so step c4o_${lib}_$rep 300 python -u tools/cfg_one.py C4_orset_gossip
  done
done
