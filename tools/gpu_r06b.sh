#!/bin/bash
# Round 6: the sparse-serial counter fault -- the knob build three times (is the wrong
# count deterministic?), then the LDS-shadow builds (1: flush the LDS shadow, 2: flush the registers).
set -o pipefail
mkdir -p gpurun_out
T="--timeout 100 --timeout-method thread -p no:cacheprovider"
for v in ${VARS:-r06ser r06ser r06ser r06sh1 r06sh2 r06sh1 r06sh2}; do
  AKKA_AMD_LIB=akka_amd/lib/var/$v.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -q \
    -k "test_multipass_grouping and crdt" $T > gpurun_out/r06b_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"; grep -a "emitted gpu\|passed\|failed" gpurun_out/r06b_$v.log | cut -c1-200
  [ $rc -le 1 ] || exit 1
done
