#!/bin/bash
# Round 6: is round 4's counter fault the ockl __syncthreads_and in the presorted check?  The
# sparse-serial build with that reduction restored (r06old, three times), then its LDS-shadow builds
# (old1: flush the LDS shadow count, old2: flush the acc registers); then the dense profile test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 100 --timeout-method thread -p no:cacheprovider"
for v in ${VARS:-r06old r06old r06old r06old1 r06old2 r06old1 r06old2}; do
  AKKA_AMD_LIB=akka_amd/lib/var/$v.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -q \
    -k "test_multipass_grouping and crdt" $T > gpurun_out/r06e_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"; grep -a "emitted\|passed\|failed" gpurun_out/r06e_$v.log | cut -c1-240 | head -8
  [ $rc -le 1 ] || exit 1
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_dense.py -q -k "profile_counts" $T > gpurun_out/r06e_dense.log 2>&1 || { tail -30 gpurun_out/r06e_dense.log; exit 1; }
tail -1 gpurun_out/r06e_dense.log
