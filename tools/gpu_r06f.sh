#!/bin/bash
# Round 6: (1) round 4's counter fault on its own tree (21fc9ac + -DAGX_SPARSE_SERIAL, three runs);
# (2) agx_run's host overhead per budget on the 1M ring; (3) C5 at 100M: backlog arena (default) vs
# the ring pool (AGX_RING_SLOTS=8192) vs the ring apply (AGX_RING_APPLY=1), the bench's window.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 100 --timeout-method thread -p no:cacheprovider"
for v in r21ser r21ser r21ser; do
  AKKA_AMD_LIB=akka_amd/lib/var/$v.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -q \
    -k "test_multipass_grouping and crdt" $T > gpurun_out/r06f_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"; grep -a "emitted\|passed\|failed" gpurun_out/r06f_$v.log | cut -c1-240 | head -8
  [ $rc -le 1 ] || exit 1
done
timeout -k 10 120 python tools/host_overhead.py > gpurun_out/r06f_overhead.log 2>&1 || { tail -5 gpurun_out/r06f_overhead.log; exit 1; }
cat gpurun_out/r06f_overhead.log
for e in "X=0" "AGX_RING_SLOTS=8192" "AGX_RING_APPLY=1"; do
  env $e timeout -k 10 300 python tools/cfg_one.py C5_power_law_bounded > gpurun_out/r06f_c5_${e%%=*}.json 2> gpurun_out/r06f_c5_${e%%=*}.err || { tail -5 gpurun_out/r06f_c5_${e%%=*}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['C5_power_law_bounded']; print(sys.argv[2], '%.3g'%d['value'], round(d['ms_per_step'],3), d.get('kernel_ms_per_step'))" gpurun_out/r06f_c5_${e%%=*}.json "$e"
done
