#!/bin/bash
# round-5 diagnostics: sparse-row A/B variants, RCCL row-slab fallback cases, captured multi-rank replay
set -o pipefail
mkdir -p gpurun_out
T="--timeout 100 --timeout-method thread -p no:cacheprovider"
for v in ${VARS:-knob_c8630 wpe2_c8630}; do
  AKKA_AMD_LIB=akka_amd/lib/var/$v.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -q \
    -k "test_multipass_grouping and crdt" $T > gpurun_out/mp_$v.log 2>&1
  echo "$v rc=$?"; tail -3 gpurun_out/mp_$v.log
done
timeout -k 10 500 python -u -m pytest tests/test_rccl_ranks.py -v -k "orset" --timeout 290 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/rccl_orset.log 2>&1 || { echo "rccl orset failed"; tail -30 gpurun_out/rccl_orset.log; exit 1; }
tail -3 gpurun_out/rccl_orset.log
for w in orset zipf; do
  AGX_MR_ROW_MB=0 timeout -k 10 150 python -u tools/rccl_two_rank.py --split-hosts --world 2 --n 6000 --hops 6 --workload $w \
    > gpurun_out/xinfo_host_$w.log 2>&1 && timeout -k 10 150 python -u tools/rccl_two_rank.py --split-hosts --world 2 --n 6000 \
    --hops 6 --workload $w > gpurun_out/xinfo_dev_$w.log 2>&1 || { echo "xinfo $w failed"; exit 1; }
  grep -h "exchange rank\|parity" gpurun_out/xinfo_host_$w.log gpurun_out/xinfo_dev_$w.log
done
if [ -n "$MRGRAPH" ]; then
  AGX_MR_GRAPH=1 AGX_MR_DEBUG=1 NCCL_DEBUG=WARN timeout -k 10 120 python -u tools/rccl_two_rank.py --split-hosts --world 2 \
    --n 20000 --hops 24 --workload ring > gpurun_out/mrgraph.log 2>&1
  echo "mrgraph rc=$?"; tail -25 gpurun_out/mrgraph.log
fi
