#!/bin/bash
# round-5: NT-store A/B at 1M (fused) and 100M (multi-pass dense launch); dense parity subset first
set -o pipefail
mkdir -p gpurun_out
T="--timeout 110 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -q -x $T > gpurun_out/r05c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05c_pytest.log; [ $rc -eq 0 ] || exit 1
for n in 1000000 100000000; do
  st=60; [ $n -gt 1000000 ] && st=8
  for v in nt1 nt0; do
    case $v in nt1) E="AGX_X=1";; nt0) E="AKKA_AMD_LIB=akka_amd/lib/var/nt0.so";; esac
    env $E timeout -k 10 200 python tools/perf.py --n $n --steps $st --reps 5 \
      > gpurun_out/r05c_perf_${v}_$n.json 2> gpurun_out/r05c_perf_${v}_$n.err || { tail -5 gpurun_out/r05c_perf_${v}_$n.err; exit 1; }
    echo "$n $v: $(python -c "import json;d=json.loads(open('gpurun_out/r05c_perf_${v}_$n.json').read().strip().splitlines()[-1]);print(round(d['us_per_step_median'],2), 'us')")"
  done
done
