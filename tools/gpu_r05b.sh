#!/bin/bash
# round-5: fused dense launch -- parity, then the 1M / 100M ring A/B (AGX_DENSE_FUSED=0 vs 1)
set -o pipefail
mkdir -p gpurun_out
T="--timeout 110 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -q -x \
  -k "${PK:-dense or ring or strict or partial or ping or zipf or conservation}" $T > gpurun_out/r05b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r05b_pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in old dense nt; do
    case $v in old) E="AGX_DENSE_FUSED=0";; dense) E="AGX_DENSE_FUSED=1";; nt) E="AKKA_AMD_LIB=akka_amd/lib/var/nt.so";; esac
    env $E timeout -k 10 120 python tools/perf.py --n 1000000 --steps 60 --reps 5 \
      > gpurun_out/r05b_perf_$v.json 2> gpurun_out/r05b_perf_$v.err || { tail -5 gpurun_out/r05b_perf_$v.err; exit 1; }
    echo "$v: $(python -c "import json;d=json.loads(open('gpurun_out/r05b_perf_$v.json').read().strip().splitlines()[-1]);print(round(d['us_per_step_median'],2), 'us')")"
  done
done
