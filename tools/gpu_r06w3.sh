#!/bin/bash
# Round 6: C4 full-state gossip bucket width, the workload default vs 1024 vs 2048 (AGX_BUCKET_ACTORS).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C4_orset_gossip C4_gcounter_gossip C4_gcounter_delta_gossip; do
for i in 1 2; do
for ba in 0 1024 2048; do
  if [ $ba = 0 ]; then unset AGX_BUCKET_ACTORS; else export AGX_BUCKET_ACTORS=$ba; fi
  timeout -k 10 300 python tools/cfg_one.py $c > gpurun_out/r06w3_$ba.json 2> gpurun_out/r06w3_$ba.err || { tail -20 gpurun_out/r06w3_$ba.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4)) for k, v in d.items()]" gpurun_out/r06w3_$ba.json $ba
done
done
done
unset AGX_BUCKET_ACTORS
echo done
