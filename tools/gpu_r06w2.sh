#!/bin/bash
# Round 6: ORSet-delta bucket width 1024 (the workload default) vs 2048 (AGX_BUCKET_ACTORS), timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for ba in 1024 2048; do
  AGX_BUCKET_ACTORS=$ba timeout -k 10 300 python tools/cfg_one.py C4_orset_delta_gossip > gpurun_out/r06w2_$ba.json 2> gpurun_out/r06w2_$ba.err || { tail -20 gpurun_out/r06w2_$ba.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step', {}).get('bucket_apply'), v.get('kernel_ms_per_step', {}).get('bucket_apply_skew')) for k, v in d.items()]" gpurun_out/r06w2_$ba.json $ba
done
done
echo done
