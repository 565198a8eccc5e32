#!/bin/bash
# Round 6: delta-CRDT bucket width after the phase-B class schedule -- 512 (default) vs 1024 vs 256
# (AGX_BUCKET_ACTORS), C4 ORSet-delta and GCounter-delta timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C4_orset_delta_gossip C4_gcounter_delta_gossip; do
for i in 1 2; do
for ba in 512 1024 256; do
  AGX_BUCKET_ACTORS=$ba timeout -k 10 300 python tools/cfg_one.py $c > gpurun_out/r06w_$ba.json 2> gpurun_out/r06w_$ba.err || { tail -20 gpurun_out/r06w_$ba.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step', {}).get('bucket_apply'), v.get('kernel_ms_per_step', {}).get('bucket_apply_skew')) for k, v in d.items()]" gpurun_out/r06w_$ba.json $ba
done
done
done
echo done
