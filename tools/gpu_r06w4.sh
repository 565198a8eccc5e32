#!/bin/bash
# Round 6: C3 bucket width, the default (2048) vs 1024 vs 512 (AGX_BUCKET_ACTORS), timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C3_zipf_fanout C3_zipf_tree C3_zipf_steady_spec; do
for ba in 0 1024 512; do
  if [ $ba = 0 ]; then unset AGX_BUCKET_ACTORS; else export AGX_BUCKET_ACTORS=$ba; fi
  timeout -k 10 300 python tools/cfg_one.py $c > gpurun_out/r06w4_$ba.json 2> gpurun_out/r06w4_$ba.err || { tail -20 gpurun_out/r06w4_$ba.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4)) for k, v in d.items()]" gpurun_out/r06w4_$ba.json $ba
done
done
unset AGX_BUCKET_ACTORS
echo done
