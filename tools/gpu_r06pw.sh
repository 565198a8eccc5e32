#!/bin/bash
# Round 6: C1 bucket width after the message-parallel PingPong drain (AGX_BUCKET_ACTORS 32 = the
# workload's choice, 16, 8, 64), timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for ba in 32 16 8 64; do
  AGX_BUCKET_ACTORS=$ba timeout -k 10 300 python tools/cfg_one.py C1_ping_pong > gpurun_out/r06pw_$ba.json 2> gpurun_out/r06pw_$ba.err || { tail -20 gpurun_out/r06pw_$ba.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step')) for k, v in d.items()]" gpurun_out/r06pw_$ba.json $ba
done
done
echo done
