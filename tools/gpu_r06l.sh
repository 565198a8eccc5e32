#!/bin/bash
# Round 6: C5 at 100M -- block-apply phase stamps, then the first-pass unit width A/B (AGX_UNIT_G:
# buckets per chunk-pass histogram column; hot R-MAT senders cluster at low ids, so a 24-bucket unit
# can hold ~240 K tells for one downsweep block).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AGX_STAMPS=1 timeout -k 10 300 python tools/diag_c5.py --steps 6 > gpurun_out/r06l_stamps.log 2>&1 || { tail -5 gpurun_out/r06l_stamps.log; exit 1; }
grep -a "stamps\|^step" gpurun_out/r06l_stamps.log | cut -c1-300 | tail -8
for g in 24 8 2 1; do
  AGX_UNIT_G=$g timeout -k 10 300 python tools/cfg_one.py C5_power_law_bounded > gpurun_out/r06l_g$g.json 2> gpurun_out/r06l_g$g.err || { tail -5 gpurun_out/r06l_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['C5_power_law_bounded']; print('G', sys.argv[2], '%.3g'%d['value'], round(d['ms_per_step'],3), d.get('kernel_ms_per_step'))" gpurun_out/r06l_g$g.json $g
done
