#!/bin/bash
# Round 6: C5 at 100M, environment A/Bs on one box: the first (chunk-list) pass's digit width
# (AGX_PASS0_BITS; default: 16 bucket bits spread 8 + 8), the wave-path threshold (AGX_TINY), and the
# skew launch grid (AGX_SKEW_GRID).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in X=0 AGX_PASS0_BITS=5 AGX_PASS0_BITS=7 AGX_TINY=64 AGX_SKEW_GRID=2048 X=1; do
  env $e timeout -k 10 300 python tools/cfg_one.py C5_power_law_bounded > gpurun_out/r06m_$e.json 2> gpurun_out/r06m_$e.err || { tail -5 gpurun_out/r06m_$e.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['C5_power_law_bounded']; print(sys.argv[2], '%.3g'%d['value'], round(d['ms_per_step'],3), d.get('kernel_ms_per_step'))" gpurun_out/r06m_$e.json $e
done
