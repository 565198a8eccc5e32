#!/bin/bash
# A/B of alternative builds on one BASELINE config: tools/ab_cfg.sh CONFIG lib1.so lib2.so[:ENV=VAL] ...
set -o pipefail
mkdir -p gpurun_out
CFG=$1; shift
for rep in $(seq ${AB_REPS:-1}); do
  for item in "$@"; do
    lib=${item%%:*}; envs=""; [ "$item" != "$lib" ] && envs=${item#*:}
    env $envs AKKA_AMD_LIB=$lib timeout -k 10 300 python tools/cfg_one.py $CFG > gpurun_out/abc_tmp.json 2>gpurun_out/abc.err || { tail -20 gpurun_out/abc.err; exit 1; }
    python3 -c "import json; d=list(json.load(open('gpurun_out/abc_tmp.json')).values())[0]; print('$item $CFG', '%.4g' % d.get('value', 0), round(d.get('ms_per_step', 0), 3), {k: v for k, v in d.get('kernel_ms_per_step', {}).items() if v > 0.02}, d.get('error', ''))"
  done
done
