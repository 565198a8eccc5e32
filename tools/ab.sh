#!/bin/bash
# A/B of alternative builds on one box: tools/ab.sh TAG lib1.so lib2.so:ENV=VAL[,..] ...  (PERF_NS, PERF_STEPS, AB_REPS)
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
for rep in $(seq ${AB_REPS:-2}); do
  for item in "$@"; do
    lib=${item%%:*}; envs=""; [ "$item" != "$lib" ] && envs=${item#*:}
    for n in ${PERF_NS:-1000000 100000000}; do
      env $envs AKKA_AMD_LIB=$lib timeout -k 10 200 python tools/perf.py --n $n --steps ${PERF_STEPS:-40} --reps 5 --prof ${PERF_ARGS} > gpurun_out/${TAG}_tmp.json 2>gpurun_out/${TAG}_ab.err || { tail -20 gpurun_out/${TAG}_ab.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print('$item', d['n'], round(d['us_per_step_median'],1), {k:v for k,v in d.get('kernel_us_per_step',{}).items() if v>1})" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
