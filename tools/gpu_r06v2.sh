#!/bin/bash
# Round 6: 17/16 initial exchange slabs -- RCCL rank suite, then the bench's torchrun path rehearsed with
# 2 and 4 RCCL processes on the one GPU (AGX_MR_DEBUG off; exchange_info printed by the bench line).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_rccl_ranks.py -q $T > gpurun_out/r06v2_rccl.log 2>&1 || { echo "rccl failed"; tail -40 gpurun_out/r06v2_rccl.log; exit 1; }
tail -1 gpurun_out/r06v2_rccl.log
for w in 2 4; do
  timeout -k 10 400 python tools/bench_ranks_one_gpu.py --world $w -- --steps 20 --warmup 5 --large-actors 0 > gpurun_out/r06v2_bench$w.json 2> gpurun_out/r06v2_bench$w.err || { tail -20 gpurun_out/r06v2_bench$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r06v2_bench$w.json').read().strip().splitlines()[-1]); print('world $w', d['value'], d['ms_per_step'], d['n_gpus'])"
done
