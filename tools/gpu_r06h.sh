#!/bin/bash
# Round 6: multi-rank superstep baseline -- loopback groups R = 2 / 8 x 1M actors (tools/perf_group.py),
# the bench's torchrun path rehearsed with 2 RCCL processes on the one GPU, and rocprofv3 kernel stats
# of the R = 8 loopback group.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06h}
for R in 2 8; do
  timeout -k 10 200 python tools/perf_group.py --ranks $R --steps 20 > gpurun_out/${TAG}_pg$R.json 2>&1 || { tail -5 gpurun_out/${TAG}_pg$R.json; exit 1; }
  tail -1 gpurun_out/${TAG}_pg$R.json
done
timeout -k 10 300 python tools/bench_ranks_one_gpu.py --world 2 -- --steps 20 --warmup 5 --large-actors 0 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { tail -20 gpurun_out/${TAG}_bench2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench2.json').read().strip().splitlines()[-1]); print('bench world2', d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o pg --output-format csv -- python3 tools/perf_group.py --ranks 8 --steps 20 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8
