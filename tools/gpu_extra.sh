#!/bin/bash
# Round extras: ring superstep scaling (tools/gpu_scale.sh) and the multi-rank loopback cost
# (tools/perf_group.py: R engines in ONE process on the one GPU, R=2,4; rocprofv3 kernel stats of R=2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
bash tools/gpu_scale.sh $TAG > /dev/null || exit 1
rm -f gpurun_out/${TAG}_group.jsonl
for r in 2 4; do
  timeout -k 10 200 python tools/perf_group.py --ranks $r --n 1000000 >> gpurun_out/${TAG}_group.jsonl 2>gpurun_out/${TAG}_group.err || { tail -20 gpurun_out/${TAG}_group.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_gprof -o run -- python3 tools/perf_group.py --ranks 2 --steps 20 > gpurun_out/${TAG}_gprof.log 2>&1 || { tail -20 gpurun_out/${TAG}_gprof.log; exit 1; }
cat gpurun_out/${TAG}_scale.jsonl gpurun_out/${TAG}_group.jsonl
