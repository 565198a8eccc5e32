#!/bin/bash
# Ring superstep time vs population (per-kernel breakdown) -> gpurun_out/${TAG}_scale.jsonl
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-scale}
rm -f gpurun_out/${TAG}_scale.jsonl
for n in 1000000 4000000 10000000 12500000 100000000; do
  timeout -k 10 200 python tools/perf.py --n $n --steps 40 --reps 5 --prof >> gpurun_out/${TAG}_scale.jsonl 2>gpurun_out/${TAG}_scale.err || { tail -5 gpurun_out/${TAG}_scale.err; exit 1; }
done
timeout -k 10 200 python tools/perf.py --n 1000000 --steps 12 --reps 3 --prof --workload powerlaw >> gpurun_out/${TAG}_scale.jsonl 2>>gpurun_out/${TAG}_scale.err || exit 1
cat gpurun_out/${TAG}_scale.jsonl
