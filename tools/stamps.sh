#!/bin/bash
# Per-phase cycle stamps of k_bucket_apply (AGX_STAMPS diagnostic; graphs off).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-st}
for n in ${STAMP_NS:-1000000 100000000}; do
  AGX_STAMPS=1 timeout -k 10 200 python tools/perf.py --n $n --steps 4 --reps 1 > gpurun_out/${TAG}_stamps_$n.log 2>&1 || exit 1
  tail -n 2 gpurun_out/${TAG}_stamps_$n.log
done
