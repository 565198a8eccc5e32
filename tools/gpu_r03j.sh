#!/bin/bash
# Delta-CRDT bucket width A/B (AGX_BUCKET_ACTORS) on the C4 delta configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03j}
L=akka_amd/lib/libakka_gpu.so
for c in C4_orset_delta_gossip C4_gcounter_delta_gossip; do
  AB_REPS=1 bash tools/ab_cfg.sh $c $L $L:AGX_BUCKET_ACTORS=256 $L:AGX_BUCKET_ACTORS=1024 $L >> gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
done
cat gpurun_out/${TAG}_ab.log
