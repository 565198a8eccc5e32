#!/bin/bash
# Ring (C2 1M / 100M) at bucket widths 2048 / 1024 / 512 (AGX_BUCKET_ACTORS), same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=akka_amd/lib/libakka_gpu.so
AB_REPS=2 bash tools/ab.sh r03u $L $L:AGX_BUCKET_ACTORS=1024 $L:AGX_BUCKET_ACTORS=512
