#!/bin/bash
# GPU tests, then same-box A/B of the ring (1M fused, 100M identity multi-pass): this build vs
# variant builds under akka_amd/lib/var/ (tools/build_variant.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03c}
L=akka_amd/lib/libakka_gpu.so
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
AB_REPS=${AB_REPS:-2} bash tools/ab.sh ${TAG} $L ${VARIANTS} > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
