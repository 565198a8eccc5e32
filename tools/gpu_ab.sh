#!/bin/bash
# Same-box A/B of alternative builds (tools/build_variant.sh) or environment switches, after a GPU
# test subset:  tools/gpu_ab.sh TAG lib_a.so lib_b.so[:ENV=VAL] ...
#   TESTS  pytest -k filter ("" = the whole -m gpu suite, "none" = no tests)
#   PERF_NS  ring sizes for tools/ab.sh ("none" = skip; default "1000000 100000000")
#   CFGS   BASELINE configs for tools/ab_cfg.sh (default none), AB_REPS repetitions (default 2)
#   STAMPS=1  also per-phase cycle stamps of the first build (tools/stamps.sh, graphs off)
# Logs: gpurun_out/TAG_pytest.log, TAG_ab.txt (ring), TAG_abc.log (configs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
if [ "${TESTS-}" != "none" ]; then
  K=(); [ -n "${TESTS-}" ] && K=(-k "$TESTS")
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu "${K[@]}" --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
if [ "${PERF_NS-}" != "none" ]; then
  PERF_NS="${PERF_NS:-1000000 100000000}" AB_REPS=${AB_REPS:-2} bash tools/ab.sh ${TAG} "$@" || exit 1
fi
for c in ${CFGS-}; do
  AB_REPS=${AB_REPS:-2} bash tools/ab_cfg.sh $c "$@" >> gpurun_out/${TAG}_abc.log 2>&1 || { cat gpurun_out/${TAG}_abc.log; exit 1; }
done
[ -n "${CFGS-}" ] && cat gpurun_out/${TAG}_abc.log
if [ "${STAMPS-}" = "1" ]; then
  AKKA_AMD_LIB=${1%%:*} bash tools/stamps.sh ${TAG} || exit 1
fi
exit 0
