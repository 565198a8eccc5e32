#!/bin/bash
# round-5: owner-mode dense launch -- parity (dense, sharded, RCCL ring), then loopback R x 1M A/B
set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_benched.py -q -x \
  -k "${PK:-dense or sharded or loopback}" $T > gpurun_out/r05d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05d_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_rccl_ranks.py -q -x -k "ring" $T > gpurun_out/r05d_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -2 gpurun_out/r05d_rccl.log; [ $rc -eq 0 ] || exit 1
for r in 2 8; do
  for v in 1 0; do
    AGX_DENSE_OWNER=$v timeout -k 10 200 python tools/perf_group.py --ranks $r --n 1000000 --steps 20 \
      > gpurun_out/r05d_group_${r}_$v.json 2> gpurun_out/r05d_group_${r}_$v.err || { tail -5 gpurun_out/r05d_group_${r}_$v.err; exit 1; }
    echo "R=$r DENSE_OWNER=$v: $(tail -1 gpurun_out/r05d_group_${r}_$v.json | cut -c1-400)"
  done
done
