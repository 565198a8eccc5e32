#!/bin/bash
# Round 6: persistent fused supersteps + tell boundary on the GPU -- dense tests, a same-box A/B of
# the 1M ring (AGX_PERSIST=1 / 0), then the whole -m gpu suite, smoke and the driver's bench command.
# Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06d}
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_tellq.py tests/test_abi_c.py -x -v $T > gpurun_out/${TAG}_dense.log 2>&1 || { echo "dense/boundary tests failed"; tail -40 gpurun_out/${TAG}_dense.log; exit 1; }
tail -1 gpurun_out/${TAG}_dense.log
for i in 1 2; do
  for p in 1 0; do
    AGX_PERSIST=$p timeout -k 10 120 python tools/perf.py --n 1000000 --steps 200 --reps 5 > gpurun_out/${TAG}_perf_p${p}_${i}.json 2>&1 || { echo "perf failed"; tail -5 gpurun_out/${TAG}_perf_p${p}_${i}.json; exit 1; }
    echo "persist=$p $(tail -1 gpurun_out/${TAG}_perf_p${p}_${i}.json)"
  done
done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu $T > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(json.dumps(d['roofline'])); print(json.dumps(d.get('summary')))"
bash tools/gpu_r06b.sh
