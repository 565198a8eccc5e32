#!/bin/bash
# GPU tests, the driver-shaped bench, per-kernel times of the 100M ring and C3 (HIP events).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03d}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary'])); print(json.dumps(d['at_100M_actors']['roofline']))"
timeout -k 10 300 python tools/perf.py --n 100000000 --steps 20 --reps 3 --prof > gpurun_out/${TAG}_perf100m.json 2>&1 || { tail -20 gpurun_out/${TAG}_perf100m.json; exit 1; }
cat gpurun_out/${TAG}_perf100m.json
