#!/bin/bash
# Final-tree evidence (round 5, last kernel change): GPU tests, smoke, the driver's bench command, rocprofv3
# headline bench, FETCH / WRITE / SQ counter passes (ring) and FETCH / WRITE (C4 ORSet, C5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fin}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary'])); print(json.dumps(d['roofline']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
echo "rocprof ok"
