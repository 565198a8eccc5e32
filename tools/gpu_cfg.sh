#!/bin/bash
# parity tests, then the other-config measurements only (quick headline)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-cfg}
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --large-actors 0 --steps 50 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().split('\n')[-1])
print('C2', d['value'], d['ms_per_step'])
for k,v in d.get('configs',{}).items(): print(k, v.get('value'), v.get('ms_per_step'), v.get('kernel_ms_per_step'), v.get('error'))"
