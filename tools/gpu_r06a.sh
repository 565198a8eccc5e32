#!/bin/bash
# Round 6: the boundary changes first (tell path, ABI harnesses, RCCL ranks), then the whole -m gpu
# suite, smoke and the driver's bench command.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tellq.py tests/test_abi_c.py tests/test_rccl_ranks.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_boundary.log 2>&1 || { echo "boundary tests failed"; tail -40 gpurun_out/${TAG}_boundary.log; exit 1; }
tail -1 gpurun_out/${TAG}_boundary.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print(json.dumps(d['roofline']))"
