#!/bin/bash
# GPU tests, 100M ring kernel times, 1M apply phase stamps, C4 ORSet kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03e}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python tools/perf.py --n 100000000 --steps 20 --reps 3 --prof > gpurun_out/${TAG}_perf100m.json 2>&1 || { tail -20 gpurun_out/${TAG}_perf100m.json; exit 1; }
tail -1 gpurun_out/${TAG}_perf100m.json
AGX_STAMPS=1 AGX_NO_GRAPH=1 timeout -k 10 200 python tools/perf.py --n 1000000 --steps 4 --reps 1 > gpurun_out/${TAG}_stamps1m.log 2>&1 || { tail -20 gpurun_out/${TAG}_stamps1m.log; exit 1; }
grep "agx stamps" gpurun_out/${TAG}_stamps1m.log | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c4prof -o run -- python3 tools/cfg_one.py C4_orset_gossip > gpurun_out/${TAG}_c4prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4prof.log; exit 1; }
cut -d, -f1-4 gpurun_out/${TAG}_c4prof/run_kernel_stats.csv | head -12
