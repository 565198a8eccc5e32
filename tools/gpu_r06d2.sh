#!/bin/bash
# Round 6: counters keep each slot's last delta (no 64-entry log) -- delta parity (incl. 150 unsent
# seqNrs), the full-size delta runs as benched, the sharded benched delta cases, then the two C4 delta
# configs timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_fullsize.py tests/test_gpu_benched.py -q -k "delta" $T > gpurun_out/r06d2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06d2_tests.log; exit 1; }
tail -1 gpurun_out/r06d2_tests.log
for c in C4_gcounter_delta_gossip C4_orset_delta_gossip; do
  timeout -k 10 300 python tools/cfg_one.py $c > gpurun_out/r06d2_$c.json 2> gpurun_out/r06d2_$c.err || { tail -20 gpurun_out/r06d2_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step')) for k, v in d.items()]" gpurun_out/r06d2_$c.json
done
echo done
