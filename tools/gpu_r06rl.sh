#!/bin/bash
# Round 6 A/B: queued DeltaPropagation rows copied a lane each (the tree) vs by the wave one after the other
# (var/r06nolane.so, -DAGX_DELTA_ROW_LANE=0; measured and reverted): delta parity
# first (throughput caps queue DeltaPropagations), then the C4 delta configs timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_fullsize.py tests/test_gpu_benched.py tests/test_rccl_ranks.py tests/test_gpu_parity.py -q -k "delta or crdt or orset" $T > gpurun_out/r06rl_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06rl_tests.log; exit 1; }
tail -1 gpurun_out/r06rl_tests.log
for c in C4_orset_delta_gossip C4_gcounter_delta_gossip; do
for i in 1 2; do
for lib in akka_amd/lib/var/r06nolane.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 300 python tools/cfg_one.py $c > gpurun_out/r06rl_$n.json 2> gpurun_out/r06rl_$n.err || { tail -20 gpurun_out/r06rl_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4)) for k, v in d.items()]" gpurun_out/r06rl_$n.json $n
done
done
done
echo done
