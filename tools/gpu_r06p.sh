#!/bin/bash
# Round 6 A/B: ORSet full-state wave merge with the run's first messages' rows loaded before any is
# applied (the tree: 3 messages; var/r06pre2.so: 2) vs the per-message loads (var/r06base5.so):
# ORSet parity first, then C4 ORSet gossip timed as bench.py does, alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_benched.py -q -k "orset or crdt" $T > gpurun_out/r06p_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06p_tests.log; exit 1; }
tail -1 gpurun_out/r06p_tests.log
for i in 1 2; do
for lib in akka_amd/lib/var/r06base5.so akka_amd/lib/var/r06pre2.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 300 python tools/cfg_one.py C4_orset_gossip > gpurun_out/r06p_$n.json 2> gpurun_out/r06p_$n.err || { tail -20 gpurun_out/r06p_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step')) for k, v in d.items()]" gpurun_out/r06p_$n.json $n
done
done
echo done
