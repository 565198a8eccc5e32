#!/bin/bash
# Round 6 A/B: ORSet delta merge / group rows with batched loads (the tree) vs HEAD~ (var/r06base5.so,
# same ORSet layout): delta parity first, then C4 ORSet-delta timed as bench.py does, alternating.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta_crdt.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -k "delta or crdt or orset" $T > gpurun_out/r06o_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06o_tests.log; exit 1; }
tail -1 gpurun_out/r06o_tests.log
for i in 1 2; do
for lib in akka_amd/lib/var/r06base5.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 300 python tools/cfg_one.py C4_orset_delta_gossip > gpurun_out/r06o_$n.json 2> gpurun_out/r06o_$n.err || { tail -20 gpurun_out/r06o_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step')) for k, v in d.items()]" gpurun_out/r06o_$n.json $n
done
done
AGX_STAMPS=1 timeout -k 10 120 python tools/diag_c5.py --workload c4od --steps 3 > gpurun_out/r06o_c4od.log 2>&1 || { tail -20 gpurun_out/r06o_c4od.log; exit 1; }
grep "mean cycles" gpurun_out/r06o_c4od.log
echo done
