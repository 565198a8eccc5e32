#!/bin/bash
# Round 6 A/B: PingPong drains message-parallel (the tree) vs the serial per-actor drain
# (var/r06noping.so, -DAGX_PING_PAR=0): ping-pong parity first, then C1 timed as bench.py does.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_benched.py -q -k "ping or outbox or host or reply or mixed" $T > gpurun_out/r06pp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06pp_tests.log; exit 1; }
tail -1 gpurun_out/r06pp_tests.log
for i in 1 2; do
for lib in akka_amd/lib/var/r06noping.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 300 python tools/cfg_one.py C1_ping_pong > gpurun_out/r06pp_$n.json 2> gpurun_out/r06pp_$n.err || { tail -20 gpurun_out/r06pp_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, '%.4g' % v['value'], round(v['ms_per_step'], 4), v.get('kernel_ms_per_step')) for k, v in d.items()]" gpurun_out/r06pp_$n.json $n
done
done
AGX_STAMPS=1 timeout -k 10 120 python tools/diag_c5.py --workload c1 --steps 2 > gpurun_out/r06pp_c1.log 2>&1 || { tail -20 gpurun_out/r06pp_c1.log; exit 1; }
grep -a "mean cycles" gpurun_out/r06pp_c1.log
echo done
