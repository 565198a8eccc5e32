#!/bin/bash
# Round 6 A/B: multi-rank RING route entries loaded during the inbox round trip (the tree) vs HEAD
# (var/r06base2.so) -- R = 8 x 1M loopback, one hardware queue, rocprofv3 kernel stats; sharded tests first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py -q -k "sharded or loopback" $T > gpurun_out/r06s_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06s_tests.log; exit 1; }
tail -1 gpurun_out/r06s_tests.log
for lib in akka_amd/lib/var/r06base2.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  GPU_MAX_HW_QUEUES=1 AKKA_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06s_$n -o pg --output-format csv -- python3 tools/perf_group.py --ranks 8 --steps 20 > gpurun_out/r06s_$n.log 2>&1 || { tail -30 gpurun_out/r06s_$n.log; exit 1; }
  f=$(find gpurun_out/r06s_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv,sys; [print(sys.argv[2], '%-55s %5s min %7.1f avg %7.1f' % (x['Name'][:55], x['Calls'], float(x['MinNs'])/1e3, float(x['AverageNs'])/1e3)) for x in list(csv.DictReader(open(sys.argv[1])))[:4]]" "$f" $n
done
