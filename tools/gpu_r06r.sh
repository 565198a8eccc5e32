#!/bin/bash
# Round 6: peer runs written straight into the send slabs (device-resident multi-rank replays) and the
# branch-free RING apply in owner mode -- RCCL rank suite (incl. 64-envelope slabs: overflow -> repair ->
# exact exchange), loopback sharded tests, then rocprofv3 of a 2-rank RCCL ring (direct vs AGX_MR_NO_DIRECT).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_rccl_ranks.py tests/test_gpu_dense.py tests/test_gpu_parity.py -q -k "rccl or sharded or loopback" $T > gpurun_out/r06r_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06r_tests.log; exit 1; }
tail -1 gpurun_out/r06r_tests.log
for d in 0 1; do
  if [ $d = 1 ]; then export AGX_MR_NO_DIRECT=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06r_prof$d -o p --output-format csv -- python3 tools/rccl_two_rank.py --split-hosts --world 2 --n 1000000 --hops 40 --workload ring > gpurun_out/r06r_prof$d.log 2>&1 || { tail -20 gpurun_out/r06r_prof$d.log; exit 1; }
  f=$(find gpurun_out/r06r_prof$d -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv,sys; [print(sys.argv[2], '%-50s %6s avg %8.2f us' % (x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e3)) for x in list(csv.DictReader(open(sys.argv[1])))[:12]]" "$f" nodirect=$d
done
