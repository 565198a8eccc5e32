#!/bin/bash
# Round 6 A/B: k_mcompact_copy copies a bucket's R owner runs as one flattened block pass (the tree)
# vs R sequential block copies (HEAD, var/r06base5.so).  Multi-rank parity first (loopback, sharded,
# RCCL ranks on one GPU), then R = 8 x 1M loopback kernel stats under one hardware queue per variant,
# the world-2 bench line (its exchange object), and the delta-CRDT stamps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_rccl_ranks.py -q -k "sharded or loopback or rccl" $T > gpurun_out/r06z_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06z_tests.log; exit 1; }
tail -1 gpurun_out/r06z_tests.log
for lib in akka_amd/lib/var/r06base5.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  GPU_MAX_HW_QUEUES=1 AKKA_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06z_$n -o pg --output-format csv -- python3 tools/perf_group.py --ranks 8 --steps 20 > gpurun_out/r06z_$n.log 2>&1 || { tail -30 gpurun_out/r06z_$n.log; exit 1; }
  f=$(find gpurun_out/r06z_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv,sys; [print(sys.argv[2], '%-55s %5s min %7.1f avg %7.1f' % (x['Name'][:55], x['Calls'], float(x['MinNs'])/1e3, float(x['AverageNs'])/1e3)) for x in csv.DictReader(open(sys.argv[1])) if 'mcompact' in x['Name'] or 'mr_' in x['Name']]" "$f" $n
  tail -2 gpurun_out/r06z_$n.log
done
for lib in akka_amd/lib/var/r06base5.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 400 python tools/bench_ranks_one_gpu.py --world 2 -- --steps 20 --warmup 5 --large-actors 0 > gpurun_out/r06z_xb_$n.json 2> gpurun_out/r06z_xb_$n.err || { tail -30 gpurun_out/r06z_xb_$n.err; exit 1; }
  echo "$n"; tail -c 1500 gpurun_out/r06z_xb_$n.json
done
for w in c4gd c4od; do
  AGX_STAMPS=1 timeout -k 10 120 python tools/diag_c5.py --workload $w --steps 3 > gpurun_out/r06z_$w.log 2>&1 || { tail -20 gpurun_out/r06z_$w.log; exit 1; }
done
echo done
