#!/bin/bash
# Round 6 A/B: k_dense_fused without the RING-unused word-1 loads (the
# tree's build) against HEAD (akka_amd/lib/var/r06base4.so); 1M ring medians, three alternations,
# then rocprofv3 kernel stats of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for lib in akka_amd/lib/var/r06base4.so akka_amd/lib/libakka_gpu.so; do
    AKKA_AMD_LIB=$lib timeout -k 10 120 python tools/perf.py --n 1000000 --steps 200 --reps 5 > gpurun_out/r06y_perf.json 2>&1 || { tail -5 gpurun_out/r06y_perf.json; exit 1; }
    echo "$(basename $lib) $(tail -1 gpurun_out/r06y_perf.json)"
  done
done
for lib in akka_amd/lib/var/r06base4.so akka_amd/lib/libakka_gpu.so; do
  n=$(basename $lib .so)
  AKKA_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06y_prof_$n -o p --output-format csv -- python3 tools/perf.py --n 1000000 --steps 200 --reps 3 > gpurun_out/r06y_prof_$n.log 2>&1 || { tail -5 gpurun_out/r06y_prof_$n.log; exit 1; }
  f=$(find gpurun_out/r06y_prof_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv,sys; [print(sys.argv[2], '%-50s %6s avg %7.2f us' % (x['Name'][:50], x['Calls'], float(x['AverageNs'])/1e3)) for x in list(csv.DictReader(open(sys.argv[1])))[:3]]" "$f" $n
done
