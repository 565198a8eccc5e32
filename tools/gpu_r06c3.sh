#!/bin/bash
# Round 6: where a nearly idle C3 superstep (spec shape, 10M actors) spends its time -- eager per-class
# profile, then rocprofv3 kernel stats of the same run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag_c5.py --workload c3s --steps 4 > gpurun_out/r06c3_diag.log 2>&1 || { tail -20 gpurun_out/r06c3_diag.log; exit 1; }
grep "^step" gpurun_out/r06c3_diag.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06c3_prof -o run --output-format csv -- python3 tools/diag_c5.py --workload c3s --steps 4 > gpurun_out/r06c3_prof.log 2>&1 || { tail -20 gpurun_out/r06c3_prof.log; exit 1; }
f=$(find gpurun_out/r06c3_prof -name "*kernel_stats.csv" | head -1)
python3 -c "import csv,sys; [print('%-70s %6s avg %9.1f us tot %9.1f' % (x['Name'][:70], x['Calls'], float(x['AverageNs'])/1e3, float(x['TotalDurationNs'])/1e3)) for x in list(csv.DictReader(open(sys.argv[1])))[:25]]" "$f"
