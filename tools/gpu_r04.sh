#!/bin/bash
# Round-4 GPU check: the full-size parity tests, the rest of the -m gpu suite, the driver's bench
# command.  Each GPU step has its own time limit; the first failure ends the script.
#   STEPS="full gpu ab bench" (default: full gpu bench); ab: CFGS (bench configs) for every library in
#   LIBS (default: akka_amd/lib/var/base.so and the tree's build), AB_REPS times; prof: rocprofv3
#   kernel trace + stats of PROF_CFGS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
STEPS=${STEPS:-"full gpu bench"}
for s in $STEPS; do
  case $s in
    full)
      timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py -x -v -k "${FULL_K:-.}" --timeout 900 --timeout-method thread \
        > gpurun_out/${TAG}_full.log 2>&1 || { echo "fullsize failed"; tail -60 gpurun_out/${TAG}_full.log; exit 1; }
      tail -3 gpurun_out/${TAG}_full.log ;;
    gpu)
      timeout -k 10 900 python -u -m pytest tests -x -q -m "gpu and not fullsize" --timeout 280 --timeout-method thread \
        > gpurun_out/${TAG}_gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/${TAG}_gpu.log; exit 1; }
      tail -3 gpurun_out/${TAG}_gpu.log ;;
    sub)  # a subset of the GPU suite: SUB_FILES (default tests), SUB_K (pytest -k expression)
      timeout -k 10 900 python -u -m pytest ${SUB_FILES:-tests} -x -q -m "gpu and not fullsize" -k "${SUB_K:-.}" \
        --timeout 280 --timeout-method thread > gpurun_out/${TAG}_sub.log 2>&1 || { echo "gpu subset failed"; tail -60 gpurun_out/${TAG}_sub.log; exit 1; }
      tail -3 gpurun_out/${TAG}_sub.log ;;
    ab)
      for c in ${CFGS:-C3_zipf_fanout C3_zipf_tree C5_power_law_bounded}; do
        AB_REPS=${AB_REPS:-2} bash tools/ab_cfg.sh $c ${LIBS:-akka_amd/lib/var/base.so akka_amd/lib/libakka_gpu.so} \
          >> gpurun_out/${TAG}_ab.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/${TAG}_ab.log; exit 1; }
      done
      cat gpurun_out/${TAG}_ab.log ;;
    abring)  # the ring at 1M / 100M actors (tools/ab.sh, PERF_NS) for every library in LIBS
      PERF_NS="${PERF_NS:-1000000 100000000}" AB_REPS=${AB_REPS:-2} bash tools/ab.sh ${TAG}ring \
        ${LIBS:-akka_amd/lib/var/base.so akka_amd/lib/libakka_gpu.so} > /dev/null 2>&1 \
        || { echo "abring failed"; tail -30 gpurun_out/${TAG}ring_ab.err; exit 1; }
      cat gpurun_out/${TAG}ring_ab.txt ;;
    stamps)  # per-phase cycle stamps of the block apply (AGX_STAMPS, eager) on STAMP_WL (tools/diag_c5.py)
      for wlname in ${STAMP_WL:-c5 c3}; do
        AGX_STAMPS=1 timeout -k 10 300 python tools/diag_c5.py --workload $wlname --steps 3 \
          > gpurun_out/${TAG}_stamps_$wlname.log 2>&1 || { echo "stamps $wlname failed"; tail -20 gpurun_out/${TAG}_stamps_$wlname.log; exit 1; }
        grep -a "agx stamps\|^step" gpurun_out/${TAG}_stamps_$wlname.log | tail -8
      done ;;
    pmc)  # FETCH_SIZE / WRITE_SIZE passes (separate runs) of PMC_CFGS "name:warmup", per-superstep window sums
      for cw in ${PMC_CFGS:-C5_power_law_bounded:2 C3_zipf_fanout:2}; do
        c=${cw%%:*}; wu=${cw##*:}
        for grp in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_pmc_${c}_$grp -o run \
            -- python3 tools/cfg_one.py $c > gpurun_out/${TAG}_pmc_${c}_$grp.log 2>&1 || { echo "pmc $c $grp failed"; tail -20 gpurun_out/${TAG}_pmc_${c}_$grp.log; exit 1; }
        done
        python3 tools/pmc_window.py $c gpurun_out/${TAG}_pmc_${c}_FETCH_SIZE gpurun_out/${TAG}_pmc_${c}_WRITE_SIZE \
          gpurun_out/${TAG}_pmc_${c}_FETCH_SIZE.log --warmup $wu | tee gpurun_out/${TAG}_pmc_${c}.json
      done ;;
    prof)  # rocprofv3 kernel trace + stats of single bench configs (PROF_CFGS), the tree's build
      for c in ${PROF_CFGS:-C5_power_law_bounded C3_zipf_fanout C3_zipf_tree}; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$c -o run \
          -- python3 tools/cfg_one.py $c > gpurun_out/${TAG}_prof_$c.log 2>&1 || { echo "prof $c failed"; tail -30 gpurun_out/${TAG}_prof_$c.log; exit 1; }
        echo "prof $c ok"
      done ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { echo "smoke failed"; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    benchprof)  # rocprofv3 kernel trace + stats of the driver's bench command itself
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_benchprof -o run \
        -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_benchprof.json 2> gpurun_out/${TAG}_benchprof.err \
        || { echo "benchprof failed"; tail -30 gpurun_out/${TAG}_benchprof.err; exit 1; }
      echo "benchprof ok" ;;
    pmcring)  # counter passes of the ring operating points (1M fused + 100M multi-pass), one run each
      i=0
      for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_ring_p$i -o run \
          -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-configs --large-steps 8 > gpurun_out/${TAG}_ring_p$i.log 2>&1 \
          || { echo "ring pmc pass $i failed"; tail -20 gpurun_out/${TAG}_ring_p$i.log; exit 1; }
        echo "ring pmc pass $i ok"
      done ;;
    bench)
      timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json \
        2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -40 gpurun_out/${TAG}_bench.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary']))" ;;
  esac
done
exit 0
