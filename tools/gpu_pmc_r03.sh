#!/bin/bash
# Round-3 counter passes (each its own rocprofv3 run, no trace domains):
#   ring (1M fused + 100M multi-pass): FETCH_SIZE, WRITE_SIZE, SQ wait/issue counters
#   C4 ORSet full state and C5: FETCH_SIZE, WRITE_SIZE (tools/cfg_one.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc3}
ARGS="--steps 20 --warmup 4 --no-cpu-baseline --no-configs --large-steps 8"
i=0
for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_ring_p$i -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_ring_p$i.log 2>&1 || { echo "ring pmc pass $i ($grp) failed"; tail -20 gpurun_out/${TAG}_ring_p$i.log; exit 1; }
  echo "ring pass $i ok: $grp"
done
for cfg in ${CFGS:-C4_orset_gossip C5_power_law_bounded}; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${cfg}_p$i -o run -- python3 tools/cfg_one.py $cfg > gpurun_out/${TAG}_${cfg}_p$i.log 2>&1 || { echo "pmc $cfg $grp failed"; tail -20 gpurun_out/${TAG}_${cfg}_p$i.log; exit 1; }
    echo "pmc $cfg $grp ok"
  done
done
echo done
