#!/bin/bash
# Round 2, first box: RCCL two-rank parity on one device (split host ids) + short headline bench.
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop the script after a timeout / abort / crash
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r02a/$name.out" 2> "gpurun_out/r02a/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after $name"; exit $rc;; esac
}
step rccl_ring 300 python -u tools/rccl_two_rank.py --split-hosts --n 20000 --hops 8
step rccl_mixed 300 python -u tools/rccl_two_rank.py --split-hosts --n 20000 --workload mixed
step bench20 240 python -u bench.py --steps 20 --warmup 5 --no-configs --large-actors 0 --no-cpu-baseline
step bench200 240 python -u bench.py --steps 200 --warmup 16 --no-configs --large-actors 0 --no-cpu-baseline
