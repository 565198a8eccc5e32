#!/bin/bash
# Round 6 A/B: (1) the wide CRDT kernels at 256 VGPRs (no spills, one block per CU: r06w2 =
# -DAGX_WIDE_WPE=2) vs the default 128 VGPRs on the C4 configs; (2) delta-CRDT configs with
# 256-replica buckets (AGX_BUCKET_ACTORS=256: ~1000 tells per bucket, below one tile) vs 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
one() {  # tag env... config
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python tools/cfg_one.py $cfg > gpurun_out/r06g_${tag}_$cfg.json 2> gpurun_out/r06g_${tag}_$cfg.err || { tail -5 gpurun_out/r06g_${tag}_$cfg.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))[sys.argv[2]]; print(sys.argv[3], sys.argv[2], '%.3g'%d['value'], round(d['ms_per_step'],3), d.get('kernel_ms_per_step'))" gpurun_out/r06g_${tag}_$cfg.json $cfg $tag
}
for c in C4_gcounter_gossip C4_orset_gossip C4_orset_delta_gossip C4_gcounter_delta_gossip; do
  one def $c X=0 && one w2 $c AKKA_AMD_LIB=akka_amd/lib/var/r06w2.so || exit 1
done
for c in C4_orset_delta_gossip C4_gcounter_delta_gossip; do
  one b256 $c AGX_BUCKET_ACTORS=256 && one b1024 $c AGX_BUCKET_ACTORS=1024 || exit 1
done
