#!/bin/bash
# Build libakka_gpu.so with extra compile flags into akka_amd/lib/var/NAME.so (A/B builds for
# tools/ab.sh / tools/ab_cfg.sh via AKKA_AMD_LIB): tools/build_variant.sh NAME -DFOO=0 ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=${SRC:-$ROOT}  # (SRC=dir: build another checkout's akka_amd/csrc, e.g. a git archive of HEAD)
OUT=$ROOT/akka_amd/lib/var/$NAME; mkdir -p "$OUT"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -I/opt/rocm/include $*"
pids=()
/opt/rocm/bin/hipcc $F -c -o "$OUT/e.o" "$SRC/akka_amd/csrc/agx_engine.hip" & pids+=($!)
for g in 0 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc $F -DAGX_VGROUP=$g -c -o "$OUT/a$g.o" "$SRC/akka_amd/csrc/agx_apply.hip" & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/akka_amd/lib/var/$NAME.so" "$OUT"/*.o -L/opt/rocm/lib -lrccl
rm -rf "$OUT"
echo "$ROOT/akka_amd/lib/var/$NAME.so"
