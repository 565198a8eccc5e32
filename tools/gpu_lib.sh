# helpers for gpurun scripts: `source tools/gpu_lib.sh <outdir>`; then `step <name> <timeout> <cmd...>`
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # stop the whole script after a timeout / abort / crash (no further GPU work in this call)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after $name"; exit $rc;; esac
  return 0
}
