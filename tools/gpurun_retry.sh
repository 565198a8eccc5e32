#!/bin/bash
# gpurun with retries on INFRASTRUCTURE transients only (box lost before the command ran, no slot,
# back-off): tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'.  A command that ran (pass or fail) is
# never retried.  Waits the back-off gpurun names ("retry in Ns"), else 240 s.
out=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then
    w=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | tail -1)
    w=$(( ${w:-230} + 10 ))
    echo "transient (try $i), retrying in $w s" >> "$out.retries"; sleep $w; continue
  fi
  echo "rc=$rc" >> "$out.retries"
  exit $rc
done
exit 3
