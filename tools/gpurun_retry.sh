#!/bin/bash
# gpurun with retries on INFRASTRUCTURE transients only (box lost before the command ran, no slot):
# tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'.  A command that ran (pass or fail) is never retried.
out=$1; to=$2; shift 2
for i in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then
    echo "transient (try $i), retrying in 240 s" >> "$out.retries"; sleep 240; continue
  fi
  echo "rc=$rc" >> "$out.retries"
  exit $rc
done
exit 3
