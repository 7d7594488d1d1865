#!/usr/bin/env bash
# gpurun with retries ONLY for infrastructure outcomes that ran nothing
# (status=transient / exit 3: no box, box lost while being prepared).  A call
# whose command ran is never repeated.  Usage: scripts/gpurun_retry.sh LOG TIMEOUT 'cmd'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ "$rc" -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "attempt $i: infrastructure ($rc), retrying in 90 s" >> "$log.retries"
    sleep 90
    continue
  fi
  exit $rc
done
exit $rc
