#!/usr/bin/env bash
# r04: exact-LCP debug probes on the free-body parity states, then the LCP suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
for m in double cube rock; do
  timeout -k 10 120 python -u scripts/dbg_free_exact.py $m > "$OUT/dbg_$m.log" 2>&1
  rc=$?; echo "dbg $m rc=$rc"; head -5 "$OUT/dbg_$m.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash scripts/r04_lcp.sh "${1:-r04e}"
