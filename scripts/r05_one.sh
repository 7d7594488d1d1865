#!/usr/bin/env bash
# r05: selected GPU tests (-s) on one library, then its legs and phase profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; lib=$2; shift 2
OUT=gpurun_out/$tag
mkdir -p "$OUT"
MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 600 python -u -m pytest "$@" -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_$lib.log" 2>&1
rc=$?; echo "pytest $lib rc=$rc"; grep -E "passed|failed" "$OUT/pytest_$lib.log" | tail -1
grep -E "x512|random states" "$OUT/pytest_$lib.log" | cut -c1-400
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
exit 0
