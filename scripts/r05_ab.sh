#!/usr/bin/env bash
# r05: unit test of the LCP linear solve, the GPU suite (-s) on the default
# library, the contact legs per library build (A/B, one process per library),
# then the driver's bench command.  A test failure (exit 1) does not stop the
# session; a timeout / abort / crash does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r05b}; shift
OUT=gpurun_out/$tag
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 120 python -u -m pytest tests/test_gpu_lcp_solve.py -v -s --timeout 100 --timeout-method thread > "$OUT/pytest_lcp_solve.log" 2>&1
rc=$?; echo "lcp solve rc=$rc"; grep -E "passed|failed|worst" "$OUT/pytest_lcp_solve.log" | tail -4; fatal $rc lcp_solve
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" "$OUT/pytest_gpu.log" | tail -1; grep -E "^tests.*(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head; fatal $rc suite
fi
for lib in "$@"; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 400 python -u scripts/leg_probe.py ${LEGS:-humanoid humanoid/8 contacts quadruped scene} > "$OUT/legs_$lib.log" 2>&1
  rc=$?; echo "$lib legs rc=$rc"; grep -o '^[a-z/0-9]* \|"ms_per_step": [0-9.]*\|"projected_ms_per_step": [0-9.]*\|"lcp_unconverged_world_steps": [0-9]*' "$OUT/legs_$lib.log" | tr '\n' ' '; echo
  fatal $rc legs
done
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; head -c 600 "$OUT/bench.json"; echo; fatal $rc bench
fi
exit 0
