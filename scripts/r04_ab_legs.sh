#!/usr/bin/env bash
# r04: contact legs per library build (A/B), then the contact tests on the first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04p}; shift
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
for lib in "$@"; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 400 python -u scripts/leg_probe.py humanoid contacts quadruped scene > "$OUT/legs_$lib.log" 2>&1
  rc=$?; echo "$lib legs rc=$rc"; grep -o '^[a-z/0-9]* \|"ms_per_step": [0-9.]*\|"lcp_unconverged_world_steps": [0-9]*' "$OUT/legs_$lib.log" | tr '\n' ' '; echo
  fatal $rc legs
done
MWSTEP_LIB=gym-ignition_amd/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_float_tree.py tests/test_gpu_scene.py \
  tests/test_gpu_scenario_scene.py tests/test_gpu_free_body.py tests/test_gpu_health.py tests/test_gpu_shard.py \
  -v -s --timeout 400 --timeout-method thread > "$OUT/pytest_$1.log" 2>&1
rc=$?; echo "pytest $1 rc=$rc"; grep -E "passed|failed" "$OUT/pytest_$1.log" | tail -1; grep -E "^tests.*FAILED" "$OUT/pytest_$1.log" | head
exit $rc
