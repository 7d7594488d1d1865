#!/usr/bin/env bash
# r04: scene kernel with the two-stage warm record -- scene tests, the scene leg
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04i}
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py tests/test_gpu_ball_joint.py \
  tests/test_gpu_health.py tests/test_gpu_mesh.py -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_scene.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest_scene.log" | tail -1; grep FAILED "$OUT/pytest_scene.log" | head
fatal $rc pytest
timeout -k 10 300 python -u scripts/leg_probe.py scene > "$OUT/legs_scene.log" 2>&1
rc=$?; echo "legs rc=$rc"; grep -v amdgpu.ids "$OUT/legs_scene.log" | cut -c1-600; fatal $rc legs
exit 0
