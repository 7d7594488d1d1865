#!/usr/bin/env bash
# r04: exact-LCP change check -- the contact tests, the contact legs, scene profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04o}
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_float_tree.py tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py \
  tests/test_gpu_mesh.py tests/test_gpu_ball_joint.py tests/test_gpu_health.py tests/test_gpu_golden.py tests/test_gpu_shard.py \
  tests/test_gpu_free_body.py -v -s --timeout 400 --timeout-method thread > "$OUT/pytest_lcp.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest_lcp.log" | tail -1; grep -E "^tests.*FAILED" "$OUT/pytest_lcp.log" | head; fatal $rc pytest
timeout -k 10 400 python -u scripts/leg_probe.py humanoid humanoid/8 contacts quadruped scene > "$OUT/legs.log" 2>&1
rc=$?; echo "legs rc=$rc"; grep -o '^[a-z/0-9]* \|"ms_per_step": [0-9.]*\|"lcp_unconverged_world_steps": [0-9]*' "$OUT/legs.log" | tr '\n' ' '; echo; fatal $rc legs
MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so MW_PROF_MODEL=scene3 MW_PROF_T=100 timeout -k 10 300 python -u scripts/wave_prof.py 4096 > "$OUT/scene_prof.log" 2>&1
rc=$?; echo "scene prof rc=$rc"; grep -v amdgpu.ids "$OUT/scene_prof.log"; fatal $rc scene_prof
MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so MW_PROF_RANDOM=1 MW_PROF_T=200 timeout -k 10 200 python -u scripts/wave_prof.py 512 50 > "$OUT/wave_prof.log" 2>&1
rc=$?; echo "wave_prof rc=$rc"; tail -10 "$OUT/wave_prof.log"; fatal $rc wave_prof
exit 0
