#!/usr/bin/env bash
# r04: DART two-stage exact LCP -- contact GPU tests, then the config-5 legs
# (512 worlds and the 8-GPU share projection).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04b}
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_float_tree.py tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py \
  tests/test_gpu_mesh.py tests/test_gpu_ball_joint.py tests/test_gpu_health.py tests/test_gpu_golden.py tests/test_gpu_shard.py tests/test_gpu_free_body.py \
  -v -s --timeout 400 --timeout-method thread > "$OUT/pytest_lcp.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest_lcp.log" | tail -2; fatal $rc pytest
timeout -k 10 300 python -u scripts/leg_probe.py humanoid humanoid/8 contacts quadruped > "$OUT/legs.log" 2>&1
rc=$?; echo "legs rc=$rc"; tail -c 1500 "$OUT/legs.log"; fatal $rc legs
if [ -f gym-ignition_amd/libmwstep_prof.so ]; then
  MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so MW_PROF_RANDOM=1 MW_PROF_T=200 timeout -k 10 200 \
    python -u scripts/wave_prof.py 512 50 > "$OUT/wave_prof.log" 2>&1
  rc=$?; echo "wave_prof rc=$rc"; tail -14 "$OUT/wave_prof.log"; fatal $rc wave_prof
fi
exit 0
