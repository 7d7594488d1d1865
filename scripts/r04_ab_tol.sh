#!/usr/bin/env bash
# r04: exact-LCP tolerance A/B -- per library the contact legs, then the
# contact KATs / parity tests (one pytest process per library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04f}; shift
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
for lib in "$@"; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 300 python -u scripts/leg_probe.py humanoid contacts > "$OUT/legs_$lib.log" 2>&1
  rc=$?; echo "$lib legs rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"lcp_unconverged_world_steps": [0-9]*' "$OUT/legs_$lib.log" | tr '\n' ' '; echo
  fatal $rc legs
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py \
    tests/test_gpu_free_body.py tests/test_gpu_float_tree.py -v -s --timeout 400 --timeout-method thread > "$OUT/pytest_$lib.log" 2>&1
  rc=$?; echo "$lib pytest rc=$rc"; grep -E "passed|failed" "$OUT/pytest_$lib.log" | tail -1; grep -E "FAILED" "$OUT/pytest_$lib.log" | head
  fatal $rc pytest
done
for plib in libmwstep_prof.so libmwstep_prof4.so; do
  [ -f gym-ignition_amd/$plib ] || continue
  MWSTEP_LIB=gym-ignition_amd/$plib MW_PROF_RANDOM=1 MW_PROF_T=200 timeout -k 10 200 \
    python -u scripts/wave_prof.py 512 50 > "$OUT/wave_prof_$plib.log" 2>&1
  rc=$?; echo "wave_prof $plib rc=$rc"; tail -3 "$OUT/wave_prof_$plib.log"; fatal $rc wave_prof
  MWSTEP_LIB=gym-ignition_amd/$plib MW_PROF_MODEL=cube MW_PROF_T=200 timeout -k 10 200 \
    python -u scripts/wave_prof.py 4096 > "$OUT/wave_prof_cube_$plib.log" 2>&1
  rc=$?; echo "wave_prof cube $plib rc=$rc"; cat "$OUT/wave_prof_cube_$plib.log" | grep -v amdgpu.ids; fatal $rc wave_prof
done
exit 0
