#!/usr/bin/env bash
# A/B of the exact-LCP legs: the in-tree library vs gym-ignition_amd/libmwstep_base.so
# (one library per process), then the contact GPU tests on the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"; tag="${1:-ab}"
for lib in libmwstep_base.so libmwstep.so; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 240 python -u scripts/leg_probe.py humanoid scene > "$OUT/ab_${tag}_$lib.log" 2>&1
  rc=$?; echo "$lib rc=$rc"; cat "$OUT/ab_${tag}_$lib.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_float_tree.py tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/ab_${tag}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/ab_${tag}_pytest.log"; exit $rc
