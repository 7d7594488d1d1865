#!/usr/bin/env bash
# Round 6: large-contact scene steps -- their GPU tests, the scene GPU suite, the scene leg
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06e}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_scene_big.py -x -v -s --timeout 200 --timeout-method thread > "$OUT/pytest_big.log" 2>&1
rc=$?; echo "big rc=$rc"; tail -15 "$OUT/pytest_big.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_scene.py tests/test_gpu_scenario_scene.py tests/test_gpu_lcp_converge.py tests/test_gpu_mesh.py -v -s --timeout 200 --timeout-method thread > "$OUT/pytest_scene.log" 2>&1
rc2=$?; echo "scene rc=$rc2"; tail -4 "$OUT/pytest_scene.log"
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 200 python scripts/leg_probe.py scene > "$OUT/legs.log" 2>&1
rc3=$?; echo "legs rc=$rc3"; tail -3 "$OUT/legs.log"
exit $(( rc || rc2 || rc3 ))
