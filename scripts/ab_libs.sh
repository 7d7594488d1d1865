#!/usr/bin/env bash
# A/B of bench legs over several builds of the library (one per process):
#   scripts/ab_libs.sh TAG "LEGS" lib1.so lib2.so ...   (libraries under gym-ignition_amd/)
# then, if AB_TESTS is set, those GPU tests on the last library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"; tag="$1"; legs="$2"; shift 2
last=""
for lib in "$@"; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 300 python -u scripts/leg_probe.py $legs > "$OUT/ab_${tag}_$lib.log" 2>&1
  rc=$?; echo "$lib rc=$rc"; grep -v amdgpu.ids "$OUT/ab_${tag}_$lib.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
  last=$lib
done
if [ -n "${AB_TESTS:-}" ]; then
  MWSTEP_LIB=gym-ignition_amd/$last timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/ab_${tag}_pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/ab_${tag}_pytest.log"; exit $rc
fi
