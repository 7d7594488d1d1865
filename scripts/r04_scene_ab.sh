#!/usr/bin/env bash
# r04: scene leg per library build (tolerance A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04j}; shift
mkdir -p "$OUT"
for lib in "$@"; do
  MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 300 python -u scripts/leg_probe.py scene > "$OUT/legs_scene_$lib.log" 2>&1
  rc=$?; echo "$lib rc=$rc"; grep -v amdgpu.ids "$OUT/legs_scene_$lib.log" | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
done
