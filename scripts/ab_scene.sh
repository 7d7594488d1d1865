#!/usr/bin/env bash
# A/B of scene-kernel builds on the scene leg, one library per process:
#   bash scripts/ab_scene.sh <out dir> lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    MWSTEP_LIB=$PWD/gym-ignition_amd/$lib timeout -k 10 120 python scripts/leg_probe.py scene > "$OUT/leg_${lib}_$rep.log" 2>&1
    rc=$?; echo "$lib rep $rep rc=$rc: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/leg_${lib}_$rep.log")"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
