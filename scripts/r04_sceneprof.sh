#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04l}
mkdir -p "$OUT"
MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so MW_PROF_MODEL=scene3 MW_PROF_T=100 timeout -k 10 300 python -u scripts/wave_prof.py 4096 > "$OUT/scene_prof.log" 2>&1
rc=$?; echo "scene prof rc=$rc"; grep -v amdgpu.ids "$OUT/scene_prof.log"; exit $rc
