#!/usr/bin/env bash
# r05: wave-kernel phase profiles (shader-clock counters, MW_WAVE_PROF builds)
# for each library given, at 512 and 64 humanoid worlds (the bench leg's random
# start), one process per library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r05h}; shift
OUT=gpurun_out/$tag
mkdir -p "$OUT"
for lib in "$@"; do
  for W in ${WORLDS:-512 64}; do
    MW_PROF_RANDOM=1 MW_PROF_T=200 MWSTEP_LIB=gym-ignition_amd/$lib timeout -k 10 180 python -u scripts/wave_prof.py $W 50 > "$OUT/prof_${lib}_$W.log" 2>&1
    rc=$?; echo "$lib W=$W rc=$rc"; cat "$OUT/prof_${lib}_$W.log" | grep -v amdgpu.ids
    if [ "$rc" -ne 0 ]; then exit $rc; fi
  done
done
exit 0
