#!/usr/bin/env bash
# r05: dump unconverged exact LCPs (debug library built with
# EXTRA="-DMW_WAVE_PROF -DMW_DUMP_FAIL" as libmwstep_dump.so) from the contacts
# leg (4096 cubes), the scene leg (4096 x 3 cubes) and the humanoid (512,
# random start); scripts/lcp_dump_check.py reads them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05q}
mkdir -p "$OUT"
for m in cube:4096 scene3:4096 humanoid32:512; do
  model=${m%%:*}; w=${m##*:}
  MW_PROF_RANDOM=1 MW_PROF_MODEL=$model MWSTEP_LIB=gym-ignition_amd/libmwstep_dump.so timeout -k 10 180 python -u scripts/wave_prof.py "$w" > "$OUT/dump_$model.log" 2>&1
  rc=$?; echo "dump $model rc=$rc"; tail -12 "$OUT/dump_$model.log"
  if [ "$rc" -ne 0 ]; then exit $rc; fi
  for f in wave_dump.npz scene_dump.npz; do
    if [ -f gpurun_out/$f ]; then mv gpurun_out/$f "$OUT/${model}_$f"; fi
  done
done
exit 0
