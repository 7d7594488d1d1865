#!/usr/bin/env bash
# r04: elimination variants -- contact legs + contact tests (r04_ab_legs.sh),
# then the wave kernel's phase split per profiling build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
bash scripts/r04_ab_legs.sh "$tag" "$@" || exit $?
for l in "$@"; do
  p=${l/libmwstep/libmwstep_prof}
  [ -f "gym-ignition_amd/$p" ] || continue
  MWSTEP_LIB=gym-ignition_amd/$p MW_PROF_RANDOM=1 MW_PROF_T=200 timeout -k 10 200 python -u scripts/wave_prof.py 512 50 \
    > "gpurun_out/$tag/wave_prof_$p.log" 2>&1 || { echo "FATAL wave_prof $p rc=$?"; exit 1; }
  echo "$p"; grep -E "wall|linear solves|ABA|responses|PGS \+" "gpurun_out/$tag/wave_prof_$p.log"
done
