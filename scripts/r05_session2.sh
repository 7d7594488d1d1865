#!/usr/bin/env bash
# r05: counter list, cube / humanoid phase profiles (debug build), Panda
# counter passes that split the L2 fetches of vecenv_pid_group_kernel<9>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r05o}
OUT=gpurun_out/$tag
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"
grep -oE "(SQC|TCC|TCP|TA|TD)_[A-Z0-9_]+" "$OUT/counters.txt" | sort -u > "$OUT/counter_names.txt"; wc -l < "$OUT/counter_names.txt"
MW_PROF_MODEL=cube MW_PROF_T=200 MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so timeout -k 10 180 python -u scripts/wave_prof.py 4096 20 > "$OUT/prof_cube.log" 2>&1
rc=$?; echo "cube prof rc=$rc"; grep -v amdgpu.ids "$OUT/prof_cube.log"; fatal $rc cube
MW_PROF_RANDOM=1 MW_PROF_T=200 MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so timeout -k 10 180 python -u scripts/wave_prof.py 64 50 > "$OUT/prof_h64.log" 2>&1
rc=$?; echo "humanoid prof rc=$rc"; grep -v amdgpu.ids "$OUT/prof_h64.log"; fatal $rc hprof
for set in "${PMC_SETS[@]:-}"; do :; done
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$OUT/pmc_panda_$i" -o run -- python3 scripts/profile_panda.py > "$OUT/pmc_panda_$i.log" 2>&1
  rc=$?; echo "pmc set $i ($ctrs) rc=$rc"; fatal $rc pmc
done < "${PMC_FILE:-/dev/null}"
exit 0
