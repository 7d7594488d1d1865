#!/usr/bin/env bash
# SQ / SQC counter passes of the scene leg (scene_run_kernel), one library per pass set:
#   bash scripts/pmc_scene.sh <out dir> lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for lib in "$@"; do
  n=0
  for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SALU SQ_INSTS_LDS"; do
    n=$((n+1))
    MWSTEP_LIB=$PWD/gym-ignition_amd/$lib timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$OUT/${lib}_p$n" -o run --output-format csv -- python3 scripts/leg_probe.py scene > "$OUT/${lib}_p$n.log" 2>&1
    rc=$?; echo "$lib pass $n rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${lib}_p$n.log"; exit $rc; fi
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, statistics, sys
out = sys.argv[1]
for lib in sys.argv[2:]:
    vals = {}
    for f in glob.glob(f"{out}/{lib}_p*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "scene_run_kernel" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(lib, {k: round(statistics.median(v), 1) for k, v in sorted(vals.items())})
PY
