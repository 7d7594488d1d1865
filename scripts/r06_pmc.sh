#!/usr/bin/env bash
# Counter passes of round 6's final tree, one rocprofv3 run per pass (no trace
# domains with --pmc): HBM bytes of the headline step kernel and of config 4's
# group kernel, and the SQ pass of config 5's wave kernel on the iCub model.
# A pass that times out or faults ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
tag="${1:-r06pmc}"
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1" | tee -a "$OUT/pmc_session_$tag.log"; exit "$1"; fi; }
: > "$OUT/pmc_session_$tag.log"
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== headline pmc $ctr" | tee -a "$OUT/pmc_session_$tag.log"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_${ctr}_$tag" -o run -- \
    python3 scripts/profile_step.py > "$OUT/pmc_${ctr}_$tag.log" 2>&1
  fatal $? "headline pmc $ctr"
  echo "== panda pmc $ctr" | tee -a "$OUT/pmc_session_$tag.log"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_panda_${ctr}_$tag" -o run -- \
    python3 scripts/profile_panda.py > "$OUT/pmc_panda_${ctr}_$tag.log" 2>&1
  fatal $? "panda pmc $ctr"
done
echo "== wave kernel SQ pmc humanoid" | tee -a "$OUT/pmc_session_$tag.log"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES \
  SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_wave_humanoid_$tag" -o run -- \
  python3 scripts/leg_probe.py humanoid > "$OUT/pmc_wave_humanoid_$tag.log" 2>&1
fatal $? "wave pmc"
echo "done" | tee -a "$OUT/pmc_session_$tag.log"
