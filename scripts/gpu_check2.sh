#!/usr/bin/env bash
# One GPU-box session, part 2: the PMC passes of scripts/gpu_check.sh.
# A normal test failure (pytest exit 1) does not stop the session; a timeout,
# abort, segfault or any other exit status does (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
tag="${1:-r01}"
stop_if_fatal() {  # $1 = exit code, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "FATAL: step '$2' exited with $1; no further GPU steps" | tee -a "$OUT/session_pmc.log"
    exit "$1"
  fi
}
echo "== pmc session" > "$OUT/session_pmc.log"
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr" | tee -a "$OUT/session_pmc.log"
  timeout -k 10 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_${ctr}_$tag" -o run -- \
    python3 scripts/profile_step.py > "$OUT/pmc_${ctr}_$tag.log" 2>&1
  rc=$?; echo "pmc $ctr rc=$rc" | tee -a "$OUT/session_pmc.log"
  stop_if_fatal $rc pmc
done
# config 4 (Panda): kernel trace + HBM counters of the position-target env kernel
echo "== panda kernel trace" | tee -a "$OUT/session_pmc.log"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_panda_$tag" -o run --output-format csv -- \
  python3 scripts/profile_panda.py > "$OUT/prof_panda_$tag.log" 2>&1
rc=$?; echo "panda trace rc=$rc" | tee -a "$OUT/session_pmc.log"
stop_if_fatal $rc panda_trace
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== panda pmc $ctr" | tee -a "$OUT/session_pmc.log"
  timeout -k 10 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc_panda_${ctr}_$tag" -o run -- \
    python3 scripts/profile_panda.py > "$OUT/pmc_panda_${ctr}_$tag.log" 2>&1
  rc=$?; echo "panda pmc $ctr rc=$rc" | tee -a "$OUT/session_pmc.log"
  stop_if_fatal $rc panda_pmc
done
# config 5 (humanoid, wave kernel): SQ counters of the step kernel on the bench's
# own humanoid legs (exact LCP, PGS only), one pass each -> profiles/pmc_summary_wave.json
for leg in humanoid humanoid_pgs; do
  echo "== wave kernel SQ pmc $leg" | tee -a "$OUT/session_pmc.log"
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES \
    SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_wave_${leg}_$tag" -o run -- \
    python3 scripts/leg_probe.py $leg > "$OUT/pmc_wave_${leg}_$tag.log" 2>&1
  rc=$?; echo "wave pmc $leg rc=$rc" | tee -a "$OUT/session_pmc.log"
  stop_if_fatal $rc wave_pmc
done
exit 0
