#!/usr/bin/env bash
# One GPU-box session, part 1: tests -> smoke -> bench -> rocprofv3 kernel trace
# (scripts/gpu_check.sh split in two so each gpurun call stays short).
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
    echo "FATAL: step '$2' exited with $1; no further GPU steps" | tee -a "$OUT/session.log"
    exit "$1"
  fi
}
echo "== pytest -m gpu" | tee "$OUT/session.log"
timeout -k 10 720 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$tag.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/session.log"; tail -5 "$OUT/pytest_gpu_$tag.log"
stop_if_fatal $rc pytest
echo "== smoke" | tee -a "$OUT/session.log"
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$tag.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/session.log"; tail -3 "$OUT/smoke_$tag.log"
stop_if_fatal $rc smoke
echo "== bench" | tee -a "$OUT/session.log"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_$tag.json"; tail -3 "$OUT/bench_$tag.err"
stop_if_fatal $rc bench
echo "== rocprofv3" | tee -a "$OUT/session.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
  python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/bench_prof_$tag.json" 2> "$OUT/prof_$tag.err"
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/session.log"; tail -3 "$OUT/prof_$tag.err"
find "$OUT/prof_$tag" -name "*stats*" | head
stop_if_fatal $rc rocprof
exit 0
