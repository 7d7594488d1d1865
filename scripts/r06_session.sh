#!/usr/bin/env bash
# One GPU-box session of round 6: GPU tests, smoke, the driver's bench command.
# Any step that times out, aborts or faults ends the session (no further GPU work);
# a plain test failure (pytest exit 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
tag="${1:-r06}"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1" | tee -a "$OUT/session_$tag.log"; exit "$1"; fi; }
echo "== pytest -m gpu" | tee "$OUT/session_$tag.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$tag.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/session_$tag.log"; tail -3 "$OUT/pytest_gpu_$tag.log"; fatal $rc pytest
echo "== smoke" | tee -a "$OUT/session_$tag.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$tag.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/session_$tag.log"; tail -2 "$OUT/smoke_$tag.log"; fatal $rc smoke
echo "== bench" | tee -a "$OUT/session_$tag.log"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/session_$tag.log"; tail -c 600 "$OUT/bench_$tag.json"; fatal $rc bench
if [ "${TRACE:-1}" = "1" ]; then
  # the driver's own command under the kernel tracer (no counters): the timed
  # dispatches of the headline kernel (scripts/trace_summary.py)
  echo "== rocprofv3 kernel trace of the driver command" | tee -a "$OUT/session_$tag.log"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_prof_$tag.json" 2> "$OUT/prof_$tag.err"
  rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/session_$tag.log"; fatal $rc rocprof
  python scripts/trace_summary.py "$(find "$OUT/prof_$tag" -name 'run_kernel_trace.csv' | head -1)" "$OUT/bench_prof_$tag.json" \
    > "$OUT/trace_summary_$tag.json"; cat "$OUT/trace_summary_$tag.json"
fi
exit 0
