#!/usr/bin/env bash
# r04: GPU tests of the new health / snapshot paths, then the timing evidence
# of the headline kernel (kernel trace of the driver's bench command, an SQ /
# GRBM counter pass) and the Pendulum kernel's HBM counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04a}
mkdir -p "$OUT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL $2 rc=$1"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_health.py tests/test_gpu_panda.py tests/test_gpu_scenario_scene.py \
  -v --timeout 300 --timeout-method thread > "$OUT/pytest_health.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_health.log"; fatal $rc pytest
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err"
rc=$?; echo "trace rc=$rc"; fatal $rc trace
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  --output-format csv -d "$OUT/pmc_clock" -o run -- python3 scripts/profile_step.py > "$OUT/pmc_clock.log" 2>&1
rc=$?; echo "pmc clock rc=$rc"; fatal $rc pmc_clock
for ctr in FETCH_SIZE WRITE_SIZE; do
  MW_TASK=PendulumSwingUp MW_W=2048 timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
    -d "$OUT/pmc_pend_$ctr" -o run -- python3 scripts/profile_step.py > "$OUT/pmc_pend_$ctr.log" 2>&1
  rc=$?; echo "pmc pend $ctr rc=$rc"; fatal $rc pmc_pend
done
exit 0
