#!/usr/bin/env bash
# Copy the judged summaries of one gpu_check.sh session from gpurun_out/ into
# profiles/<tag>/ (tracked).  Usage: scripts/collect_profiles.sh r02a
set -eu
tag="$1"; G=gpurun_out; P=profiles/$tag
mkdir -p "$P"
cp "$G/bench_$tag.json" "$P/bench.json"
cp "$G/pytest_gpu_$tag.log" "$P/pytest_gpu.log"
cp "$G/smoke_$tag.log" "$P/smoke.log"
cp "$G/session.log" "$P/session.log"
cp "$G/prof_$tag/run_kernel_stats.csv" "$P/bench_kernel_stats.csv"
[ -f "$G/prof_panda_$tag/run_kernel_stats.csv" ] && cp "$G/prof_panda_$tag/run_kernel_stats.csv" "$P/panda_kernel_stats.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | tr A-Z a-z)
  [ -f "$G/pmc_${c}_$tag/run_counter_collection.csv" ] && cp "$G/pmc_${c}_$tag/run_counter_collection.csv" "$P/pmc_$lc.csv"
  [ -f "$G/pmc_panda_${c}_$tag/run_counter_collection.csv" ] && cp "$G/pmc_panda_${c}_$tag/run_counter_collection.csv" "$P/pmc_panda_$lc.csv"
done
[ -f "$G/pmc_wave_$tag/run_counter_collection.csv" ] && cp "$G/pmc_wave_$tag/run_counter_collection.csv" "$P/pmc_wave_sq.csv"
python scripts/trace_summary.py "$G/prof_$tag/run_kernel_trace.csv" "$G/bench_prof_$tag.json" > "$P/trace_summary.json" || true
python scripts/pmc_summary.py "$G/pmc_FETCH_SIZE_$tag" "$G/pmc_WRITE_SIZE_$tag" profiles/pmc_summary.json
python scripts/pmc_summary.py "$G/pmc_panda_FETCH_SIZE_$tag" "$G/pmc_panda_WRITE_SIZE_$tag" profiles/pmc_summary_panda.json \
  --kernel vecenv_pid_group_kernel --task PandaPositionTracking --worlds 1024
ls -la "$P"
