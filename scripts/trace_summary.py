"""Summarise a rocprofv3 --kernel-trace CSV of bench.py for the dominant
kernel: per-dispatch durations of the timed region vs the bench's own
HIP-event figure.  Usage: trace_summary.py run_kernel_trace.csv bench.json"""
import csv
import json
import statistics
import sys

trace, bench = sys.argv[1], sys.argv[2]
b = json.load(open(bench))
W = b["config"]["worlds_per_gpu"]
rows = [r for r in csv.DictReader(open(trace))
        if "vecenv_step_kernel<2, 0, false, true, false" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == W]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
start = [int(r["Start_Timestamp"]) for r in rows]
warm, steps = b["warmup"], b["steps"]
lo, hi = warm + steps, warm + 2 * steps          # warmup eager, one settle replay of every graph, timed replays
timed = dur[lo:hi]
period = [start[i + 1] - start[i] for i in range(lo, min(hi, len(start)) - 1)]
out = {"kernel": rows[0]["Kernel_Name"].split("(")[0] if rows else None, "worlds": W, "dispatches": len(dur),
       "timed_dispatches": len(timed), "timed_median_ns": statistics.median(timed),
       "timed_mean_ns": round(statistics.mean(timed), 1),
       "timed_min_ns": min(timed), "timed_max_ns": max(timed),
       "timed_start_to_start_mean_ns": round(statistics.mean(period), 1) if period else None,
       "bench_ms_per_step_same_run": b["ms_per_step"],
       "bench_event_us_per_launch": b["roofline"]["kernel_us_per_launch"]}
print(json.dumps(out, indent=1))
