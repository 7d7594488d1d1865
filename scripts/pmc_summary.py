"""Summarise rocprofv3 PMC passes of scripts/profile_step.py into
profiles/pmc_summary.json (per-launch HBM bytes of the step kernel).

    python scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE_rNN gpurun_out/pmc_WRITE_SIZE_rNN out.json
    python scripts/pmc_summary.py FETCH_DIR WRITE_DIR out.json --kernel vecenv_pid_step_kernel \
        --task PandaPositionTracking --worlds 1024        (config-4 Panda env)

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters
from TCC_EA0_RDREQ/WRREQ).  MI355X_MICROARCH.md: FETCH_SIZE reads exactly half
of a wide (16 B/lane) coalesced streaming read; other widths are uncalibrated.
The step kernel's loads are 4 B/lane (SoA q, qd, action, counters), so the raw
value is reported; both raw counters are kept in the summary.
"""
import csv
import json
import os
import statistics
import sys


def median_counter(d, name, kernel):
    path = os.path.join(d, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and kernel in r["Kernel_Name"]]
    return statistics.median(vals), len(vals)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="vecenv_step_kernel")
    ap.add_argument("--task", default="CartPoleDiscreteBalancing")
    ap.add_argument("--worlds", type=int, default=4096)
    a = ap.parse_args()
    fdir, wdir, out = a.fetch_dir, a.write_dir, a.out
    fetch, nf = median_counter(fdir, "FETCH_SIZE", a.kernel)
    write, nw = median_counter(wdir, "WRITE_SIZE", a.kernel)
    d = {"task": a.task, "worlds": a.worlds, "kernel": a.kernel, "dispatches": [nf, nw],
         "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
         "bytes_per_launch": int(round((fetch + write) * 1024)),
         "note": "raw FETCH_SIZE + WRITE_SIZE (KiB x 1024) per dispatch, median over dispatches; "
                 "4 B/lane loads: the gfx950 x2 FETCH correction for 16 B/lane streams is not applied"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
