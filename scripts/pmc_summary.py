"""Summarise rocprofv3 PMC passes of scripts/profile_step.py into
profiles/pmc_summary.json (per-launch HBM bytes of the step kernel).

    python scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE_rNN gpurun_out/pmc_WRITE_SIZE_rNN out.json

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


def median_counter(d, name):
    path = os.path.join(d, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and "vecenv_step_kernel" in r["Kernel_Name"]]
    return statistics.median(vals), len(vals)


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, nf = median_counter(fdir, "FETCH_SIZE")
    write, nw = median_counter(wdir, "WRITE_SIZE")
    d = {"task": "CartPoleDiscreteBalancing", "worlds": 4096, "dispatches": [nf, nw],
         "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
         "bytes_per_launch": int(round((fetch + write) * 1024)),
         "note": "raw FETCH_SIZE + WRITE_SIZE (KiB x 1024) per dispatch, median over dispatches; "
                 "4 B/lane loads: the gfx950 x2 FETCH correction for 16 B/lane streams is not applied"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
