"""Summarise rocprofv3 --pmc passes over the config-5 humanoid leg
(scripts/leg_probe.py humanoid / humanoid_pgs) into profiles/pmc_summary_wave.json:
per-launch SQ counters of wave_run_kernel at the leg's world count, median over
the dispatches of that size.  bench.py's valu_roofline reads the entry that
matches its world count and solver mode.

    python scripts/pmc_wave_summary.py OUT.json DIR:exact DIR:pgs [--worlds 512]"""
import argparse
import csv
import glob
import json
import os
import statistics

COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_WAVES", "SQ_WAVE_CYCLES",
            "SQ_WAIT_ANY", "SQ_BUSY_CYCLES")


def _rows(d):
    """(kernel, grid size in work-items, dispatch, counter, value) from the pass's
    CSV (--output-format csv) or its rocpd database (the default output)"""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if path:
        for r in csv.DictReader(open(path[0])):
            yield (r["Kernel_Name"], int(r["Grid_Size"]), r["Dispatch_Id"], r["Counter_Name"],
                   float(r["Counter_Value"])), path[0]
        return
    path = glob.glob(os.path.join(d, "**", "*_results.db"), recursive=True)
    if not path:
        raise SystemExit(f"no counter collection under {d}")
    import sqlite3
    con = sqlite3.connect(path[0])
    q = "select kernel_name, grid_size, dispatch_id, counter_name, value from counters_collection"
    for r in con.execute(q):
        yield (r[0], int(r[1]), r[2], r[3], float(r[4])), path[0]


def summarise(d, worlds):
    per, src = {}, None
    for (kernel, grid, disp, name, value), src in _rows(d):
        if "wave_run_kernel" not in kernel or grid != worlds * 64:
            continue
        per.setdefault(name, {}).setdefault(disp, 0.0)
        per[name][disp] += value
    out = {k: statistics.median(v.values()) for k, v in per.items()}
    n = max((len(v) for v in per.values()), default=0)
    return out, n, os.path.relpath(src) if src else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+", help="DIR:exact or DIR:pgs")
    ap.add_argument("--worlds", type=int, default=512)
    a = ap.parse_args()
    entries = []
    for spec in a.dirs:
        d, mode = spec.rsplit(":", 1)
        c, n, src = summarise(d, a.worlds)
        e = {"worlds": a.worlds, "exact_lcp": mode == "exact", "dispatches": n, "source": src,
             "valu_insts_per_launch": c.get("SQ_INSTS_VALU")}
        e.update({k.lower(): c.get(k) for k in COUNTERS})
        if c.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
        entries.append(e)
    json.dump({"kernel": "wave_run_kernel (wave_tree.hpp), humanoid32", "entries": entries,
               "counters": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass per solver mode)"},
              open(a.out, "w"), indent=1)
    print(json.dumps(entries, indent=1))


if __name__ == "__main__":
    main()
