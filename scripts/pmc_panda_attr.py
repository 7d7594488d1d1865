#!/usr/bin/env python3
"""Attribute config 4's counter traffic.

Reads the per-dispatch counter CSVs that scripts/r05_pmc_panda.sh leaves
under gpurun_out/<tag>/pmc_*/ and reports, for vecenv_pid_group_kernel<9>,
the median per launch of every counter together with a fit of FETCH_SIZE over
the world count: FETCH(W) = code + data(W).  The code term is compared with
the kernel's code-object size (llvm-readelf on the gfx950 object that
`hipcc --save-temps` leaves for csrc/group_kernel.hip) times the 8 XCDs whose
L2 each fetch a copy.

    python3 scripts/pmc_panda_attr.py gpurun_out/r05p --code-object \
        /tmp/t/group_kernel-hip-amdgcn-amd-amdhsa-gfx950.out > profiles/r05p/...json
"""
import argparse
import csv
import glob
import json
import os
import statistics
import subprocess

KERNEL = "vecenv_pid_group_kernel<9, false, true>"
WORLDS = {"pmc_fetch64": 64, "pmc_fetch256": 256, "pmc_fetch1024": 1024}


def code_bytes(obj):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--syms", "-C", obj],
                         capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        if KERNEL in line and "FUNC" in line and ".kd" not in line:
            return int(line.split()[2], 0)
    raise SystemExit(f"{KERNEL} not in {obj}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--code-object")
    ap.add_argument("--alg-read-per-world", type=float, default=260.0,
                    help="algorithmic bytes read per world per launch (bench.py panda_bytes_per_env_step)")
    ap.add_argument("--alg-write-per-world", type=float, default=297.0)
    a = ap.parse_args()
    med = {}
    for d in sorted(glob.glob(os.path.join(a.root, "pmc_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        acc = {}
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        med[os.path.basename(d)] = {c: statistics.median(v) for c, v in acc.items()}
    res = {"kernel": KERNEL, "median_per_launch": med}
    fetch = {WORLDS[k]: med[k]["FETCH_SIZE"] * 1024 for k in WORLDS if k in med}
    res["fetch_bytes_by_worlds"] = fetch
    if a.code_object:
        cb = code_bytes(a.code_object)
        res["code_bytes"] = cb
        res["code_bytes_x8_xcd"] = 8 * cb
        res["data_fetch_bytes_by_worlds"] = {w: f - 8 * cb for w, f in fetch.items()}
        res["alg_read_bytes_by_worlds"] = {w: a.alg_read_per_world * w for w in fetch}
        if "pmc_write1024" in med and 1024 in fetch:
            wr = med["pmc_write1024"]["WRITE_SIZE"] * 1024
            alg = (a.alg_read_per_world + a.alg_write_per_world) * 1024
            res["at_1024"] = {
                "fetch": fetch[1024], "write": wr, "algorithmic": alg,
                "ratio_all": (fetch[1024] + wr) / alg,
                "ratio_without_code": (fetch[1024] - 8 * cb + wr) / alg,
            }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
