"""Run selected bench.py legs alone (one GPU) and print their JSON:
    python scripts/leg_probe.py humanoid humanoid_pgs scene contacts quadruped panda
Legs skip their CPU baselines.  humanoid/N, humanoid_pgs/N and panda/N run
every rank's share of an N-GPU strong split of configs 5 / 4 one after another
on this GPU (no collective: the worlds are independent) and print each share's
time and the max over the shares: the projected N-GPU step time."""
import json
import os
import sys
import types

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

args = types.SimpleNamespace(seed=42, groups=1, graph_chunk=100, no_cpu_baseline=True, cpu_leg_seconds=0.0)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
bench.hip_runtime()
from mwstep import sim as _sim  # noqa: E402

_init = _sim.Simulator.__init__


from mwstep import scene as _scene  # noqa: E402

_sinit = _scene.Scene.__init__


def _with_budget(budget):
    """legs named leg@B run the exact LCP with a budget of B linear solves"""
    def init(self, *a, **kw):
        _init(self, *a, **kw)
        if budget:
            self.set_lcp_solver(True, budget)

    def sinit(self, *a, **kw):
        _sinit(self, *a, **kw)
        if budget:
            self.set_lcp_solver(True, budget)
    _sim.Simulator.__init__ = init
    _scene.Scene.__init__ = sinit


_NoDist = bench._NoDist


def _shares(fn, n):
    rows = []
    for r in range(n):
        o = fn(r)
        rows.append({"rank": r, "worlds": o.get("worlds_per_gpu"), "ms_per_step": o["ms_per_step"],
                     "kernel_us_per_launch": o.get("kernel_us_per_launch")})
    worst = max(x["ms_per_step"] for x in rows)
    return {"shares": rows, "projected_ms_per_step": worst}


for spec in sys.argv[1:] or ["humanoid", "humanoid_pgs", "scene"]:
    spec_leg, _, nshare = spec.partition("/")
    spec_leg, _, sweeps = spec_leg.partition("%")  # humanoid%20: at most 20 PGS sweeps before the exact solve
    leg, _, budget = spec_leg.partition("@")
    if nshare:
        n = int(nshare)
        _with_budget(int(budget) if budget else 0)
        if leg in ("humanoid", "humanoid_pgs"):
            out = _shares(lambda r: bench.humanoid_leg(args, dev, torch, _NoDist, n, r, exact=(leg == "humanoid")), n)
        elif leg == "panda":
            out = _shares(lambda r: bench.panda_leg(args, dev, torch, _NoDist, n, r), n)
        else:
            raise SystemExit(f"no share run for {leg}")
        print(spec, json.dumps(out), flush=True)
        continue
    _with_budget(int(budget) if budget else 0)
    if leg == "humanoid":
        out = bench.humanoid_leg(args, dev, torch, pgs=int(sweeps) if sweeps else 50)
    elif leg == "humanoid_pgs":
        out = bench.humanoid_leg(args, dev, torch, exact=False)
    elif leg == "scene":
        out = bench.scene_leg(args, dev, torch)
    elif leg == "contacts":
        out = bench.contact_leg(args, dev, torch)
    elif leg == "quadruped":
        out = bench.quadruped_leg(args, dev, torch)
    elif leg == "panda":
        out = bench.panda_leg(args, dev, torch, None)
    else:
        raise SystemExit(f"unknown leg {leg}")
    keep = {k: v for k, v in out.items() if k not in ("workload",)}
    print(spec, json.dumps(keep), flush=True)
    if os.environ.get("LEG_DUMP", "0") == "1":
        # debug library (MW_WAVE_PROF, MW_DUMP_FAIL): the leg's unconverged LCPs
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from lcp_dumps import save_dumps
        from mwstep import native as _N
        if leg == "scene":
            save_dumps(_N.lib().mw_debug_scene_dump, 8, f"leg_{leg}_scene_dump.npz")
        else:
            save_dumps(_N.lib().mw_debug_wave_dump, 9, f"leg_{leg}_wave_dump.npz")
