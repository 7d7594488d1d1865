"""Run selected bench.py legs alone (one GPU) and print their JSON:
    python scripts/leg_probe.py humanoid humanoid_pgs scene contacts quadruped panda
Legs skip their CPU baselines."""
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


def _with_budget(budget):
    """legs named leg@B run the exact LCP with a budget of B linear solves"""
    def init(self, *a, **kw):
        _init(self, *a, **kw)
        if budget:
            self.set_lcp_solver(True, budget)
    _sim.Simulator.__init__ = init


for spec in sys.argv[1:] or ["humanoid", "humanoid_pgs", "scene"]:
    leg, _, budget = spec.partition("@")
    _with_budget(int(budget) if budget else 0)
    if leg == "humanoid":
        out = bench.humanoid_leg(args, dev, torch)
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
