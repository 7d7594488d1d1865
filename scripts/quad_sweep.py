"""Quadruped (floating base + contacts) throughput vs world count on one GPU:
the bench's quadruped leg at several W.  Usage: python scripts/quad_sweep.py [W ...]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    # args: W ... [pgs=K] [ground=0|1]
    opts = dict(a.split("=") for a in sys.argv[1:] if "=" in a)
    sizes = [int(a) for a in sys.argv[1:] if "=" not in a] or [1024, 4096, 16384, 65536]
    pgs, ground = int(opts.get("pgs", 20)), opts.get("ground", "1") != "0"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    args = types.SimpleNamespace(seed=42)
    for W in sizes:
        r = bench.quadruped_leg(args, dev, torch, W=W, pgs=pgs, ground=ground)
        print(json.dumps({"worlds": W, "pgs": pgs, "ground": ground, "env_steps_per_s": r["value"],
                          "us_per_step": r["kernel_us_per_launch"], "contacts": r["contact_points_sampled"]}),
              flush=True)
