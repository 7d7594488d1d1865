"""Worlds-in-flight probe of the scene kernel: the scene leg at W = 256 .. 1536
(one wave per world).  A launch whose worlds all fit on the chip at once
costs one world-step chain; the step time doubles where they stop fitting,
so the knee gives the worlds (waves) resident per CU:
    python scripts/scene_occupancy.py"""
import json
import os
import sys
import types

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

args = types.SimpleNamespace(seed=42)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for W in [int(x) for x in os.environ.get("OCC_W", "256,512,640,768,1024,1536").split(",")]:
    o = bench.scene_leg(args, dev, torch, W=W, K=int(os.environ.get("OCC_K", "200")), warm=int(os.environ.get("OCC_WARM", "20")), G=20)
    print(json.dumps({"worlds": W, "ms_per_step": o["ms_per_step"]}), flush=True)
