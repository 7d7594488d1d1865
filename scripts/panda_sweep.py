"""Per-GPU step time of BASELINE config 4 (PandaPositionTracking, the group
kernel) at the world counts one rank holds when the 1,024 worlds are split
over 1, 2, 4 and 8 GPUs: runs bench.py's panda_leg on one GPU with
W_global = 1024 / N (one rank's share, same graphs and timing).
    python scripts/panda_sweep.py [W ...]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
import torch  # noqa: E402

import bench  # noqa: E402

Ws = [int(a) for a in sys.argv[1:]] or [128, 256, 512, 1024]
args = types.SimpleNamespace(groups=1, seed=42, graph_chunk=100)
dev = torch.device("cuda", 0)
for W in Ws:
    r = bench.panda_leg(args, dev, torch, None, world_size=1, rank=0, W_global=W)
    print(json.dumps({"worlds": W, "kernel_us_per_launch": r["kernel_us_per_launch"],
                      "ms_per_step": r["ms_per_step"], "env_steps_per_s": r["value"]}), flush=True)
