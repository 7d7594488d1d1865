"""Profiling workload: 200 PandaPositionTracking steps of 1024 worlds (config 4),
eager launches, for rocprofv3 kernel traces / PMC passes."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import torch  # noqa: E402

from mwstep.vecenv import VecEnv  # noqa: E402

W, T = int(os.environ.get("PANDA_WORLDS", "1024")), 200
env = VecEnv("PandaPositionTracking", n_worlds=W, seed=42)
q0 = env.reset()[:, :9].clone()
t = torch.arange(T, device="cuda", dtype=torch.float32) * 1e-3
s = torch.sin(2 * math.pi * 0.33 * t)[:, None]
tg = q0[None].repeat(T, 1, 1)
tg[:, :, 0] += 0.9 * 2.8973 * s
tg[:, :, 5] += 0.9 * 1.885 * s
tg = tg.contiguous()
for k in range(T):
    env.step(tg[k])
torch.cuda.synchronize()
print("ok", env.sim.baked_model())
