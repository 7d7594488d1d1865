"""Per-dof error of the Panda vecenv (fp32 HIP) against the fp64 oracle:
free-running tracking (the test_panda_vecenv_vs_oracle setup) and the error
curve over time, to find which joints carry the fp32/fp64 drift."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as oracle  # noqa: E402
from mwstep import get_model_file  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402
from test_gpu_panda import _oracle_world  # noqa: E402

W, H = 32, 300
env = VecEnv("PandaPositionTracking", n_worlds=W, seed=3, max_episode_steps=10000)
cm = oracle.load_urdf(get_model_file("panda"))
for i in range(cm.n):
    cm.model.lower[i] = float(np.float32(cm.model.lower[i]))
    cm.model.upper[i] = float(np.float32(cm.model.upper[i]))
obs0 = env.reset().cpu().numpy()
ows = [_oracle_world(oracle, cm, obs0[w, :9], np.zeros(9), obs0[w, :9].astype(float), oracle.POSITION)
       for w in range(W)]
phase = np.linspace(0, np.pi, W)
eq = np.zeros(9)
eqd = np.zeros(9)
curve = []
for k in range(H):
    t = k * 1e-3
    tgt = obs0[:, :9].astype(np.float64).copy()
    tgt[:, 0] += 0.9 * 2.8973 * np.sin(2 * np.pi * 0.33 * t + phase)
    tgt[:, 5] += 0.9 * 1.885 * np.sin(2 * np.pi * 0.33 * t + phase)
    tgt = tgt.astype(np.float32)
    o = env.step(torch.from_numpy(tgt).cuda())[0].cpu().numpy()
    step_worst = 0.0
    for w in range(W):
        ows[w].ptgt[:] = tgt[w]
        ows[w].run()
        dq = np.abs(o[w, :9] - ows[w].q)
        dqd = np.abs(o[w, 9:] - ows[w].qd)
        eq = np.maximum(eq, dq)
        eqd = np.maximum(eqd, dqd)
        step_worst = max(step_worst, dqd.max(), dq.max())
    if k % 20 == 0 or k == H - 1:
        curve.append((k, step_worst))
np.set_printoptions(precision=2)
print("max |dq| per dof ", eq)
print("max |dqd| per dof", eqd)
print("curve", [(k, f"{e:.1e}") for k, e in curve])
# the one-step (fresh PID) case: per dof
