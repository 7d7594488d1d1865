"""Debug helper: first (step, world, dof) where the PandaPositionTracking env
diverges from the oracle ScenarioWorld (prints the joint's state vs its limits)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gym-ignition_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as O  # noqa: E402
from mwstep import get_model_file  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402
from test_gpu_panda import _oracle_world  # noqa: E402

W, H = 32, 300
env = VecEnv("PandaPositionTracking", n_worlds=W, seed=3, max_episode_steps=0)
cm = O.load_urdf(get_model_file("panda"))
for i in range(cm.n):
    cm.model.lower[i] = float(np.float32(cm.model.lower[i]))
    cm.model.upper[i] = float(np.float32(cm.model.upper[i]))
obs0 = env.reset().cpu().numpy()
ows = [_oracle_world(O, cm, obs0[w, :9], np.zeros(9), obs0[w, :9].astype(float), O.POSITION) for w in range(W)]
phase = np.linspace(0, np.pi, W)
lo = np.array([cm.model.lower[i] for i in range(9)])
hi = np.array([cm.model.upper[i] for i in range(9)])
reported = 0
for k in range(H):
    t = k * 1e-3
    tgt = obs0[:, :9].astype(np.float64).copy()
    tgt[:, 0] += 0.9 * 2.8973 * np.sin(2 * np.pi * 0.33 * t + phase)
    tgt[:, 5] += 0.9 * 1.885 * np.sin(2 * np.pi * 0.33 * t + phase)
    tgt = tgt.astype(np.float32)
    o, r, d, info = env.step(torch.from_numpy(tgt).cuda())
    o = o.cpu().numpy()
    for w in range(W):
        qprev = ows[w].q.copy()
        ows[w].ptgt[:] = tgt[w]
        ows[w].run()
        e = np.abs(o[w, 9:] - ows[w].qd)
        if e.max() > 1e-3 and reported < 8:
            dd = int(e.argmax())
            print(f"step {k} world {w} dof {dd}: qd gpu {o[w, 9 + dd]:.6f} oracle {ows[w].qd[dd]:.6f} | "
                  f"q prev {qprev[dd]:.9f} now {ows[w].q[dd]:.9f} gpu {o[w, dd]:.9f} lim [{lo[dd]:.9f}, {hi[dd]:.9f}] "
                  f"tgt {tgt[w, dd]:.6f}")
            reported += 1
print("done")
