"""Debug helper: world-0 state of the Panda env kernel, the scenario kernel and
the oracle for the first steps from the same start state."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gym-ignition_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as O  # noqa: E402
from mwstep import get_model_file  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402
from test_gpu_panda import _oracle_world, _sim  # noqa: E402

np.set_printoptions(precision=7, suppress=False, linewidth=200)
W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
env = VecEnv("PandaPositionTracking", n_worlds=W, seed=3, max_episode_steps=0)
cm = O.load_urdf(get_model_file("panda"))
obs0 = env.reset().cpu().numpy()
q0 = obs0[0, :9].copy()
print("q0", q0)
ow = _oracle_world(O, cm, q0, np.zeros(9), q0.astype(float), O.POSITION)
sim = _sim(1)
sim.set("reset_q", q0[None])
sim.run(paused=True)
sim.set_control_mode(5)
tg_all = np.repeat(obs0[:, :9][None], 3, axis=0).astype(np.float32)
for k in range(3):
    tg_all[k, :, 0] += np.float32(0.9 * 2.8973 * np.sin(2 * np.pi * 0.33 * k * 1e-3))
    tg_all[k, :, 5] += np.float32(0.9 * 1.885 * np.sin(2 * np.pi * 0.33 * k * 1e-3))
for k in range(3):
    tgt = tg_all[k]
    o = env.step(torch.from_numpy(np.ascontiguousarray(tgt)).cuda())[0].cpu().numpy()
    sim.set("position_target", tgt[0][None].astype(np.float64))
    sim.run()
    ow.ptgt[:] = tgt[0]
    ow.run()
    print(f"--- step {k}")
    print(" env  q ", o[0, :9]); print(" scen q ", sim.get("q")[0]); print(" orc  q ", ow.q)
    print(" env  qd", o[0, 9:]); print(" scen qd", sim.get("qd")[0]); print(" orc  qd", ow.qd)
