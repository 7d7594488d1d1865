"""per-world wrench indexing: W=8 batch vs W=1 runs of each world (debug)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-ignition_amd", "python"))
import numpy as np
from mwstep import get_model_file
from mwstep import native as N
from mwstep.scene import Scene
from mwstep.sim import Simulator
path = get_model_file("humanoid32")
pose = (0.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0)
rng = np.random.default_rng(7)
W = 8
base_w = np.column_stack([rng.uniform(-5, 5, (W, 3)), rng.uniform(-0.5, 0.5, (W, 3))])


def make(kind, n):
    if kind == "sim":
        s = Simulator(path, n_worlds=n, steps_per_run=1, pose=pose)
    else:
        s = Scene(n_worlds=n, steps_per_run=1)
        s.insert_model(open(path).read(), pose, "h")
    s.set_gravity([0.0, 0.0, 0.0])
    s.run(paused=True)
    if kind == "sim":
        s.set_control_mode(N.MODE_FORCE)
    else:
        s.set_control_mode(N.MODE_FORCE, m=0)
    return s


for kind in ("sim", "scene"):
    s = make(kind, W)
    (s.apply_world_wrench(-1, base_w, 0.010) if kind == "sim" else s.apply_world_wrench(0, -1, base_w, 0.010))
    for _ in range(12):
        s.run()
    qd = s.get("qd") if kind == "sim" else s.get("qd", 0)
    errs = []
    for k in range(W):
        t = make(kind, 1)
        (t.apply_world_wrench(-1, base_w[k:k + 1], 0.010) if kind == "sim" else t.apply_world_wrench(0, -1, base_w[k:k + 1], 0.010))
        for _ in range(12):
            t.run()
        q1 = t.get("qd") if kind == "sim" else t.get("qd", 0)
        errs.append(float(np.abs(q1[0] - qd[k]).max()))
        t.close()
    print(kind, "batch vs single-world per world:", ["%.1e" % e for e in errs], flush=True)
    s.close()
