"""wave vs scene kernel for the free-floating humanoid without wrenches (the
control of tests/test_gpu_sim_wrench.py)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-ignition_amd", "python"))
import numpy as np
from mwstep import get_model_file
from mwstep import native as N
from mwstep.scene import Scene
from mwstep.sim import Simulator
W, spr = 8, 3
path = get_model_file("humanoid32")
pose = (0.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0)
sim = Simulator(path, n_worlds=W, steps_per_run=spr, pose=pose)
sc = Scene(n_worlds=W, steps_per_run=spr)
sc.insert_model(open(path).read(), pose, "h")
for s in (sim, sc):
    s.set_gravity([0.0, 0.0, 0.0])
sim.run(paused=True); sc.run(paused=True)
sim.set_control_mode(N.MODE_FORCE); sc.set_control_mode(N.MODE_FORCE, m=0)
for r in range(15):
    sim.run(); sc.run()
    print(r, np.abs(sim.get("qd") - sc.get("qd", 0)).max(), np.abs(sim.get("q") - sc.get("q", 0)).max())
