"""wave vs scene kernel world wrenches: variants of the test configuration (debug)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-ignition_amd", "python"))
import numpy as np
from mwstep import get_model_file
from mwstep import native as N
from mwstep.scene import Scene
from mwstep.sim import Simulator
path = get_model_file("humanoid32")
pose = (0.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0)


def run(W, spr, runs, dup, arm_on, scale):
    sim = Simulator(path, n_worlds=W, steps_per_run=spr, pose=pose)
    sc = Scene(n_worlds=W, steps_per_run=spr)
    sc.insert_model(open(path).read(), pose, "h")
    for s in (sim, sc):
        s.set_gravity([0.0, 0.0, 0.0])
    sim.run(paused=True); sc.run(paused=True)
    sim.set_control_mode(N.MODE_FORCE); sc.set_control_mode(N.MODE_FORCE, m=0)
    rng = np.random.default_rng(7)
    base_w = scale * np.column_stack([rng.uniform(-5, 5, (W, 3)), rng.uniform(-0.5, 0.5, (W, 3))])
    arm_w = scale * np.column_stack([rng.uniform(-2, 2, (W, 3)), rng.uniform(-0.1, 0.1, (W, 3))])
    for k in range(2 if dup else 1):
        sim.apply_world_wrench(-1, base_w, 0.010); sc.apply_world_wrench(0, -1, base_w, 0.010)
    if arm_on:
        sim.apply_world_wrench(6, arm_w, 0.0255); sc.apply_world_wrench(0, 6, arm_w, 0.0255)
    worst = 0.0
    first = None
    for r in range(runs):
        sim.run(); sc.run()
        d = float(np.abs(sim.get("qd") - sc.get("qd", 0)).max())
        if d > 1e-6 and first is None:
            first = r
        worst = max(worst, d)
    print(f"W {W} spr {spr} dup {dup} arm {arm_on} scale {scale}: worst qd diff {worst:.2e}, first > 1e-6 at run {first}",
          flush=True)
    sim.close(); sc.close()


for args in [(8, 3, 15, True, True, 1), (8, 1, 45, True, True, 1), (8, 3, 15, False, True, 1), (8, 3, 15, True, False, 1),
             (2, 1, 45, False, True, 1), (8, 1, 45, False, False, 1)]:
    run(*args)
