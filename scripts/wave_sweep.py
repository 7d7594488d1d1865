"""Time the one-world-per-wavefront kernel (wave_tree.hpp) on BASELINE
config 5's workload (the iCub-class model standing under PID hold) for several world
counts and PGS iteration counts; the PGS cost per sweep is the slope.
    python scripts/wave_sweep.py [model] [W ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402

from mwstep import get_model_file  # noqa: E402
from mwstep import native as N  # noqa: E402
from mwstep.sim import Simulator  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "icub"
Ws = [int(a) for a in sys.argv[2:]] or [64, 512]
from mwstep.models import ICUB_POSE, icub_posture  # noqa: E402
pose0 = {"icub": ICUB_POSE, "quadruped": (0, 0, 0.45, 1, 0, 0, 0)}[model]
T = 40
for W in Ws:
    for pgs in (0, 10, 50):
        sim = Simulator(get_model_file(model), n_worlds=W, pgs_iters=pgs, pose=pose0)
        names = sim.joint_names
        sim.set_ground_plane(True, 1.0)
        sim.enable_contacts(True)
        sim.set_controller_period(1e-3)
        for d, n in enumerate(names):
            stiff = any(k in n for k in ("hip", "knee", "ankle", "torso")) or model == "quadruped"
            p, dd = (500.0, 5.0) if stiff else (50.0, 0.5)
            sim.set_pid(d, [p, 0.0, dd, -80.0, 80.0, 0.0, 0.0, -1.0])
        sim.set_control_mode(N.MODE_POSITION)
        q0 = np.tile([0.6, -1.2] * 4 if model == "quadruped" else icub_posture(names), (W, 1))
        sim.set("reset_q", q0)
        sim.set("position_target", q0)
        sim.run(paused=True)
        sim.run_device(20)
        sim.get("q")
        t0 = time.perf_counter()
        sim.run_device(T)
        sim.get("q")
        dt = (time.perf_counter() - t0) / T
        print(f"{model} W={W:5d} pgs={pgs:3d}: {dt * 1e6:9.1f} us/step  {W / dt:12.0f} env-steps/s  "
              f"contacts(w0)={len(sim.contacts(0))}", flush=True)
        sim.close()
