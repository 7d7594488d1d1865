"""Time the world-per-wavefront kernel on BASELINE config 5's workload
(humanoid32 standing under the PID hold; first 40 steps dropped from up to
3 cm so impacts are included) for solver configurations: PGS sweeps, warm
start, exact LCP; prints us/step and the exact solve's unconverged count.
    python scripts/wave_lcp_sweep.py [W ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402

from mwstep import get_model_file  # noqa: E402
from mwstep import native as N  # noqa: E402
from mwstep.sim import Simulator  # noqa: E402

Ws = [int(a) for a in sys.argv[1:]] or [64, 512]
z0, T = 0.535, 40
CONFIGS = [  # (pgs sweeps, warm start, exact)
    (50, False, False), (50, False, True), (20, False, True), (10, False, True),
    (10, True, True), (5, True, True), (2, True, True), (1, True, True)]
for W in Ws:
    for pgs, warm, exact in CONFIGS:
        sim = Simulator(get_model_file("humanoid32"), n_worlds=W, pgs_iters=pgs, pose=(0, 0, z0, 1, 0, 0, 0))
        names = sim.joint_names
        sim.set_ground_plane(True, 1.0)
        sim.enable_contacts(True)
        sim.set_controller_period(1e-3)
        for d, n in enumerate(names):
            p, dd = (500.0, 5.0) if ("leg" in n or "torso" in n) else (50.0, 0.5)
            sim.set_pid(d, [p, 0.0, dd, -80.0, 80.0, 0.0, 0.0, -1.0])
        sim.set_control_mode(N.MODE_POSITION)
        sim.set_lcp_solver(exact)
        if warm:
            sim.set_pgs_options(0.0, True)
        rng = np.random.default_rng(0)
        pose = np.column_stack([np.zeros((W, 2)), z0 + rng.uniform(0, 0.03, W), np.ones(W), np.zeros((W, 3))])
        sim.reset_base_pose(pose)
        sim.set("position_target", np.zeros((W, sim.dofs)))
        sim.run(paused=True)
        u0 = sim.lcp_unconverged()
        sim.run_device(T)   # drops and impacts
        sim.get("q")
        t0 = time.perf_counter()
        sim.run_device(T)   # settling / standing
        sim.get("q")
        dt = (time.perf_counter() - t0) / T
        print(f"humanoid32 W={W:4d} pgs={pgs:3d} warm={int(warm)} exact={int(exact)}: {dt * 1e6:8.1f} us/step "
              f"{W / dt:11.0f} env-steps/s  unconverged {sim.lcp_unconverged() - u0}/{2 * T * W}  "
              f"contacts(w0)={len(sim.contacts(0))} overflow={sim.constraint_overflow()}", flush=True)
        sim.close()
