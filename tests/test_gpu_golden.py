"""The HIP kernels against the committed golden fixtures (tests/golden/,
fp64 oracle outputs with their inputs; see make_golden.py) -- a parity check
that does not need the oracle at run time.

  * CartPoleDiscreteBalancing / PendulumSwingUp, 16 worlds x 300 env steps of
    the batched env (device Philox resets, stored actions): free-running
    observations within 1e-4 of the fp64 fixture while the done flags agree,
    rewards within 1e-4, done-flag mismatches (fp32 vs fp64 at a threshold)
    at most 0.5 % of the world-steps;
  * the iCub-class humanoid standing under the PID hold (wave kernel, PGS 50):
    joint positions within 1e-3 rad and base position within 1e-4 m every 10
    steps for 300 steps, foot contact forces within 0.5 N in total.
"""

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("task, name", [("CartPoleDiscreteBalancing", "cartpole_discrete"),
                                        ("PendulumSwingUp", "pendulum_swingup")])
def test_vecenv_matches_golden(require_gpu, task, name):
    import torch
    from mwstep.vecenv import VecEnv
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    T, W = g["actions"].shape
    env = VecEnv(task, n_worlds=W, device=0, seed=42)
    o0 = env.reset().cpu().numpy()
    assert np.abs(o0 - g["obs0"]).max() <= 1e-6
    dtype = torch.int32 if g["actions"].dtype.kind == "i" else torch.float32
    alive = np.ones(W, bool)     # worlds whose done history still agrees
    worst, mism = 0.0, 0
    for t in range(T):
        o, r, d, _ = env.step(torch.as_tensor(g["actions"][t], dtype=dtype).cuda())
        o, r, d = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy().astype(bool)
        mism += int(((d != g["done"][t]) & alive).sum())
        alive &= d == g["done"][t]
        if alive.any():
            worst = max(worst, float(np.abs(o[alive] - g["obs"][t][alive]).max()))
            assert np.abs(r[alive] - g["reward"][t][alive]).max() <= 1e-4
    env.close()
    print(f"{task} vs golden: free-running max|obs err| {worst:.2e} over {T} steps, done mismatches {mism}")
    assert worst <= 1e-4
    assert mism <= 0.005 * T * W


def test_humanoid_matches_golden(require_gpu):
    """BASELINE config 5's model as the reference wrapper inserts it
    (icub_stand.npz: models/icub.urdf, the wrapper's posture and pose) under
    the posture hold, free-running 600 steps against the fp64 fixture."""
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    from mwstep.sim import Simulator
    g = np.load(os.path.join(GOLDEN, "icub_stand.npz"))
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    sim = Simulator(get_model_file("icub"), n_worlds=4, pgs_iters=50, pose=ICUB_POSE)
    assert list(sim.joint_names) == [str(s) for s in g["joint_names"]]
    q0 = np.tile(icub_posture(sim.joint_names), (4, 1))
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    sim.set("reset_q", q0)
    sim.set_controller_period(1e-3)
    for d, (p, dd) in enumerate(icub_pid_gains(sim.joint_names)):
        sim.set_pid(d, [p, 0.0, dd, -80.0, 80.0, 0.0, 0.0, -1.0])
    sim.set_control_mode(N.MODE_POSITION)
    sim.set("position_target", q0)
    wq = wp = 0.0
    for k in range(make_golden.HUMANOID_STEPS):
        sim.run()
        if k % make_golden.HUMANOID_EVERY == make_golden.HUMANOID_EVERY - 1:
            i = k // make_golden.HUMANOID_EVERY
            wq = max(wq, float(np.abs(sim.get("q") - g["q"][i]).max()))
            wp = max(wp, float(np.abs(sim.base_pose()[:, :3] - g["p"][i]).max()))
    fz = [sum(r[8] for r in sim.contacts(w)) for w in range(4)]
    sim.close()
    print(f"icub vs golden: max|dq| {wq:.2e}, max|dp| {wp:.2e}, sum Fz {fz} vs {g['contact_fz'].sum():.3f}")
    assert wq <= 1e-4 and wp <= 1e-5
    for f in fz:
        assert f == pytest.approx(float(g["contact_fz"].sum()), abs=0.5)
