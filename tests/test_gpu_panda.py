"""GPU tests of the Panda row (BASELINE config 4): a branched 9-dof model in
Position (PID) control, on the HIP scenario kernel.

  * the reference's PID known-answer test, through the ScenarI/O mirror
    (tests/test_scenario/test_pid_controllers.py:34-115; gains :20-30,
    controller period = step size, hold 1000 steps within 1 deg, track
    q0 + 0.9 range/2 sin(2 pi 0.33 t) on joints 1 and 6 within 3 deg); joint 4
    starts at its published upper limit instead of 0 (see
    tests/test_oracle_tree_pid.py);
  * teacher-forced one-step parity against the fp64 oracle
    (pyoracle.ScenarioWorld: JointController PID + tree ABA + limit rows) over
    many worlds with random states / targets: fp32 vs fp64, <= 1e-5 rad on q
    and <= 1e-4 rad/s on qd (the north star's observation bound);
  * free-running parity of a PID tracking run (H = 500) against the oracle,
    <= 1e-4 rad (the joint positions are integrated compensated, q = q_hi +
    qlo, so the PID's d/dt gain does not amplify the float32 rounding of q);
  * controller-period gating and Velocity-mode PID against the oracle.
"""

import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GAINS = {  # test_pid_controllers.py:20-30
    "panda_joint1": (50, 0, 20), "panda_joint2": (10000, 0, 500),
    "panda_joint3": (100, 0, 10), "panda_joint4": (1000, 0, 50),
    "panda_joint5": (100, 0, 10), "panda_joint6": (100, 0, 10),
    "panda_joint7": (10, 0.5, 0.1), "panda_finger_joint1": (100, 0, 50),
    "panda_finger_joint2": (100, 0, 50),
}
BIG = float(np.finfo(np.float64).max)


def test_position_pid_kat(require_gpu):
    from mwstep import get_model_file
    from scenario import core
    from scenario import gazebo as scenario
    gazebo = scenario.GazeboSimulator(1.0 / 1000, 1.0, 1)
    assert gazebo.initialize()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("panda"))
    assert "panda" in world.model_names()
    panda = world.get_model("panda").to_gazebo()
    joint1 = panda.get_joint("panda_joint1").to_gazebo()
    joint1_range = abs(joint1.position_limit().max - joint1.position_limit().min)
    assert joint1.reset_position(joint1.position_limit().min + joint1_range / 2)
    joint6 = panda.get_joint("panda_joint6").to_gazebo()
    joint6_range = abs(joint6.position_limit().max - joint6.position_limit().min)
    assert joint6.reset_position(joint6.position_limit().min + joint6_range / 2)
    assert panda.get_joint("panda_joint4").reset_position(-0.0698)
    assert gazebo.run(paused=True)
    assert panda.set_controller_period(gazebo.step_size())
    assert set(panda.joint_names()) == set(GAINS)
    for name, g in GAINS.items():
        assert panda.get_joint(name).set_pid(pid=core.PID(*g))
    assert panda.set_joint_control_mode(core.JointControlMode_position)
    assert panda.joint_position_targets() == pytest.approx(panda.joint_positions())
    for _ in range(1000):
        assert gazebo.run()
    assert panda.joint_positions() == pytest.approx(panda.joint_position_targets(), abs=np.deg2rad(1))
    q01, q06 = joint1.position(), joint6.position()
    worst = 0.0
    for k in range(5000):
        t = k * gazebo.step_size()
        r1 = q01 + 0.9 * joint1_range / 2 * np.sin(2 * np.pi * 0.33 * t)
        r6 = q06 + 0.9 * joint6_range / 2 * np.sin(2 * np.pi * 0.33 * t)
        assert joint1.set_position_target(position=r1)
        assert joint6.set_position_target(position=r6)
        assert gazebo.run()
        worst = max(worst, abs(joint1.position() - r1), abs(joint6.position() - r6))
        assert joint1.position() == pytest.approx(r1, abs=np.deg2rad(3))
        assert joint6.position() == pytest.approx(r6, abs=np.deg2rad(3))
    print(f"panda tracking worst error {np.degrees(worst):.3f} deg")
    gazebo.close()


def test_panda_model_wrapper(require_gpu):
    """gym_ignition_environments.models.panda.Panda (models/panda.py:11-77):
    home configuration, gains on every joint; with the period set to the step
    size, a Position-mode hold settles near the home pose (the gains have no
    integral term on joints 4 and 6, so gravity leaves a steady-state offset:
    measured 1.3 deg)."""
    from gym_ignition_environments.models import panda as panda_model
    from scenario import core
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(1e-3, 1.0, 1)
    assert gz.initialize()
    world = gz.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    panda = panda_model.Panda(world=world)
    assert gz.run(paused=True)
    arm = [f"panda_joint{i}" for i in range(1, 8)]
    assert panda.joint_positions(arm) == pytest.approx(panda_model.Panda.HOME, abs=1e-6)
    for name, g in GAINS.items():
        pid = panda.get_joint(name).to_gazebo().pid()
        assert (pid.p, pid.i, pid.d) == pytest.approx(g)
    assert panda.controller_period() == pytest.approx(1000.0)
    assert panda.set_controller_period(gz.step_size())
    assert panda.set_joint_control_mode(core.JointControlMode_position)
    for _ in range(1000):
        assert gz.run()
    assert panda.joint_positions(arm) == pytest.approx(panda_model.Panda.HOME, abs=np.deg2rad(3))
    assert np.abs(panda.joint_velocities(arm)).max() < 1e-2
    gz.close()


def _sim(W, spr=1, period=1e-3):
    from mwstep import get_model_file
    from mwstep.sim import Simulator
    sim = Simulator(get_model_file("panda"), n_worlds=W, steps_per_run=spr, pgs_iters=20)
    for d, name in enumerate(sim.joint_names):
        p, i, dd = GAINS[name]
        sim.set_pid(d, [p, i, dd, -BIG, BIG, 0.0, -BIG, BIG])
    sim.set_controller_period(period)
    return sim


def _oracle_world(oracle, cm, q, qd, tgt, mode, period_ns=1_000_000, spr=1, vtgt=None):
    w = oracle.ScenarioWorld(cm, 1e-3, spr, 20)
    w.q, w.qd = q.astype(float).copy(), qd.astype(float).copy()
    w.period_ns = period_ns
    for d, name in enumerate(cm.joint_names):
        w.set_pid(d, *GAINS[name])
        w.set_mode(d, mode)
    w.ptgt[:] = tgt
    if vtgt is not None:
        w.vtgt[:] = vtgt
    return w


def _random_states(cm, W, rng):
    n = cm.n
    lo = np.array([cm.model.lower[i] for i in range(n)])
    hi = np.array([cm.model.upper[i] for i in range(n)])
    q = rng.uniform(lo, hi, size=(W, n))
    # some joints 1 mrad beyond a limit: exactly AT a limit, fp32 and fp64
    # may disagree on whether the limit row activates (a threshold case)
    at = rng.uniform(size=(W, n)) < 0.15
    q[at] = np.where(rng.uniform(size=(W, n)) < 0.5, lo - 1e-3, hi + 1e-3)[at]
    qd = rng.uniform(-0.5, 0.5, size=(W, n))
    tgt = np.clip(q + rng.uniform(-0.05, 0.05, size=(W, n)), lo, hi)
    return q.astype(np.float32), qd.astype(np.float32), tgt


def test_one_step_parity_position_pid(require_gpu, oracle, panda_file):
    W = 256
    rng = np.random.default_rng(3)
    cm = oracle.load_urdf(panda_file)
    q, qd, tgt = _random_states(cm, W, rng)
    sim = _sim(W)
    sim.set("reset_q", q)
    sim.set("reset_qd", qd)
    sim.run(paused=True)
    sim.set_control_mode(5)                       # Position: targets = current q, PID reset
    sim.set("position_target", tgt)
    sim.run()
    gq, gqd = sim.get("q"), sim.get("qd")
    wq = wqd = 0.0
    for w in range(W):
        ow = _oracle_world(oracle, cm, q[w], qd[w], tgt[w], oracle.POSITION)
        ow.run()
        wq = max(wq, float(np.abs(gq[w] - ow.q).max()))
        wqd = max(wqd, float(np.abs(gqd[w] - ow.qd).max()))
    print(f"panda one-step: max|dq| {wq:.2e}, max|dqd| {wqd:.2e}")
    assert wq <= 1e-5 and wqd <= 1e-4   # measured r01: 1.3e-7 / 4.2e-5
    sim.close()


def test_free_running_tracking_parity(require_gpu, oracle, panda_file):
    """8 worlds, 500 steps of sinusoidal targets on joints 1 and 6: the PID
    feedback keeps fp32 and fp64 trajectories within 1e-4 rad."""
    W, H = 8, 500
    cm = oracle.load_urdf(panda_file)
    n = cm.n
    q0 = np.zeros((W, n), np.float32)
    q0[:, 3] = -0.0698
    q0[:, 5] = 1.8675
    q0[:, 0] = np.linspace(-1, 1, W)
    sim = _sim(W)
    sim.set("reset_q", q0)
    sim.run(paused=True)
    sim.set_control_mode(5)
    ows = [_oracle_world(oracle, cm, q0[w], np.zeros(n), q0[w].astype(float), oracle.POSITION)
           for w in range(W)]
    worst = 0.0
    for k in range(H):
        t = k * 1e-3
        tgt = q0.astype(float).copy()
        tgt[:, 0] += 0.9 * 2.8973 * np.sin(2 * np.pi * 0.33 * t)
        tgt[:, 5] += 0.9 * 1.885 * np.sin(2 * np.pi * 0.33 * t)
        sim.set("position_target", tgt)
        sim.run()
        gq = sim.get("q")
        for w in range(W):
            ows[w].ptgt[:] = tgt[w]
            ows[w].run()
            worst = max(worst, float(np.abs(gq[w] - ows[w].q).max()))
    print(f"panda free-running H={H}: max|dq| {worst:.2e}")
    assert worst <= 1e-4   # measured r01: 4.1e-5
    sim.close()


def test_period_gating_and_velocity_pid(require_gpu, oracle, panda_file):
    """controller period = 3 steps with steps_per_run = 2 (the gate crosses run
    boundaries), Velocity-mode PID on every joint, vs the oracle."""
    W, H = 16, 60
    rng = np.random.default_rng(8)
    cm = oracle.load_urdf(panda_file)
    q, qd, _ = _random_states(cm, W, rng)
    vt = rng.uniform(-0.3, 0.3, size=(W, cm.n))
    sim = _sim(W, spr=2, period=3e-3)
    sim.set("reset_q", q)
    sim.set("reset_qd", qd)
    sim.run(paused=True)
    sim.set_control_mode(3)                       # Velocity
    sim.set("velocity_target", vt)
    ows = [_oracle_world(oracle, cm, q[w], qd[w], q[w], oracle.VELOCITY, period_ns=3_000_000,
                         spr=2, vtgt=vt[w]) for w in range(W)]
    worst = 0.0
    for _ in range(H):
        sim.run()
        gq = sim.get("q")
        for w in range(W):
            ows[w].run()
            worst = max(worst, float(np.abs(gq[w] - ows[w].q).max()))
    print(f"panda velocity PID, period 3 dt: max|dq| {worst:.2e}")
    assert worst <= 1e-4   # measured r01: 2.9e-6
    sim.close()


# --------------------------------------------------------------------------
# batched position-target env (BASELINE config 4 path): PandaPositionTracking
# --------------------------------------------------------------------------

def _unif32(x, lo, hi):
    t = np.float32((x >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0))
    return np.float32(lo) + (np.float32(hi) - np.float32(lo)) * t


def _panda_reset_ref(oracle, cm, seed, world, episode):
    """Restatement of the kernel's reset: the Panda wrapper's pose
    (models/panda.py:41-44) with joints 1 and 6 at mid-range
    (test_pid_controllers.py:49-59) and the fingers half open, + U(-0.05, 0.05)
    from Philox4x32-10 keyed by the seed, counter (world, episode, block, 0),
    clipped into the limits."""
    n = cm.n
    home = np.array([0.0, -0.785, 0.0, -2.356, 0.0, 1.571, 0.785, 0.0, 0.0])
    for d in (0, 5, 7, 8):
        home[d] = 0.5 * (cm.model.lower[d] + cm.model.upper[d])
    q = np.zeros(n, np.float32)
    for b in range((n + 3) // 4):
        r = oracle.philox_raw([world, episode, b, 0], [seed & 0xFFFFFFFF, seed >> 32])
        for k in range(4):
            d = 4 * b + k
            if d < n:
                x = np.float32(home[d]) + _unif32(np.array([r[k]], np.uint32), -0.05, 0.05)[0]
                q[d] = np.clip(x, np.float32(cm.model.lower[d]), np.float32(cm.model.upper[d]))
    return q


def test_panda_vecenv_reset(require_gpu, oracle, panda_file):
    from mwstep.vecenv import VecEnv
    W = 300
    env = VecEnv("PandaPositionTracking", n_worlds=W, seed=7)
    obs = env.reset().cpu().numpy()
    cm = oracle.load_urdf(panda_file)
    for w in range(0, W, 7):
        ref = _panda_reset_ref(oracle, cm, 7, w, 0)
        assert np.abs(obs[w, :9] - ref).max() <= 1e-6
        assert np.all(obs[w, 9:] == 0)
    env.close()


def test_panda_vecenv_vs_oracle(require_gpu, oracle, panda_file):
    """Free-running PandaPositionTracking vs per-world oracle ScenarioWorlds
    (same start state, PID gains, period = dt): obs within 1e-4, reward
    within 1e-5 relative; TimeLimit auto-reset at step 150."""
    import torch
    from mwstep.vecenv import VecEnv
    W, H, T_LIM = 32, 300, 150
    env = VecEnv("PandaPositionTracking", n_worlds=W, seed=3, max_episode_steps=T_LIM)
    cm = oracle.load_urdf(panda_file)
    # resets clip onto the limits exactly: give the oracle the kernel's float32
    # limits so that "at the limit" means the same thing to both
    for i in range(cm.n):
        cm.model.lower[i] = float(np.float32(cm.model.lower[i]))
        cm.model.upper[i] = float(np.float32(cm.model.upper[i]))
    obs0 = env.reset().cpu().numpy()
    ows = [_oracle_world(oracle, cm, obs0[w, :9], np.zeros(9), obs0[w, :9].astype(float), oracle.POSITION)
           for w in range(W)]
    phase = np.linspace(0, np.pi, W)
    worst_o = worst_r = 0.0
    for k in range(H):
        t = k * 1e-3
        tgt = obs0[:, :9].astype(np.float64).copy()
        tgt[:, 0] += 0.9 * 2.8973 * np.sin(2 * np.pi * 0.33 * t + phase)
        tgt[:, 5] += 0.9 * 1.885 * np.sin(2 * np.pi * 0.33 * t + phase)
        tgt = tgt.astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(tgt).cuda())
        o, r, d = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy().astype(bool)
        assert d.all() == ((k + 1) % T_LIM == 0) and d.any() == d.all()
        for w in range(W):
            ow = ows[w]
            ow.ptgt[:] = tgt[w]
            ow.run()
            ref_obs = np.concatenate([ow.q, ow.qd])
            ref_r = -float(np.sum((ow.q - tgt[w].astype(np.float64)) ** 2))
            if d[w]:
                term = info["terminal_obs"].cpu().numpy()[w]
                worst_o = max(worst_o, float(np.abs(term - ref_obs).max()))
                # restart the oracle world from the kernel's reset state
                ep = (k + 1) // T_LIM
                qr = _panda_reset_ref(oracle, cm, 3, w, ep)
                assert np.abs(o[w, :9] - qr).max() <= 1e-6 and np.all(o[w, 9:] == 0)
                ows[w] = _oracle_world(oracle, cm, o[w, :9], np.zeros(9), o[w, :9].astype(float),
                                       oracle.POSITION)
                ows[w].prev_ns = 0
            else:
                worst_o = max(worst_o, float(np.abs(o[w] - ref_obs).max()))
            worst_r = max(worst_r, abs(r[w] - ref_r) / (1.0 + abs(ref_r)))
    print(f"PandaPositionTracking vs oracle, H={H}: max|obs err| {worst_o:.2e}, reward rel err {worst_r:.2e}")
    # measured r01 1.5e-4 (joint 6 qd: the d/dt gain on the float32 rounding of
    # q); r02, compensated q: 2.9e-5
    assert worst_o <= 1e-4 and worst_r <= 1e-4
    env.close()


def test_panda_baked_matches_generic(require_gpu, monkeypatch):
    """The constant-folded Panda kernel against the generic one on the same
    inputs (rounding differs; the high-gain PID feedback carries it): obs within
    1e-4 after 300 tracking steps (measured r01: 1.5e-4, the same size as the
    fp32-vs-fp64 drift of test_panda_vecenv_vs_oracle)."""
    import torch
    from mwstep.vecenv import VecEnv
    W, H = 512, 300
    # the constant-folded kernels are the one-world-per-lane ones
    monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "lane")
    a = VecEnv("PandaPositionTracking", n_worlds=W, seed=4)
    b = VecEnv("PandaPositionTracking", n_worlds=W, seed=4)
    assert a.sim.baked_model() == 3
    q0 = a.reset()[:, :9].clone()
    b.reset()
    worst = 0.0
    for k in range(H):
        tgt = q0.clone()
        tgt[:, 0] += 0.9 * 2.8973 * math.sin(2 * math.pi * 0.33 * k * 1e-3)
        tgt[:, 5] += 0.9 * 1.885 * math.sin(2 * math.pi * 0.33 * k * 1e-3)
        monkeypatch.delenv("MWSTEP_DISABLE_BAKED", raising=False)
        oa = a.step(tgt)[0]
        monkeypatch.setenv("MWSTEP_DISABLE_BAKED", "1")
        ob = b.step(tgt)[0]
        worst = max(worst, float((oa - ob).abs().max()))
    monkeypatch.delenv("MWSTEP_DISABLE_BAKED", raising=False)
    print(f"panda baked vs generic, H={H}: max|obs diff| {worst:.2e}")
    assert worst <= 1e-4
    a.close()
    b.close()
