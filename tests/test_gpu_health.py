"""Failure detection and per-world snapshots.

  * divergence: the run kernels flag a world whose stored state is not finite
    (exponent-bit test; the kernels are finite-math-only builds).  A NaN
    injected into one world's joint velocity is flagged in that world only,
    mw_run reports it once (MW_EDIVERGED -> DivergedError), the other worlds
    step exactly as in a twin simulator without the injection, and a world
    re-armed after its reset runs clean -- on the world-per-wavefront kernel
    (humanoid), the chain kernel (Panda) and the scene kernel (ScenarI/O
    run() returns False, as the reference's failed server step does,
    GazeboSimulator.cpp:243-248);
  * snapshots: mw_get_state -> k steps -> mw_set_state -> the same k steps
    reproduces the first pass bit for bit (joint state, PID integrators, base
    pose / twist, and the exact LCP's warm-start impulses), also for a
    restored sub-range of the worlds.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
def _humanoid(W, drop=0.0):
    """BASELINE config 5's model as the reference wrapper inserts it
    (icub.py:19-40, :86), holding its posture (+ per-world offsets)."""
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    from mwstep.sim import Simulator
    pose = (*ICUB_POSE[:2], ICUB_POSE[2] + drop, *ICUB_POSE[3:])
    sim = Simulator(get_model_file("icub"), n_worlds=W, pgs_iters=50, pose=pose)
    assert sim.float_kernel() == 2
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    post = np.array(icub_posture(sim.joint_names))
    sim.set("reset_q", np.tile(post, (W, 1)))
    sim.set_controller_period(1e-3)
    for d, (p, dd) in enumerate(icub_pid_gains(sim.joint_names)):
        sim.set_pid(d, [p, 0.0, dd, -80.0, 80.0, 0.0, 0.0, -1.0])
    sim.set_control_mode(N.MODE_POSITION)
    rng = np.random.default_rng(3)
    sim.set("position_target", post + rng.uniform(-0.1, 0.1, (W, sim.dofs)))
    return sim


def _panda(W):
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.sim import Simulator
    sim = Simulator(get_model_file("panda"), n_worlds=W)
    sim.set_controller_period(1e-3)
    for d in range(sim.dofs):
        sim.set_pid(d, [600.0, 10.0, 30.0, -80.0, 80.0, 0.0, -5.0, 5.0])
    sim.set_control_mode(N.MODE_POSITION)
    rng = np.random.default_rng(4)
    sim.set("position_target", rng.uniform(-0.5, 0.5, (W, sim.dofs)))
    return sim


def _snap(sim):
    out = [sim.get("q"), sim.get("qd")]
    try:
        out += [sim.base_pose(), sim.base_velocity()]
    except RuntimeError:
        pass
    return out


@pytest.mark.parametrize("model", ["humanoid", "panda"])
def test_nan_world_is_flagged(require_gpu, model):
    from mwstep import native as N
    make = _humanoid if model == "humanoid" else _panda
    W, bad = 8, 3
    sims = [make(W), make(W)]
    for s in sims:
        for _ in range(5):
            s.run()
    qd = sims[0].get("qd")
    qd[bad, 1] = np.nan
    sims[0].set("reset_qd", qd)
    sims[1].set("reset_qd", sims[1].get("qd"))
    with pytest.raises(N.DivergedError):
        sims[0].run()
    sims[1].run()
    flags, count = sims[0].diverged()
    assert count == 1 and flags.tolist() == [w == bad for w in range(W)]
    for _ in range(3):          # reported once: the flag is sticky, not new
        sims[0].run()
        sims[1].run()
    good = [w for w in range(W) if w != bad]
    for a, b in zip(_snap(sims[0]), _snap(sims[1])):
        assert np.array_equal(a[good], b[good])   # the other worlds never notice
    # the caller resets the world: the reset re-arms its flag,
    # it runs clean again ...
    q, qd = sims[1].get("q"), sims[1].get("qd")
    sims[0].set("reset_q", q)
    sims[0].set("reset_qd", qd)
    if model == "humanoid":
        sims[0].reset_base_pose(sims[1].base_pose())
        sims[0].reset_base_velocity(sims[1].base_velocity())
    sims[0].run()
    assert sims[0].diverged()[1] == 1 and not sims[0].diverged()[0].any()
    assert np.isfinite(sims[0].get("qd")).all()
    # ... and a second divergence of the same world is reported again
    qd = sims[0].get("qd")
    qd[bad, 0] = np.inf
    sims[0].set("reset_qd", qd)
    with pytest.raises(N.DivergedError):
        sims[0].run()
    flags, count = sims[0].diverged()
    assert count == 2 and flags.tolist() == [w == bad for w in range(W)]
    # an explicit re-arm without a reset: the world is flagged again at once
    sims[0].clear_diverged(bad, 1)
    with pytest.raises(N.DivergedError):
        sims[0].run()
    assert sims[0].diverged()[1] == 3
    for s in sims:
        s.close()


def test_scenario_run_reports_divergence(require_gpu):
    """The ScenarI/O mirror (scene kernel): a world whose state goes
    non-finite makes run() return False once; the other world keeps stepping."""
    from scenario import gazebo as scenario
    from mwstep import get_model_file
    gz = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gz.insert_worlds_from_sdf('<sdf version="1.6"><world name="a"></world><world name="b"></world></sdf>')
    assert gz.initialize()
    models = []
    for n in ("a", "b"):
        w = gz.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(get_model_file("pendulum"))
        models.append(w.get_model("pendulum"))
    assert models[0].reset_joint_positions([0.3]) and models[1].reset_joint_positions([0.3])
    assert gz.run()
    assert models[0].reset_joint_velocities([float("nan")])
    assert not gz.run()           # the failed step is reported
    assert gz.run()               # once
    assert np.isfinite(models[1].joint_positions()[0])
    flags, count = gz._scene.diverged()
    assert count == 1 and flags.tolist() == [True, False]
    # a reset re-arms the world: it steps clean, and a second
    # divergence after the reset is reported again
    assert models[0].reset_joint_positions([0.3]) and models[0].reset_joint_velocities([0.0])
    assert gz.run()
    assert np.isfinite(models[0].joint_positions()[0])
    assert gz._scene.diverged()[0].tolist() == [False, False]
    assert models[0].reset_joint_velocities([float("inf")])
    assert not gz.run()
    assert gz.run()
    flags, count = gz._scene.diverged()
    assert count == 2 and flags.tolist() == [True, False]
    # removing the model and inserting it again re-arms the world too
    w0 = gz.get_world("a")
    assert w0.remove_model("pendulum")
    assert gz.run()
    assert gz._scene.diverged()[0].tolist() == [False, False]
    assert w0.insert_model(get_model_file("pendulum"))
    assert gz.run()
    gz.close()


@pytest.mark.parametrize("model", ["humanoid", "panda"])
def test_state_snapshot_round_trip(require_gpu, model):
    W = 16
    sim = _humanoid(W, drop=0.01) if model == "humanoid" else _panda(W)
    for _ in range(60):         # the humanoids land (~45 ms): contacts, warm-started exact LCP
        sim.run()
    rec = sim.get_state()
    assert rec.dtype == np.float32 and rec.shape[0] == W
    for _ in range(20):
        sim.run()
    first = _snap(sim)
    if model == "humanoid":
        c_first = [sim.contacts(w) for w in range(0, W, 5)]
    sim.set_state(rec)
    assert np.array_equal(sim.get_state(), rec)
    for _ in range(20):
        sim.run()
    for a, b in zip(first, _snap(sim)):
        assert np.array_equal(a, b)
    if model == "humanoid":
        for w, c in zip(range(0, W, 5), c_first):
            assert np.array_equal(sim.contacts(w), c)
        assert len(c_first[0]) > 0
    # a sub-range: worlds 4..7 go back 20 steps, the others run on
    mid = sim.get_state()
    sim.set_state(rec[4:8], w0=4)
    for _ in range(20):
        sim.run()
    st = sim.get_state()
    assert np.array_equal(st[4:8], mid[4:8])
    sim.close()
