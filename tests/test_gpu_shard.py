"""GPU tests of the world sharding and of the device-resident run.

  * a VecEnv of W worlds equals two VecEnvs of W/2 worlds with world_offset
    0 / W/2 (a rank's shard, and bench.py's world groups) BIT FOR BIT over 200
    closed-loop steps including TimeLimit / termination auto-resets, for the
    headline CartPole task (BASELINE configs[1]) and the Panda PID task
    (configs[3], the 1 -> 8 GPU strong split): resets are keyed by the global
    world index, so a world's trajectory does not depend on the rank count;
  * the same for floating bases with ground contacts (configs[4]'s humanoid
    split, on the wave kernel with cold and warm-started PGS, and the
    quadruped on the lane kernel): W worlds == two sims of W/2 worlds;
  * mw_run_device with a pending joint reset and a force command equals mw_run
    (the command slab is copied out of a staging buffer, so clearing the host
    mirror right after the asynchronous launch cannot drop it);
  * pending commands cannot be captured into a graph (loud error).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_split(task, W, T, max_steps, make_actions):
    import torch
    from mwstep.vecenv import VecEnv
    full = VecEnv(task, n_worlds=W, device=0, seed=7, max_episode_steps=max_steps)
    half = [VecEnv(task, n_worlds=W // 2, device=0, seed=7, world_offset=k * (W // 2),
                   max_episode_steps=max_steps) for k in range(2)]
    o_full = full.reset().clone()
    o_half = torch.cat([h.reset().clone() for h in half])
    assert torch.equal(o_full, o_half)
    n_done = 0
    for t in range(T):
        a = make_actions(t, o_full)
        o, r, d, info = full.step(a)
        parts = [h.step(a[k * (W // 2):(k + 1) * (W // 2)].contiguous()) for k, h in enumerate(half)]
        torch.cuda.synchronize()
        assert torch.equal(o, torch.cat([p[0] for p in parts])), t
        assert torch.equal(r, torch.cat([p[1] for p in parts])), t
        assert torch.equal(d, torch.cat([p[2] for p in parts])), t
        n_done += int(d.sum())
        o_full = o
    q, qd = full.state()
    qs = [h.state() for h in half]
    assert torch.equal(q, torch.cat([x[0] for x in qs], dim=1))
    assert torch.equal(qd, torch.cat([x[1] for x in qs], dim=1))
    for e in [full] + half:
        e.close()
    return n_done


def test_cartpole_shards_bit_identical(require_gpu):
    import torch
    gen = torch.Generator(device="cuda").manual_seed(43)
    acts = torch.randint(0, 2, (200, 4096), generator=gen, device="cuda", dtype=torch.int32)
    n_done = _run_split("CartPoleDiscreteBalancing", 4096, 200, 50, lambda t, o: acts[t].contiguous())
    assert n_done > 4096  # TimeLimit (50 steps) and pole-angle resets happened inside the window


def test_panda_shards_bit_identical(require_gpu):
    import torch
    T, W = 200, 1024
    state = {}

    def targets(t, obs):
        if "q0" not in state:
            state["q0"] = obs[:, :9].clone()
        tg = state["q0"].clone()
        s = float(np.sin(2 * np.pi * 0.33 * t * 1e-3))
        tg[:, 0] += 0.9 * 2.8973 * s
        tg[:, 5] += 0.9 * (3.7525 + 0.0175) / 2 * s
        return tg.contiguous()

    n_done = _run_split("PandaPositionTracking", W, T, 80, targets)
    assert n_done >= W  # every world hit the 80-step TimeLimit at least once
    del torch


def _float_sim(model, W, q0, pose, vel, pgs_opts, target=None):
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.sim import Simulator
    sim = Simulator(get_model_file(model), n_worlds=W, pgs_iters=50, pose=(0, 0, 0.6, 1, 0, 0, 0))
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    if pgs_opts is not None:
        sim.set_pgs_options(*pgs_opts)
    sim.set("reset_q", q0)
    sim.reset_base_pose(pose)
    sim.reset_base_velocity(vel)
    sim.run(paused=True)
    sim.set_controller_period(1e-3)
    for d in range(sim.dofs):
        sim.set_pid(d, [300.0, 0.0, 3.0, -80.0, 80.0, 0.0, 0.0, -1.0])
    sim.set_control_mode(N.MODE_POSITION)
    sim.set("position_target", np.zeros_like(q0) if target is None else np.tile(target, (W, 1)))
    return sim


@pytest.mark.parametrize("model,z0,pgs_opts", [("icub", 0.58, None),
                                               ("icub", 0.58, (1e-6, True)),
                                               ("quadruped", 0.47, None)])
def test_floating_shards_bit_identical(require_gpu, model, z0, pgs_opts):
    """BASELINE config 5 splits 512 humanoids over the ranks (bench.py
    humanoid_leg: the 8-GPU share is 64 worlds): a sim of W worlds equals two
    sims of W/2 worlds holding the two halves' initial states BIT FOR BIT over
    150 steps with ground impacts, sliding and (parametrised) the warm-started
    PGS, for the humanoid and the quadruped (world-per-wavefront kernel)."""
    W, T = 128, 150
    rng = np.random.default_rng(11)
    from mwstep import get_model_file
    from mwstep.sim import Simulator
    p = Simulator(get_model_file(model), n_worlds=1)
    n, names = p.dofs, list(p.joint_names)
    p.close()
    post = None
    if model == "icub":   # the reference wrapper's posture (icub.py:19-40) as the hold target
        from mwstep.models import icub_posture
        post = np.array(icub_posture(names))
    q0 = rng.uniform(-0.1, 0.1, (W, n)) + (0.0 if post is None else post)
    quat = rng.normal(size=(W, 4)) * np.array([1.0, 0.05, 0.05, 0.05])
    quat[:, 0] = np.abs(quat[:, 0]) + 1.0
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    pose = np.column_stack([rng.uniform(-5, 5, (W, 2)), z0 + rng.uniform(0.0, 0.08, W), quat])
    vel = np.column_stack([rng.uniform(-0.5, 0.5, (W, 2)), rng.uniform(-0.3, 0.0, W), rng.uniform(-0.5, 0.5, (W, 3))])
    full = _float_sim(model, W, q0, pose, vel, pgs_opts, post)
    h = W // 2
    halves = [_float_sim(model, h, q0[k * h:(k + 1) * h], pose[k * h:(k + 1) * h], vel[k * h:(k + 1) * h], pgs_opts,
                         post) for k in range(2)]
    for t in range(T):
        full.run()
        for s in halves:
            s.run()
        if t % 50 == 49 or t == T - 1:
            for what in ("q", "qd"):
                assert np.array_equal(full.get(what), np.concatenate([s.get(what) for s in halves])), (what, t)
            assert np.array_equal(full.base_pose(), np.concatenate([s.base_pose() for s in halves])), t
            assert np.array_equal(full.base_velocity(), np.concatenate([s.base_velocity() for s in halves])), t
    # the window holds impacts and contacts (not a trivially resting state)
    assert sum(len(full.contacts(w)) for w in range(0, W, 8)) > 0
    assert full.constraint_overflow() == 0
    for s in [full] + halves:
        s.close()


def test_contact_answer_independent_of_world_count(require_gpu):
    """with DART's exact LCP (the default) every floating
    model steps on one kernel whatever the world count -- round 3 switched the
    quadruped to the PGS lane kernel above 4096 worlds.  4096 and 8192
    quadrupeds from identical states (the first 4096 worlds of the larger run)
    step bit for bit alike through 200 steps of drops, slides and contacts."""
    from mwstep import get_model_file
    from mwstep.sim import Simulator
    rng = np.random.default_rng(5)
    W = 8192
    n = 8
    q0 = rng.uniform(-0.1, 0.1, (W, n)) + np.array([0.6, -1.2] * 4)
    quat = rng.normal(size=(W, 4)) * np.array([1.0, 0.05, 0.05, 0.05])
    quat[:, 0] = np.abs(quat[:, 0]) + 1.0
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    pose = np.column_stack([rng.uniform(-5, 5, (W, 2)), 0.45 + rng.uniform(0.0, 0.05, W), quat])
    vel = np.column_stack([rng.uniform(-0.5, 0.5, (W, 2)), rng.uniform(-0.3, 0.0, W), rng.uniform(-0.5, 0.5, (W, 3))])
    sims = [_float_sim("quadruped", w, q0[:w], pose[:w], vel[:w], None) for w in (4096, W)]
    for s in sims:
        assert s.float_kernel() == 2 and s.lcp_solver() == (True, 48)
    h, touching = 4096, 0
    for t in range(200):
        for s in sims:
            s.run()
        if t % 20 == 19:
            touching += sum(len(sims[0].contacts(w)) > 0 for w in range(0, h, 64))
    for what in ("q", "qd"):
        assert np.array_equal(sims[0].get(what), sims[1].get(what)[:h]), what
    assert np.array_equal(sims[0].base_pose(), sims[1].base_pose()[:h])
    assert np.array_equal(sims[0].base_velocity(), sims[1].base_velocity()[:h])
    assert touching > 0
    for s in sims:
        s.close()


@pytest.mark.parametrize("model", ["cartpole", "pendulum"])
def test_run_device_applies_pending_commands(require_gpu, model):
    """run_impl cleared the host command slab right after queueing
    its asynchronous H2D copy; a device-resident run could lose the force
    command and the reset."""
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.sim import Simulator
    W = 257
    sims = [Simulator(get_model_file(model), n_worlds=W) for _ in range(2)]
    rng = np.random.default_rng(3)
    q0 = rng.uniform(-0.3, 0.3, (W, sims[0].dofs))
    qd0 = rng.uniform(-1, 1, (W, sims[0].dofs))
    tau = rng.uniform(-5, 5, (W, sims[0].dofs))
    for s in sims:
        s.set_control_mode(N.MODE_FORCE)
        s.run(paused=True)
        s.set("reset_q", q0)
        s.set("reset_qd", qd0)
        s.set("force_target", tau)
    sims[0].run()
    sims[1].run_device(1)
    assert np.array_equal(sims[0].get("q"), sims[1].get("q"))
    assert np.array_equal(sims[0].get("qd"), sims[1].get("qd"))
    # the reset took effect (not the zero state) and the force acted
    assert np.abs(sims[1].get("q") - q0).max() < 0.01
    # a second round: new commands while the first copy may still be queued
    for s in sims:
        s.set("force_target", -tau)
    sims[0].run()
    sims[1].run_device(1)
    assert np.array_equal(sims[0].get("qd"), sims[1].get("qd"))
    for s in sims:
        s.close()


def test_pending_commands_refuse_graph_capture(require_gpu):
    import torch
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.sim import Simulator
    stream = torch.cuda.Stream()
    sim = Simulator(get_model_file("cartpole"), n_worlds=64, stream=stream.cuda_stream)
    sim.set_control_mode(N.MODE_FORCE)
    sim.run()
    sim.set("force_target", np.ones((64, 2)))
    graph = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="captured"):
        with torch.cuda.stream(stream):
            with torch.cuda.graph(graph, stream=stream):
                sim.run_device(1)
    sim.run_device(1)  # applied outside capture: fine
    with torch.cuda.stream(stream):
        stream.synchronize()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=stream):
            sim.run_device(2)
        g2.replay()
    stream.synchronize()
    sim.close()
