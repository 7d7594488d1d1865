"""World wrenches on the batched simulator (mw_apply_link_wrench,
Link::applyWorldWrench, Link.cpp:484-560): the humanoid (floating base, wave
kernel) in zero gravity, pushed at the base and at an arm with per-world
wrenches whose durations end inside a run (steps_per_run 3), against the same
model and wrenches on the scene kernel, whose world wrenches are checked
against v = F t / m in tests/test_gpu_scenario_scene.py.  The joint limits are
opened on both sides: the comparison isolates the wrench path from the two
kernels' exact LCP solves (equal only to their solve tolerance)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_sim_world_wrenches_match_the_scene(require_gpu):
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.scene import Scene
    from mwstep.sim import Simulator
    W, spr, runs = 8, 3, 15
    path = get_model_file("icub")
    text = open(path).read()
    pose = (0.0, 0.0, 1.0, 1.0, 0.0, 0.0, 0.0)
    sim = Simulator(path, n_worlds=W, steps_per_run=spr, pose=pose)
    sc = Scene(n_worlds=W, steps_per_run=spr)
    sc.insert_model(text, pose, "h")
    for s in (sim, sc):
        s.set_gravity([0.0, 0.0, 0.0])
    for d in range(sim.dofs):
        for which, v in ((N.PARAM_POSITION_LIMIT_MIN, -1e300), (N.PARAM_POSITION_LIMIT_MAX, 1e300)):
            sim.set_joint_param(d, which, v)
            sc.set_joint_param(d, which, v)
    sim.run(paused=True)
    sc.run(paused=True)
    sim.set_control_mode(N.MODE_FORCE)
    sc.set_control_mode(N.MODE_FORCE, m=0)
    assert sim.float_kernel() == 2  # the world-per-wavefront kernel
    names = sim.joint_names
    arm = next(i for i, n in enumerate(names) if "arm" in n or "elbow" in n)
    rng = np.random.default_rng(7)
    base_w = np.column_stack([rng.uniform(-60, 60, (W, 3)), rng.uniform(-3, 3, (W, 3))])
    arm_w = np.column_stack([rng.uniform(-5, 5, (W, 3)), rng.uniform(-0.2, 0.2, (W, 3))])
    for s in (sim, sc):
        args = (0,) if s is sc else ()
        s.apply_world_wrench(*args, -1, base_w, 0.010)      # 10 steps: ends inside run 4
        s.apply_world_wrench(*args, arm, arm_w, 0.0255)     # 26 steps: ends inside run 9
    sim.apply_world_wrench(-1, base_w, 0.010)                # same expiry: adds up (2x base wrench)
    sc.apply_world_wrench(0, -1, base_w, 0.010)
    worst = {}
    for r in range(runs):
        sim.run()
        sc.run()
        dqd = np.abs(sim.get("qd") - sc.get("qd", 0))
        e = {"q": np.abs(sim.get("q") - sc.get("q", 0)).max(),
             "qd": dqd.max(),
             "base": np.abs(sim.base_pose() - sc.base_pose(0)).max()}
        for k, v in e.items():
            worst[k] = max(worst.get(k, 0.0), float(v))
    moved = np.abs(sim.base_pose()[:, :3] - np.array(pose[:3])).max()
    print(f"humanoid x{W}, {runs} runs x {spr} steps with world wrenches: wave kernel vs scene kernel {worst}; "
          f"base moved {moved:.3f} m")
    assert moved > 1e-3
    assert worst["q"] <= 1e-6 and worst["qd"] <= 1e-5 and worst["base"] <= 1e-6
    # without wrenches the worlds coast: a wrench that expired does not act again
    v0 = sim.base_velocity().copy()
    sim.run()
    assert np.abs(sim.base_velocity() - v0).max() < 0.05
    with pytest.raises(RuntimeError):
        sim.apply_world_wrench(len(names), base_w, 0.01)     # link out of range
    sim.close()
    sc.close()
