"""The reference's link-kinematics KATs on the HIP backend, through the
ScenarI/O mirror (tests/test_scenario/test_link_velocities.py):

  * linear velocity (:85-139): (p_new - p_old) / dt equals the reported world
    linear velocity of the link origin within 1e-2 after every run (the
    semi-implicit Euler signature), and the body velocity is W_R_L^T of it;
  * angular velocity (:142-195): vee(skew(dR/dt R^T)) equals the reported
    world angular velocity within 5e-3, vee(skew(R^T dR/dt)) the body one;
  * linear / angular acceleration (:198-318, Panda only, as in the reference):
    the finite difference of the world velocities equals the reported
    acceleration within 0.5 / 0.2, skipping the steps the reference skips
    (any component above 100).

Models: the Panda (random joint positions from its limits, seed 10, and
joint velocities U(-1, 1), falling under gravity in Force mode with zero
torques) and the reference's 5 kg cube rotated 45 deg about x at z = 0.5 with
base velocity (0.1, -0.2, -0.3) / (-0.1, 2.0, 0.3), dropped on the ground
plane.  dt = 1e-4 as in the reference; 0.2 s of simulation instead of 0.5 s
(2,000 runs per case) to bound the test time.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = 1e-4
STEPS = 2000


def _quat_to_R(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _world():
    from mwstep import get_model_file
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(DT, 1.0, 1)
    assert gz.initialize()
    world = gz.get_world().to_gazebo()
    assert world.insert_model(get_model_file("ground_plane"))
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    return gz, world


def _random_panda(gz, world):
    from mwstep import get_model_file
    assert world.insert_model(get_model_file("panda"))
    panda = world.get_model("panda").to_gazebo()
    rng = np.random.default_rng(10)
    lims = [panda.get_joint(n).position_limit() for n in panda.joint_names()]
    q = np.array([rng.uniform(lim.min, lim.max) for lim in lims])
    dq = rng.uniform(-1.0, 1.0, size=q.shape)
    assert panda.reset_joint_positions(q.tolist())
    assert panda.reset_joint_velocities(dq.tolist())
    assert gz.run(paused=True)
    return panda


def _cube(gz, world):
    from mwstep import get_model_file
    from scenario import core
    s = np.sin(np.pi / 8)
    assert world.insert_model(get_model_file("cube"), core.Pose([0, 0, 0.5], [np.cos(np.pi / 8), s, 0, 0]))
    cube = world.get_model("cube_robot").to_gazebo()
    assert cube.reset_base_world_linear_velocity([0.1, -0.2, -0.3])
    assert cube.reset_base_world_angular_velocity([-0.1, 2.0, 0.3])
    assert gz.run(paused=True)
    return cube


def _accessors(model, link_name):
    link = model.get_link(link_name)
    if link.name() != model.base_frame():
        return link.position, link.orientation, link
    return model.base_position, model.base_orientation, None


@pytest.mark.parametrize("make, link_name", [(_random_panda, "panda_link7"), (_cube, "cube")])
def test_linear_velocity(require_gpu, make, link_name):
    gz, world = _world()
    model = make(gz, world)
    position, orientation, link = _accessors(model, link_name)
    world_lin = link.world_linear_velocity if link else model.base_world_linear_velocity
    body_lin = link.body_linear_velocity if link else model.base_body_linear_velocity
    worst = 0.0
    for _ in range(STEPS):
        p_old = np.array(position())
        assert gz.run()
        p_new = np.array(position())
        v_fd = (p_new - p_old) / DT
        v = np.array(world_lin())
        worst = max(worst, float(np.abs(v_fd - v).max()))
        assert v_fd == pytest.approx(v, abs=1e-2)
        assert _quat_to_R(orientation()).T @ v == pytest.approx(body_lin(), abs=1e-9)
    print(f"{link_name}: max |dp/dt - v| {worst:.2e}")
    gz.close()


@pytest.mark.parametrize("make, link_name", [(_random_panda, "panda_link7"), (_cube, "cube")])
def test_angular_velocity(require_gpu, make, link_name):
    gz, world = _world()
    model = make(gz, world)
    _, orientation, link = _accessors(model, link_name)
    world_ang = link.world_angular_velocity if link else model.base_world_angular_velocity
    body_ang = link.body_angular_velocity if link else model.base_body_angular_velocity
    skew = lambda m: (m - m.T) / 2
    vee = lambda m: np.array([m[2, 1], m[0, 2], m[1, 0]])
    worst = 0.0
    for _ in range(STEPS):
        R_old = _quat_to_R(orientation())
        assert gz.run()
        R_new = _quat_to_R(orientation())
        dR = (R_new - R_old) / DT
        w_fd = vee(skew(dR @ R_new.T))
        worst = max(worst, float(np.abs(w_fd - np.array(world_ang())).max()))
        assert w_fd == pytest.approx(world_ang(), abs=5e-3)
        assert vee(skew(R_new.T @ dR)) == pytest.approx(body_ang(), abs=5e-3)
    print(f"{link_name}: max |vee(dR R^T) - w| {worst:.2e}")
    gz.close()


def test_linear_acceleration(require_gpu):
    gz, world = _world()
    model = _random_panda(gz, world)
    link = model.get_link("panda_link7")
    checked = 0
    for _ in range(STEPS):
        v_old = np.array(link.world_linear_velocity())
        assert gz.run()
        a_fd = (np.array(link.world_linear_velocity()) - v_old) / DT
        a = np.array(link.world_linear_acceleration())
        if (a > 100.0).any():
            continue
        checked += 1
        assert a == pytest.approx(a_fd, abs=0.5)
        assert _quat_to_R(link.orientation()).T @ a == pytest.approx(link.body_linear_acceleration(), abs=1e-9)
    assert checked > STEPS // 2
    gz.close()


def test_angular_acceleration(require_gpu):
    gz, world = _world()
    model = _random_panda(gz, world)
    link = model.get_link("panda_link7")
    checked = 0
    for _ in range(STEPS):
        w_old = np.array(link.world_angular_velocity())
        assert gz.run()
        al_fd = (np.array(link.world_angular_velocity()) - w_old) / DT
        al = np.array(link.world_angular_acceleration())
        if (al > 100.0).any():
            continue
        checked += 1
        assert al_fd == pytest.approx(al, abs=0.2)
        assert _quat_to_R(link.orientation()).T @ al == pytest.approx(link.body_angular_acceleration(), abs=1e-9)
    assert checked > STEPS // 2
    gz.close()
