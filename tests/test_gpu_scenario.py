"""GPU tests of the ScenarI/O / gym_ignition mirror: the reference's scenario
tests restated on the HIP backend, plus trajectory parity with the oracle.

Reference tests mirrored:
  tests/test_scenario/test_velocity_direct.py:20-82
  tests/test_scenario/test_world.py:149-219 (time semantics)
  tests/test_scenario/test_model.py:69-110 (reset visible after a paused run),
                                    :264-302 (history of applied joint forces)
  tests/test_scenario/test_multi_world.py (independent worlds)
  tests/test_gym_ignition/test_reproducibility.py:24-67
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _world(step=1e-3, rtf=1.0, iters=1, physics=True):
    from mwstep import get_model_file
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(step, rtf, iters)
    assert gz.initialize()
    world = gz.get_world().to_gazebo()
    assert world.insert_model(get_model_file("ground_plane"))
    if physics:
        assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    return gz, world


def test_velocity_direct(require_gpu):
    from mwstep import get_model_file
    from scenario import core
    gz, world = _world()
    assert world.insert_model(get_model_file("pendulum"))
    pendulum = world.get_model("pendulum").to_gazebo()
    assert pendulum.get_joint("pivot").to_gazebo().set_coulomb_friction(value=0.01)
    assert pendulum.get_joint("pivot").to_gazebo().set_viscous_friction(value=0.2)
    pivot = pendulum.get_joint("pivot")
    assert pivot.to_gazebo().reset_position(position=np.deg2rad(90))
    for _ in range(5000):
        assert gz.run()
    assert np.deg2rad(179.7) <= pivot.position() <= np.deg2rad(180.3)
    assert pivot.set_control_mode(core.JointControlMode_velocity_follower_dart)
    assert pivot.set_velocity_target(np.pi)
    assert gz.run()
    assert pivot.velocity() == pytest.approx(np.pi)
    for _ in range(1500):
        gz.run()
    assert pivot.velocity() == pytest.approx(np.pi)
    assert pivot.set_velocity_target(-np.pi)
    assert gz.run()
    assert pivot.velocity() == pytest.approx(-np.pi)
    assert pivot.set_control_mode(core.JointControlMode_idle)
    for _ in range(5000):
        gz.run()
    assert 2 * np.pi + np.deg2rad(179.7) <= pivot.position() <= 2 * np.pi + np.deg2rad(180.3)
    # parameters are frozen once the model has been stepped (Joint.cpp:262-266)
    assert not pivot.set_coulomb_friction(0.5)
    gz.close()


@pytest.mark.parametrize("dt", [0.001, 1e-9])
def test_sim_time_starts_from_zero(require_gpu, dt):
    gz, world = _world(step=dt, physics=False)
    assert world.time() == 0
    assert world.set_physics_engine(0)
    gz.run(paused=True)
    assert world.time() == 0
    gz.run()
    assert world.time() == dt
    gz.run()
    assert world.time() == 2 * dt
    gz.run()
    assert world.time() == pytest.approx(3 * dt)
    gz.close()


def test_physics_inserted_late_catches_up(require_gpu):
    from mwstep import get_model_file
    gz, world = _world(physics=False)
    assert world.insert_model(get_model_file("pendulum"))
    for _ in range(10):
        gz.run()
    assert world.time() == 0
    assert world.get_model("pendulum").joint_positions() == [0.0]
    assert world.set_physics_engine(0)
    gz.run()
    assert world.time() == pytest.approx(11 * gz.step_size())
    gz.run(paused=True)
    assert world.time() == pytest.approx(11 * gz.step_size())
    gz.close()


def test_reset_visible_after_paused_run(require_gpu):
    from mwstep import get_model_file
    gz, world = _world()
    assert world.insert_model(get_model_file("cartpole"))
    model = world.get_model("cartpole")
    assert model.joint_names() == ["linear", "pivot"]
    assert model.joint_positions() == pytest.approx([0.0, 0.0])
    assert model.reset_joint_positions([0.05, 0.05])
    assert model.joint_positions() == pytest.approx([0.0, 0.0])
    gz.run(paused=True)
    assert model.joint_positions() == pytest.approx([0.05, 0.05])
    assert model.joint_velocities() == pytest.approx([0.0, 0.0])
    gz.run()
    assert model.joint_velocities() != pytest.approx([0.0, 0.0])
    assert model.reset_joint_velocities([-0.1, -0.1])
    gz.run(paused=True)
    assert model.joint_velocities() == pytest.approx([-0.1, -0.1])
    assert model.reset_joint_positions([-0.4], ["pivot"])
    gz.run(paused=True)
    assert model.joint_positions(["pivot"]) == pytest.approx([-0.4])
    gz.close()


def test_force_target_modes_and_consumption(require_gpu):
    from mwstep import get_model_file
    from scenario import core
    gz, world = _world()
    assert world.insert_model(get_model_file("cartpole"))
    model = world.get_model("cartpole")
    linear = model.get_joint("linear")
    assert not linear.set_generalized_force_target(10.0)      # Idle refuses (Joint.cpp:776-790)
    assert linear.set_control_mode(core.JointControlMode_force)
    assert linear.set_generalized_force_target(10.0)
    assert linear.generalized_force_target() == 10.0
    gz.run()
    assert linear.generalized_force_target() == 0.0            # zero-filled after the run
    assert not model.set_joint_generalized_force_targets([1.0, 1.0])  # pivot is Idle
    assert model.enable_history_of_applied_joint_forces(True, 3)
    hist = []
    for k in range(6):
        assert model.set_joint_generalized_force_targets([0.1 * (k + 1)], ["linear"])
        gz.run()
        hist += [0.1 * (k + 1), 0.0]      # the Idle pivot has no force command
        assert model.history_of_applied_joint_forces() == pytest.approx(hist[-6:])
    gz.close()


def test_cartpole_runtime_matches_oracle(require_gpu, oracle):
    """CartPoleDiscreteBalancing-Gazebo-v0 through gym.make + the randomizer
    (examples/python/launch_cartpole.py), stepped on the GPU; every episode is
    replayed on the oracle from the reset observation with the same actions."""
    import gym_ignition_environments  # noqa: F401 (registrations)
    from gym_ignition_environments import randomizers
    from mwstep import get_model_file, gym_module
    gym = gym_module()
    env = randomizers.cartpole_no_rand.CartpoleEnvNoRandomizations(
        env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))
    env.seed(42)
    cm = oracle.load_urdf(get_model_file("cartpole"))
    worst = 0.0
    steps = 0
    for _ in range(5):
        obs = env.reset()
        q = np.array([obs[0], obs[2]])
        qd = np.array([obs[1], obs[3]])
        done = False
        while not done:
            action = env.action_space.sample()
            obs, reward, done, _ = env.step(action)
            force = 20.0 if action == 1 else -20.0
            q, qd, *_ = oracle.step(cm, 1e-3, q, qd, [oracle.FORCE, oracle.PASSIVE], [force, 0.0])
            worst = max(worst, float(np.abs(obs - np.array([q[0], qd[0], q[1], qd[1]])).max()))
            steps += 1
            assert isinstance(reward, float)
    print(f"runtime vs oracle over {steps} steps: max|obs err| {worst:.3e}")
    assert worst <= 1e-3
    env.close()


def test_reproducibility(require_gpu):
    """tests/test_gym_ignition/test_reproducibility.py: same seed -> same rollouts."""
    import gym_ignition_environments  # noqa: F401
    from gym_ignition_environments import randomizers
    from mwstep import gym_module
    gym = gym_module()
    make = lambda: randomizers.cartpole_no_rand.CartpoleEnvNoRandomizations(
        env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))
    e1, e2 = make(), make()
    e1.seed(42)
    e2.seed(42)
    for _ in range(3):
        o1, o2 = e1.reset(), e2.reset()
        assert o1 == pytest.approx(o2)
        for _ in range(50):
            a = e1.action_space.sample()
            assert a == e2.action_space.sample()
            s1, s2 = e1.step(a), e2.step(a)
            assert s1[0] == pytest.approx(s2[0]) and s1[1] == s2[1] and s1[2] == s2[2]
            if s1[2]:
                break
    e1.close()
    e2.close()


def test_cartpole_env_randomizer(require_gpu):
    """randomizers/cartpole.py: every reset inserts a cartpole whose link
    masses are the nominal ones + max(U(-0.2, 0.2), 0) drawn from the task
    RNG; the same seed reproduces the same masses and rollouts."""
    import gym_ignition_environments  # noqa: F401
    from gym_ignition_environments import randomizers
    from mwstep import gym_module
    gym = gym_module()
    make = lambda: randomizers.cartpole.CartpoleEnvRandomizer(
        env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))

    def masses(env):
        task = env.env.task if hasattr(env.env, "task") else env.unwrapped.task
        model = task.world.get_model(task.model_name)
        n = model.dofs()
        return model._sim.export_model()[:34 * n].reshape(n, 34)[:, 17].copy()

    e1, e2 = make(), make()
    e1.seed(42)
    e2.seed(42)
    nominal = np.array([1.0, 0.1])  # cart, pole (models/cartpole.urdf)
    seen = []
    for _ in range(4):
        o1, o2 = e1.reset(), e2.reset()
        m1, m2 = masses(e1), masses(e2)
        assert np.array_equal(m1, m2)
        assert np.all(m1 >= nominal - 1e-12) and np.all(m1 <= nominal + 0.2 + 1e-12)
        seen.append(m1)
        assert o1 == pytest.approx(o2)
        for _ in range(30):
            a = e1.action_space.sample()
            assert a == e2.action_space.sample()
            s1, s2 = e1.step(a), e2.step(a)
            assert s1[0] == pytest.approx(s2[0]) and s1[2] == s2[2]
            if s1[2]:
                break
    assert len({tuple(m) for m in seen}) > 1
    e1.close()
    e2.close()


def test_joint_limit_matches_oracle(require_gpu, oracle):
    from mwstep import get_model_file
    from scenario import core
    gz, world = _world()
    assert world.insert_model(get_model_file("cartpole"))
    model = world.get_model("cartpole")
    assert model.set_joint_control_mode(core.JointControlMode_force, ["linear"])
    assert model.reset_joint_positions([4.7, 0.3])
    gz.run(paused=True)
    cm = oracle.load_urdf(get_model_file("cartpole"))
    q, qd = np.array(model.joint_positions()), np.array(model.joint_velocities())
    worst = 0.0
    for _ in range(600):
        assert model.set_joint_generalized_force_targets([300.0], ["linear"])
        gz.run()
        q, qd, *_ = oracle.step(cm, 1e-3, q, qd, [oracle.FORCE, oracle.PASSIVE], [300.0, 0.0], 20)
        worst = max(worst, float(np.abs(np.array(model.joint_positions()) - q).max()))
    assert model.joint_positions()[0] <= 4.85
    assert worst <= 2e-3
    gz.close()


def test_multi_world_independent(require_gpu):
    from mwstep import get_model_file
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gz.insert_worlds_from_sdf(
        '<sdf version="1.6"><world name="w1"></world><world name="w2"></world></sdf>')
    assert gz.initialize()
    assert gz.world_names() == ["w1", "w2"]
    for name, q0 in (("w1", 0.5), ("w2", -1.0)):
        w = gz.get_world(name)
        assert w.set_physics_engine(0)
        assert w.insert_model(get_model_file("pendulum"))
        assert w.get_model("pendulum").reset_joint_positions([q0])
    for _ in range(100):
        assert gz.run()
    q1 = gz.get_world("w1").get_model("pendulum").joint_positions()[0]
    q2 = gz.get_world("w2").get_model("pendulum").joint_positions()[0]
    assert q1 > 0.5 and q2 < -1.0
    gz.close()
