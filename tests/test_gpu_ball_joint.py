"""Ball joints (core::JointType::Ball, Joint.cpp:318-331) on the GPU.

  * one step of a welded arm with a ball shoulder and a revolute elbow, 256
    worlds of random states and torques, on the scene kernel and through
    mw_sim, against the fp64 oracle of the same multibody (its independent
    SDF reader writes the spherical pair as three continuous URDF joints);
  * the ScenarI/O BallJoint through World / Model / Joint: a body held at its
    centre of mass by a ball joint, no gravity, spun up by reset_joint_velocity
    -- torque-free rotation against DART's discrete scheme restated in numpy
    beside it (BallJoint coordinates natively: w += dt w', R <- R exp(dt w);
    1e-5 over 0.5 s), and that scheme against the exact motion (RK4 of
    Euler's equations, dt / 10): orientation, body angular velocity and the
    world angular momentum."""

import math

import numpy as np
import pytest

from test_sdf_models import BALL_ARM_SDF

pytestmark = pytest.mark.gpu


def test_ball_arm_one_step(require_gpu, oracle):
    from mwstep import native as N
    from mwstep.scene import Scene
    from mwstep.sim import Simulator
    W = 256
    cm = oracle.load_urdf(BALL_ARM_SDF)
    n = cm.n
    assert n == 4 and not cm.floating
    rng = np.random.default_rng(5)
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    q = f32(np.column_stack([rng.uniform(-1.0, 1.0, (W, 3)), rng.uniform(-1.9, 1.9, W)]))
    qd = f32(rng.uniform(-2, 2, (W, n)))
    tau = f32(rng.uniform(-5, 5, (W, n)))
    mode = np.full(n, oracle.FORCE, np.int32)
    ref = [oracle.step(cm, 1e-3, q[w], qd[w], mode, tau[w], oracle.PGS_CONVERGED)[:2] for w in range(W)]

    def check(gq, gqd, what):
        wq = max(float(np.abs(gq[w] - ref[w][0]).max()) for w in range(W))
        wqd = max(float(np.abs(gqd[w] - ref[w][1]).max()) for w in range(W))
        print(f"ball arm, one step x{W}, {what}: max|dq| {wq:.2e}, max|dqd| {wqd:.2e}")
        assert wq <= 1e-5 and wqd <= 1e-4

    sc = Scene(n_worlds=W, pgs_iters=50)
    sc.insert_model(BALL_ARM_SDF, (0, 0, 0, 1, 0, 0, 0), "arm")
    assert sc.models[0]["dofs"] == n
    sc.set("reset_q", q, m=0)
    sc.set("reset_qd", qd, m=0)
    sc.run(paused=True)
    sc.set_control_mode(N.MODE_FORCE, m=0)
    sc.set("force_target", tau, m=0)
    sc.run()
    check(sc.get("q", 0), sc.get("qd", 0), "scene kernel")
    sc.close()
    sim = Simulator(BALL_ARM_SDF, n_worlds=W, pgs_iters=50)
    sim.set("reset_q", q)
    sim.set("reset_qd", qd)
    sim.run(paused=True)
    sim.set_control_mode(N.MODE_FORCE)
    sim.set("force_target", tau)
    sim.run()
    check(sim.get("q"), sim.get("qd"), f"mw_sim (kernel {sim.float_kernel()})")
    sim.close()


SPINNER_SDF = """<sdf version='1.7'><model name='spinner'>
  <link name='post'/>
  <joint name='fix' type='fixed'><parent>world</parent><child>post</child></joint>
  <link name='body'><pose>0 0 1 0 0 0</pose>
    <inertial><mass>3</mass>
      <inertia><ixx>0.05</ixx><iyy>0.12</iyy><izz>0.2</izz><ixy>0</ixy><ixz>0</ixz><iyz>0</iyz></inertia>
    </inertial></link>
  <joint name='pivot' type='ball'><parent>post</parent><child>body</child></joint>
</model></sdf>"""


def _torque_free(I, w0, T, dt):
    """R(t), w(t) (body frame) of a torque-free rigid body, RK4 on (R, w)"""
    Iinv = np.linalg.inv(I)
    sk = lambda v: np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])

    def f(R, w):
        return R @ sk(w), Iinv @ (-np.cross(w, I @ w))

    R, w = np.eye(3), np.array(w0, dtype=float)
    for _ in range(int(round(T / dt))):
        k1 = f(R, w)
        k2 = f(R + 0.5 * dt * k1[0], w + 0.5 * dt * k1[1])
        k3 = f(R + 0.5 * dt * k2[0], w + 0.5 * dt * k2[1])
        k4 = f(R + dt * k3[0], w + dt * k3[1])
        R = R + dt / 6 * (k1[0] + 2 * k2[0] + 2 * k3[0] + k4[0])
        w = w + dt / 6 * (k1[1] + 2 * k2[1] + 2 * k3[1] + k4[1])
        U, _, Vt = np.linalg.svd(R)
        R = U @ Vt
    return R, w


@pytest.mark.parametrize("r0", [[0.1, -0.2, 0.15], [0.0, math.pi / 2, 0.0]])
def test_scenario_ball_joint_torque_free_rotation(require_gpu, r0):
    """r0 = (0, pi/2, 0): the configuration where the round-3 X-Y-Z angle chart
    was singular -- DART's coordinates have no singularity."""
    from scenario import core
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gz.initialize()
    world = gz.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.set_gravity([0.0, 0.0, 0.0])
    assert world.insert_model_from_string(SPINNER_SDF, core.Pose([0, 0, 0], [1.0, 0, 0, 0]), "spinner")
    m = world.get_model("spinner")
    assert m.joint_names() == ["pivot"] and m.dofs() == 3
    assert "pivot#x" not in m.link_names() and "body" in m.link_names()
    j = m.get_joint("pivot")
    assert j.type() == core.JointType_ball and j.dofs() == 3
    assert j.set_control_mode(core.JointControlMode_force)
    assert not j.set_control_mode(core.JointControlMode_position)  # JointController skips ball joints
    w0 = [0.5, 0.4, 2.0]  # about the major axis, tilted: a stable precessing motion
    assert j.reset_joint_position(r0) and j.reset_joint_velocity(w0)
    gz.run(paused=True)
    assert np.allclose(j.joint_position(), r0, atol=1e-6)
    assert np.allclose(j.joint_velocity(), w0, atol=1e-5)
    I = np.diag([0.05, 0.12, 0.2])
    R0 = scenario.R_from_rotvec(r0)
    L0 = R0 @ I @ np.array(w0)
    T, dt = 0.5, 1e-3
    # DART's discrete scheme (BallJoint: ABA at the current w, w += dt w',
    # R <- R exp(dt w)), restated in numpy beside the GPU
    Rd, wd = R0.copy(), np.array(w0, dtype=float)
    worst_ang = worst_w = 0.0
    for _ in range(int(round(T / dt))):
        assert gz.run()
        wd = wd + dt * np.linalg.solve(I, -np.cross(wd, I @ wd))
        Rd = Rd @ scenario.R_from_rotvec(dt * wd)
        Rg = scenario.R_from_rotvec(j.joint_position())
        worst_ang = max(worst_ang, float(np.linalg.norm(scenario.rotvec_from_R(Rd.T @ Rg))))
        worst_w = max(worst_w, float(np.abs(np.array(j.joint_velocity()) - wd).max()))
    R, w = _torque_free(I, w0, T, 1e-4)
    Rg = scenario.R_from_rotvec(j.joint_position())
    wg = np.array(j.joint_velocity())
    ang = float(np.linalg.norm(scenario.rotvec_from_R((R0 @ R).T @ Rg)))
    Lg = Rg @ I @ wg
    E0, Eg = 0.5 * np.dot(w0, I @ w0), 0.5 * wg @ I @ wg
    print(f"torque-free spinner, {T} s: vs DART's discrete scheme orientation {worst_ang:.2e} rad, w {worst_w:.2e}; "
          f"vs the exact motion (RK4) orientation {ang:.2e} rad, |w - w_ref| {np.abs(wg - w).max():.2e}, "
          f"|L - L0| {np.abs(Lg - L0).max():.2e} (|L0| {np.linalg.norm(L0):.3f}), energy {Eg:.5f} vs {E0:.5f}")
    # the GPU's fp32 step against DART's scheme: round-off over 500 steps
    assert worst_ang <= 1e-5 and worst_w <= 1e-5
    # and the scheme itself against the exact motion: semi-implicit Euler, O(dt)
    assert abs(Eg - E0) <= 2e-3 * E0
    assert ang <= 5e-3 and np.abs(wg - w).max() <= 1e-2
    assert np.abs(Lg - L0).max() <= 5e-3 * np.linalg.norm(L0)
    # torques on the ball joint: child-frame torque about z spins the body up about z
    assert j.set_joint_generalized_force_target([0.0, 0.0, 0.4])
    assert np.allclose(j.joint_generalized_force_target(), [0.0, 0.0, 0.4], atol=1e-6)
    gz.close()
