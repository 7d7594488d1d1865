"""DART's BallJoint coordinates, host side (no GPU): the oracle's restatement
(oracle.c ball_part / joint_bias / ball_integrate) and the ScenarI/O helpers.

A ball joint (core::JointType::Ball, Joint.cpp:267-331) runs natively in
DART's coordinates: positions = the rotation vector of the joint rotation,
velocities = the child's angular velocity in the child frame, integrated as
R <- R exp(dt w) after DART's semi-implicit velocity update [EXT:
dart/dynamics/BallJoint.cpp].  Checked here:

  * the exponential / log maps invert each other (scenario.gazebo helpers);
  * a body held at its centre of mass by a ball joint, no gravity, stepped by
    the fp64 oracle, equals a numpy restatement of DART's discrete scheme
    (w' = I^-1 (tau - w x I w) at the current w, w += dt w', R <- R exp(dt w))
    to round-off over 500 steps -- which pins the joint's velocity-product term
    (the three-part listing must add no Euler-angle Coriolis terms) and the
    SO(3) position update, with the rotation vector's angle kept in [0, pi];
  * with joint damping, DART's implicit damping: (I + dt D) w' = -D w - w x I w.
"""

import math

import numpy as np
import pytest

SPINNER_SDF = """<sdf version='1.7'><model name='spinner'>
  <link name='post'/>
  <joint name='fix' type='fixed'><parent>world</parent><child>post</child></joint>
  <link name='body'><pose>0 0 1 0 0 0</pose>
    <inertial><mass>3</mass>
      <inertia><ixx>0.05</ixx><iyy>0.12</iyy><izz>0.2</izz><ixy>0.01</ixy><ixz>0</ixz><iyz>-0.02</iyz></inertia>
    </inertial></link>
  <joint name='pivot' type='ball'><parent>post</parent><child>body</child>{DAMP}</joint>
</model></sdf>"""


@pytest.fixture(scope="module")
def g():
    from scenario import gazebo
    return gazebo


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _exp(v):
    th = float(np.linalg.norm(v))
    if th < 1e-12:
        return np.eye(3) + _skew(v)
    K = _skew(v / th)
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def test_rotvec_roundtrip(g):
    rng = np.random.default_rng(0)
    for _ in range(200):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        th = rng.uniform(0, math.pi - 1e-3)
        R = g.R_from_rotvec(th * ax)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
        assert np.allclose(g.rotvec_from_R(R), th * ax, atol=1e-9)
        assert np.allclose(R, _exp(th * ax), atol=1e-12)


@pytest.mark.parametrize("damping, q0", [(0.0, (0.1, -0.2, 2.9)), (0.3, (0.1, -0.2, 2.9)),
                                         (0.0, (0.0, np.pi / 2, 0.0))])
def test_oracle_ball_joint_is_darts_discrete_rigid_body(oracle, damping, q0):
    text = SPINNER_SDF.replace("{DAMP}", f"<axis><dynamics><damping>{damping}</damping></dynamics></axis>"
                              if damping else "")
    cm = oracle.load_urdf(text)
    assert cm.n == 3 and cm.joint_names == ["pivot#x", "pivot#y", "pivot#z"]
    assert [cm.model.jtype[i] for i in range(3)] == [0x10, 0x20, 0x30]   # oracle.c ball_part
    I = np.array([[0.05, 0.01, 0.0], [0.01, 0.12, -0.02], [0.0, -0.02, 0.2]])
    D = damping * np.eye(3)
    dt, T = 1e-3, 500
    q = np.array(q0)     # |theta| near pi: the update wraps the angle; (0, pi/2, 0): the old angle chart's singularity
    qd = np.array([0.5, 0.4, 4.0])
    mode = np.full(3, oracle.FORCE, np.int32)
    tau = np.zeros(3)
    R = _exp(q)
    w = qd.copy()
    worst_R = worst_w = 0.0
    for _ in range(T):
        q, qd = oracle.step(cm, dt, q, qd, mode, tau, 0)[:2]
        # DART: ABA at the current velocity with implicit damping, then R exp(dt w)
        wd = np.linalg.solve(I + dt * D, -D @ w - np.cross(w, I @ w))
        w = w + dt * wd
        R = R @ _exp(dt * w)
        assert np.linalg.norm(q) <= math.pi + 1e-12
        worst_R = max(worst_R, float(np.abs(_exp(q) - R).max()))
        worst_w = max(worst_w, float(np.abs(qd - w).max()))
    print(f"ball joint, damping {damping}: {T} steps, max |R - R_dart| {worst_R:.1e}, |w - w_dart| {worst_w:.1e}")
    assert worst_R <= 1e-10 and worst_w <= 1e-10
