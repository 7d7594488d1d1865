"""Host-side coordinate maps of the ScenarI/O ball joint (scenario/gazebo.py
BallJoint): a ball joint runs as three revolute dofs with intrinsic X-Y-Z
angles e = (a, b, c), presented in DART's BallJoint coordinates (rotation
vector, child-frame angular velocity / acceleration / torque).  Checked here
against first principles: the exponential / log maps invert each other, the
angles reproduce the rotation, and w = J(e) e', w' = J e'' + J' e' match
finite differences of R(e(t))."""

import math

import numpy as np
import pytest


@pytest.fixture(scope="module")
def g():
    from scenario import gazebo
    return gazebo


def _skew_inv(S):
    return np.array([S[2, 1] - S[1, 2], S[0, 2] - S[2, 0], S[1, 0] - S[0, 1]]) / 2.0


def test_rotvec_roundtrip(g):
    rng = np.random.default_rng(0)
    for _ in range(200):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        th = rng.uniform(0, math.pi - 1e-3)
        r = th * ax
        R = g.R_from_rotvec(r)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.linalg.det(R) == pytest.approx(1.0)
        assert np.allclose(g.rotvec_from_R(R), r, atol=1e-9)
    assert np.allclose(g.rotvec_from_R(np.eye(3)), 0.0)


def test_angles_roundtrip(g):
    rng = np.random.default_rng(1)
    for _ in range(200):
        e = np.array([rng.uniform(-math.pi, math.pi), rng.uniform(-1.5, 1.5), rng.uniform(-math.pi, math.pi)])
        R = g.ball_R(e)
        assert np.allclose(g.ball_angles(R), e, atol=1e-9)
        # about the joint frame's own axes, in order x, y, z
        assert np.allclose(R, g._rx(e[0]) @ g._ry(e[1]) @ g._rz(e[2]))


def test_velocity_and_acceleration_maps(g):
    """w (child frame) = skew^-1(R^T dR/dt); w' = d/dt of that"""
    rng = np.random.default_rng(2)
    h = 1e-5
    for _ in range(50):
        e0 = np.array([rng.uniform(-2, 2), rng.uniform(-1.2, 1.2), rng.uniform(-2, 2)])
        ed = rng.uniform(-2, 2, 3)
        edd = rng.uniform(-3, 3, 3)
        e = lambda t: e0 + ed * t + 0.5 * edd * t * t
        w = lambda t: _skew_inv(g.ball_R(e(t)).T @ (g.ball_R(e(t + h)) - g.ball_R(e(t - h))) / (2 * h))
        J = g.ball_J(e0)
        assert np.allclose(J @ ed, w(0.0), atol=1e-7)
        wdot_fd = (w(1e-3) - w(-1e-3)) / 2e-3
        assert np.allclose(J @ edd + g.ball_Jdot(e0, ed) @ ed, wdot_fd, atol=1e-4)


def test_torque_map_is_the_power_dual(g):
    """tau_angles = J^T tau: the same power for every rate"""
    rng = np.random.default_rng(3)
    e = np.array([0.3, -0.7, 1.1])
    J = g.ball_J(e)
    tau = rng.normal(size=3)
    ed = rng.normal(size=3)
    assert (J.T @ tau) @ ed == pytest.approx(tau @ (J @ ed))
