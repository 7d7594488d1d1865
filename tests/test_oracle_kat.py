"""Pin the fp64 oracle before trusting it (CPU only).

Known answers used, all from the reference or published algorithms:
  * analytic pendulum of tests/.python/test_pendulum_wrt_ground_truth.py:26-67
    (m = 1, L = 0.5, r = 0.01, I = m (4L^2 + 3r^2) / 12, "integrate with Euler":
    velocity first, then position with the new velocity == DART's
    semi-implicit order); the reference bound is 3 deg;
  * tests/test_scenario/test_velocity_direct.py:20-82 (Coulomb 0.01 + viscous
    0.2 pendulum released at 90 deg rests within 180 +- 0.3 deg after 5000 steps;
    VelocityFollowerDart reaches the target in one run; Idle swing settles at
    2 pi + 180 deg);
  * an independent Lagrangian of the cartpole (derived here, numpy);
  * ABA == RNEA^-1 == CRBA (three independent recursions);
  * Random123 Philox4x32-10 known-answer vectors;
  * projected Gauss-Seidel vs exhaustive boxed-LCP enumeration.
"""

import itertools
import math

import numpy as np
import pytest

G = 9.8


def test_pendulum_matches_reference_ground_truth(oracle, pendulum_file):
    pm = oracle.load_urdf(pendulum_file)
    m, L, r = 1.0, 0.5, 0.01
    inertia = m * (4 * L * L + 3 * r * r) / 12
    rng = np.random.default_rng(42)
    dt = 1.0 / 4000.0          # the legacy test's agent/physics rate
    theta, theta_dot = 2.0, -0.5
    q, qd = np.array([theta]), np.array([theta_dot])
    worst = 0.0
    for _ in range(4000):
        tau = rng.uniform(-50, 50)
        # reference PendulumEnv.step (test_pendulum_wrt_ground_truth.py:53-63)
        theta_ddot = (m * G * L / 2.0 * math.sin(theta) + tau) / inertia
        theta_dot = theta_dot + theta_ddot * dt
        theta = theta + theta_dot * dt
        q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.FORCE], [tau])
        worst = max(worst, abs(q[0] - theta), abs(qd[0] - theta_dot))
    assert worst < 1e-9          # far inside the reference's 3 deg bound


@pytest.mark.parametrize("model", ["cartpole", "pendulum"])
def test_aba_rnea_crba_agree(oracle, cartpole_file, pendulum_file, model):
    cm = oracle.load_urdf(cartpole_file if model == "cartpole" else pendulum_file)
    rng = np.random.default_rng(0)
    for _ in range(20):
        q, qd, tau = rng.normal(size=(3, cm.n)) * 2
        qdd = oracle.aba(cm, q, qd, tau)
        np.testing.assert_allclose(oracle.rnea(cm, q, qd, qdd), tau, atol=1e-10)
        M = oracle.crba(cm, q)
        bias = oracle.rnea(cm, q, qd, np.zeros(cm.n))
        np.testing.assert_allclose(np.linalg.solve(M, tau - bias), qdd, atol=1e-10)
        assert np.allclose(M, M.T) and np.all(np.linalg.eigvalsh(M) > 0)


def test_cartpole_lagrangian(oracle, cartpole_file):
    """Independent equations of motion of the shipped cartpole model."""
    cm = oracle.load_urdf(cartpole_file)
    mc, mp, l, Iyy = 1.0, 0.1, 0.5, 0.0083358333
    rng = np.random.default_rng(1)
    for _ in range(50):
        x, th, dx, dth = rng.uniform(-2, 2, size=4)
        F, tau = rng.uniform(-30, 30, size=2)
        M = np.array([[mc + mp, mp * l * math.cos(th)],
                      [mp * l * math.cos(th), mp * l * l + Iyy]])
        rhs = np.array([F + mp * l * math.sin(th) * dth ** 2, tau + mp * G * l * math.sin(th)])
        expect = np.linalg.solve(M, rhs)
        got = oracle.aba(cm, [x, th], [dx, dth], [F, tau])
        np.testing.assert_allclose(got, expect, rtol=1e-9, atol=1e-9)


def test_implicit_damping_is_backward_euler(oracle, pendulum_file):
    """DART's implicit damping: qd+ = qd + dt qdd with damping on qd+."""
    pm = oracle.load_urdf(pendulum_file)
    pm.model.damping[0] = 0.7
    dt, q, qd, tau = 1e-3, 1.1, 2.0, 0.3
    M = oracle.crba(pm, [q])[0, 0]
    g = oracle.rnea(pm, [q], [0.0], [0.0])[0]
    # M (qd+ - qd)/dt = tau - g - d qd+  ->  qd+ = (M qd + dt (tau - g)) / (M + dt d)
    expect_qd = (M * qd + dt * (tau - g)) / (M + dt * 0.7)
    q1, qd1, *_ = oracle.step(pm, dt, [q], [qd], [oracle.FORCE], [tau])
    assert qd1[0] == pytest.approx(expect_qd, rel=1e-12)
    assert q1[0] == pytest.approx(q + dt * expect_qd, rel=1e-12)


def test_effort_clip(oracle, pendulum_file):
    pm = oracle.load_urdf(pendulum_file)
    pm.model.effort[0] = 500.0
    a = oracle.step(pm, 1e-3, [0.3], [0.0], [oracle.FORCE], [500.0])
    b = oracle.step(pm, 1e-3, [0.3], [0.0], [oracle.FORCE], [5000.0])
    assert a[1][0] == b[1][0]   # clipped to the 500 Nm effort limit


def test_velocity_direct_kat(oracle, pendulum_file):
    """tests/test_scenario/test_velocity_direct.py restated on the oracle."""
    pm = oracle.load_urdf(pendulum_file)
    pm.model.friction[0] = 0.01     # set_coulomb_friction(0.01)
    pm.model.damping[0] = 0.2       # set_viscous_friction(0.2)
    dt = 1e-3
    q, qd = np.array([np.deg2rad(90)]), np.array([0.0])
    for _ in range(5000):
        q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.FORCE], [0.0])
    assert np.deg2rad(179.7) <= q[0] <= np.deg2rad(180.3)
    # VelocityFollowerDart: the target is reached after one run
    q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.SERVO], [np.pi])
    assert qd[0] == pytest.approx(np.pi)
    for _ in range(1500):
        q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.SERVO], [np.pi])
    assert qd[0] == pytest.approx(np.pi)
    q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.SERVO], [-np.pi])
    assert qd[0] == pytest.approx(-np.pi)
    for _ in range(5000):
        q, qd, *_ = oracle.step(pm, dt, q, qd, [oracle.FORCE], [0.0])
    assert 2 * np.pi + np.deg2rad(179.7) <= q[0] <= 2 * np.pi + np.deg2rad(180.3)


def test_joint_limit_holds(oracle, cartpole_file):
    """A prismatic joint driven into its limit stops there (LCP limit row)."""
    cm = oracle.load_urdf(cartpole_file)
    q, qd = np.array([4.7, 0.0]), np.array([0.0, 0.0])
    for _ in range(2000):
        q, qd, *_ = oracle.step(cm, 1e-3, q, qd, [oracle.FORCE, oracle.PASSIVE], [300.0, 0.0])
    assert q[0] <= 4.8 + 0.05
    assert q[0] >= 4.7


def test_philox_known_answers(oracle):
    # Random123 kat_vectors, philox4x32-10
    assert list(oracle.philox_raw([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(oracle.philox_raw([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == \
        [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(oracle.philox_raw([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                                  [0xA4093822, 0x299F31D0])) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def _lcp_exact(A, b, lo, hi):
    """Enumerate the (lo / hi / free) pattern of a small boxed LCP A x = b + w."""
    n = len(b)
    for pattern in itertools.product((0, 1, 2), repeat=n):
        x = np.zeros(n)
        free = [i for i in range(n) if pattern[i] == 2]
        for i in range(n):
            if pattern[i] == 0:
                x[i] = lo[i]
            elif pattern[i] == 1:
                x[i] = hi[i]
        if any(not np.isfinite(x[i]) for i in range(n) if pattern[i] != 2):
            continue
        if free:
            fixed = [i for i in range(n) if pattern[i] != 2]
            rhs = b[free] - A[np.ix_(free, fixed)] @ x[fixed] if fixed else b[free]
            x[free] = np.linalg.solve(A[np.ix_(free, free)], rhs)
        w = A @ x - b
        ok = True
        for i in range(n):
            if pattern[i] == 2:
                ok &= lo[i] - 1e-12 <= x[i] <= hi[i] + 1e-12
            elif pattern[i] == 0:
                ok &= w[i] >= -1e-12
            else:
                ok &= w[i] <= 1e-12
        if ok:
            return x
    raise AssertionError("no LCP solution found")


def test_pgs_matches_exact_boxed_lcp(oracle):
    rng = np.random.default_rng(3)
    for _ in range(30):
        n = rng.integers(1, 4)
        B = rng.normal(size=(n, n))
        A = B @ B.T + 0.5 * np.eye(n)
        b = rng.normal(size=n)
        lo = -rng.uniform(0.05, 1.0, size=n)
        hi = rng.uniform(0.05, 1.0, size=n)
        lo[rng.uniform(size=n) < 0.3] = 0.0
        x = oracle.pgs(A, b, lo, hi, iters=400)
        np.testing.assert_allclose(x, _lcp_exact(A, b, lo, hi), atol=1e-8)


def test_converged_lcp_mode_is_exact(oracle):
    """The oracle's converged mode (sweep budget PGS_CONVERGED, the reference
    for the kernels' truncated PGS): box LCPs against exhaustive enumeration,
    and the friction-coupled contact LCP of a humanoid drop reaches the
    complementarity conditions to round-off at every step."""
    from mwstep import get_model_file
    rng = np.random.default_rng(7)
    for _ in range(200):
        n = rng.integers(1, 6)
        B = rng.normal(size=(n, n))
        A = B @ B.T + 0.05 * np.eye(n)
        b = rng.normal(size=n)
        lo = -rng.uniform(0.05, 1.0, size=n)
        hi = rng.uniform(0.05, 1.0, size=n)
        lo[rng.uniform(size=n) < 0.3] = 0.0
        x = oracle.pgs(A, b, lo, hi, iters=oracle.PGS_CONVERGED)
        np.testing.assert_allclose(x, _lcp_exact(A, b, lo, hi), atol=1e-9)
    from mwstep.models import icub_posture
    cm = oracle.load_urdf(get_model_file("icub"), pose_xyz=(0, 0, 0.6), pose_wxyz=(0, 0, 0, 1))
    ow = oracle.FloatWorld(cm, pgs_iters=oracle.PGS_CONVERGED)
    post = np.array(icub_posture(cm.joint_names))
    ow.set_joints(post, np.zeros(cm.n))
    ow.set_twist([0.3, 0.0, 0.2], [0.5, -0.3, -0.5])
    mode = np.full(cm.n, oracle.FORCE, np.int32)
    n_contact = 0
    for _ in range(150):
        n_contact = max(n_contact, ow.step(mode, np.clip(-500 * (ow.q - post) - 5 * ow.qd, -80, 80)))
        sweeps, res = oracle.pgs_stats()
        assert 0.0 <= res <= 1e-9
    assert n_contact >= 4
