"""The device dynamics code (gym-ignition_amd/csrc/chain_dyn.hpp) compiled for
the host (g++, float32, test-only harness tests/host_dyn/harness.cpp) against
the fp64 oracle -- catches kernel-math bugs without a GPU.  The parameter
block is the exact float32 block the library uploads (mw_device_params)."""

import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HARNESS = os.path.join(ROOT, "tests", "host_dyn", "harness.cpp")
CSRC = os.path.join(ROOT, "gym-ignition_amd", "csrc")


@pytest.fixture(scope="module")
def hd(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("hd") / "libhd.so")
    # -DMW_FAST_MATH: the device's Cody-Waite sincos is exercised on the host too
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-DMW_FAST_MATH", "-I", CSRC,
                    HARNESS, "-o", out], check=True)
    L = ctypes.CDLL(out)
    L.hd_substep.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_int, ctypes.c_void_p]
    L.hd_float_step.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                                         ctypes.c_void_p, ctypes.c_void_p]
    return L


def _params(hd, path, joint_params=()):
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0.0])
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(p), b""))
        for dof, which, v in joint_params:
            N.check(N.lib().mw_set_joint_param(h, dof, which, v))
        size = hd.hd_sizeof_chain()
        buf = ctypes.create_string_buffer(size)
        N.check(N.lib().mw_device_params(h, buf, size))
        return buf
    finally:
        N.lib().mw_destroy(h)


def _substep(hd, P, q, qd, tau, act, vc, cons, dual, pgs=20):
    n = len(q)
    f = lambda a, t=np.float32: np.array(a, dtype=t)   # copies: the harness works in place
    q, qd, tau, vc, act = f(q), f(qd), f(tau), f(vc), f(act, np.uint8)
    qdd = np.zeros(n, np.float32)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert hd.hd_substep(P, ptr(q), ptr(qd), ptr(tau), ptr(act), ptr(vc), 1e-3, pgs, int(cons),
                         int(dual), ptr(qdd)) == 0
    return q.astype(float), qd.astype(float), qdd.astype(float)


@pytest.mark.parametrize("model", ["cartpole", "pendulum", "panda"])
def test_unconstrained_substep(hd, oracle, cartpole_file, pendulum_file, panda_file, model):
    path = {"cartpole": cartpole_file, "pendulum": pendulum_file, "panda": panda_file}[model]
    P = _params(hd, path)
    cm = oracle.load_urdf(path)
    n = cm.n
    rng = np.random.default_rng(5)
    # strictly inside the position limits: no constraint row may activate
    lo = np.maximum([cm.model.lower[i] for i in range(n)], -2.0) + 1e-2
    hi = np.minimum([cm.model.upper[i] for i in range(n)], 2.0) - 1e-2
    eff = np.array([cm.model.effort[i] for i in range(n)])
    for _ in range(300):
        q = rng.uniform(lo, hi).astype(np.float32)
        qd = rng.uniform(-3, 3, n).astype(np.float32)
        # the kernel callers clip to +-effort before the substep; the oracle clips inside
        tau = np.clip(rng.uniform(-40, 40, n), -eff, eff).astype(np.float32)
        got = _substep(hd, P, q, qd, tau, np.zeros(n), np.zeros(n), cons=False, dual=False)
        ref = oracle.step(cm, 1e-3, q.astype(float), qd.astype(float), [oracle.FORCE] * n,
                          tau.astype(float))
        scale = 1.0 + np.abs(ref[2]).max()
        assert np.abs(got[2] - ref[2]).max() <= 2e-6 * scale * 10
        assert np.abs(got[1] - ref[1]).max() <= 1e-5
        assert np.abs(got[0] - ref[0]).max() <= 1e-5


def test_constraint_rows_and_damping(hd, oracle, pendulum_file, cartpole_file):
    from mwstep import native as N
    # pendulum with Coulomb friction + viscous damping (DUAL path), servo rows
    P = _params(hd, pendulum_file, [(0, N.PARAM_COULOMB_FRICTION, 0.01), (0, N.PARAM_VISCOUS_FRICTION, 0.2)])
    pm = oracle.load_urdf(pendulum_file)
    pm.model.friction[0] = 0.01
    pm.model.damping[0] = 0.2
    rng = np.random.default_rng(9)
    for _ in range(200):
        q = rng.uniform(-3, 3, 1).astype(np.float32)
        qd = rng.uniform(-0.02, 0.02, 1).astype(np.float32)
        servo = rng.uniform() < 0.5
        act = [1 if servo else 0]
        vc = rng.uniform(-4, 4, 1).astype(np.float32)
        got = _substep(hd, P, q, qd, [0.0], act, vc, cons=True, dual=True)
        ref = oracle.step(pm, 1e-3, q.astype(float), qd.astype(float),
                          [oracle.SERVO if servo else oracle.FORCE], vc.astype(float) if servo else [0.0])
        assert np.abs(got[1] - ref[1]).max() <= 2e-5, (servo, got, ref)
    # cartpole driven into the rail limit (limit row, 2 coupled dofs)
    P = _params(hd, cartpole_file)
    cm = oracle.load_urdf(cartpole_file)
    q, qd = np.array([4.79, 0.2], np.float32), np.array([0.5, -1.0], np.float32)
    qg, qdg = q.copy(), qd.copy()
    qo, qdo = q.astype(float), qd.astype(float)
    for _ in range(300):
        qg, qdg, _ = _substep(hd, P, qg, qdg, [300.0, 0.0], [0, 0], [0, 0], cons=True, dual=False)
        qo, qdo, *_ = oracle.step(cm, 1e-3, qo, qdo, [oracle.FORCE, oracle.PASSIVE], [300.0, 0.0], 20)
    assert qg[0] <= 4.85 and abs(qg[0] - qo[0]) <= 1e-3 and np.abs(qdg - qdo).max() <= 1e-2


def test_panda_tree_with_limit_rows(hd, oracle, panda_file):
    """The branched Panda (fingers on the hand) with joint-limit rows active:
    impulse columns of the tree, float32 device code vs fp64 oracle."""
    P = _params(hd, panda_file)
    cm = oracle.load_urdf(panda_file)
    n = cm.n
    lo = np.array([cm.model.lower[i] for i in range(n)])
    hi = np.array([cm.model.upper[i] for i in range(n)])
    rng = np.random.default_rng(11)
    worst = 0.0
    for _ in range(100):
        # about half of the joints sit at / beyond a limit
        q = rng.uniform(lo, hi)
        at = rng.uniform(size=n) < 0.5
        q[at] = np.where(rng.uniform(size=n) < 0.5, lo - 1e-3, hi + 1e-3)[at]
        q = q.astype(np.float32)
        qd = rng.uniform(-0.5, 0.5, n).astype(np.float32)
        tau = rng.uniform(-10, 10, n).astype(np.float32)   # within every effort limit
        got = _substep(hd, P, q, qd, tau, np.zeros(n), np.zeros(n), cons=True, dual=False, pgs=30)
        ref = oracle.step(cm, 1e-3, q.astype(float), qd.astype(float), [oracle.FORCE] * n,
                          tau.astype(float), 30)
        worst = max(worst, float(np.abs(got[1] - ref[1]).max()))
    assert worst <= 2e-4, worst


def _float_blocks(hd, text, mu):
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0.0])
        N.check(N.lib().mw_load_model(h, text.encode(), N.dptr(p), b""))
        N.check(N.lib().mw_set_ground_plane(h, 1, mu))
        P = ctypes.create_string_buffer(hd.hd_sizeof_chain())
        N.check(N.lib().mw_device_params(h, P, len(P)))
        F = ctypes.create_string_buffer(hd.hd_sizeof_float())
        N.check(N.lib().mw_device_float_params(h, F, len(F)))
        return P, F
    finally:
        N.lib().mw_destroy(h)


@pytest.mark.parametrize("name", ["quadruped", "chain2"])
def test_floating_tree_step(hd, oracle, name):
    """float_tree.hpp on the host (float32) vs or_float_step (fp64): random
    well-conditioned states (gentle velocities, joints inside their limits,
    feet / corners touching the ground)."""
    import os
    from test_float_tree_oracle import STAND, chain_urdf
    text = (open(os.path.join(ROOT, "gym-ignition_amd", "models", "quadruped.urdf")).read()
            if name == "quadruped" else chain_urdf(2))
    P, F = _float_blocks(hd, text, 0.8)
    cm = oracle.load_urdf(text)
    n = cm.n
    rng = np.random.default_rng(2)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    worst_qd = worst_v = 0.0
    n_contact = 0
    for k in range(60):
        q0 = (STAND if name == "quadruped" else np.zeros(n)) + rng.uniform(-0.2, 0.2, n)
        z = (0.44 if name == "quadruped" else 0.33) + rng.uniform(-0.01, 0.01)
        base = np.array([0.0, 0.0, z, 1, 0, 0, 0, *rng.uniform(-0.2, 0.2, 6)], np.float32)
        q, qd = q0.astype(np.float32), rng.uniform(-0.3, 0.3, n).astype(np.float32)
        tau = rng.uniform(-5, 5, n).astype(np.float32)
        ow = oracle.FloatWorld(cm, ground=True, mu=0.8, pgs_iters=50)
        ow.set_pose(base[:3].astype(float), np.eye(3))
        ow.set_twist(base[7:10].astype(float), base[10:13].astype(float))
        ow.set_joints(q.astype(float), qd.astype(float))
        ow.step(np.full(n, oracle.FORCE, np.int32), tau.astype(float))
        ws = np.zeros(4096, np.float32)
        active = ctypes.c_uint()
        assert hd.hd_float_step(P, F, ptr(base), ptr(q), ptr(qd), ptr(tau), 1e-3, 50, 1, ptr(ws),
                                ctypes.byref(active)) == 0
        assert bin(active.value).count("1") == len(ow.contacts)
        n_contact += len(ow.contacts) > 0
        worst_qd = max(worst_qd, float(np.abs(qd - ow.qd).max()))
        worst_v = max(worst_v, float(np.abs(base[7:] - ow.V).max()))
    assert n_contact >= 30
    assert worst_qd <= 1e-3 and worst_v <= 1e-3, (worst_qd, worst_v)


def test_ball_integrate_matches_library_trig(hd):
    """chain_dyn.hpp ball_integrate carries its own f64 sin / cos / atan2
    (Taylor polynomials, one tangent correction of the fp32 angle: no library
    constants held in the wave kernels' registers).  Against
    the same composition with numpy's fp64 trigonometry, rounded to fp32:
    identical on rotation vectors up to 8.7 rad, small and tiny ones."""
    rng = np.random.default_rng(3)
    n = 200000
    scale = np.repeat([1.8, 0.01, 5.0, 1e-20], n // 4)[:, None]
    th = (rng.uniform(-1, 1, (n, 3)) * scale).astype(np.float32)
    w = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
    dt = np.float32(1e-3)
    out = np.zeros((n, 3), np.float32)
    hd.hd_ball_integrate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    hd.hd_ball_integrate(th.ctypes.data, w.ctypes.data, dt, n, out.ctypes.data)

    def quat(v):
        t = np.linalg.norm(v, axis=1)
        s = np.where(t < 1e-150, 0.5, np.sin(0.5 * t) / np.where(t < 1e-150, 1.0, t))
        return np.column_stack([np.cos(0.5 * t), s[:, None] * v])
    a = quat(th.astype(np.float64))
    b = quat(float(dt) * w.astype(np.float64))
    c0 = a[:, 0] * b[:, 0] - (a[:, 1:] * b[:, 1:]).sum(1)
    cv = a[:, :1] * b[:, 1:] + b[:, :1] * a[:, 1:] + np.cross(a[:, 1:], b[:, 1:])
    sg = np.where(c0 < 0, -1.0, 1.0)
    c0, cv = c0 * sg, cv * sg[:, None]
    v = np.linalg.norm(cv, axis=1)
    f = np.where(v < 1e-150, 2.0 / c0, 2.0 * np.arctan2(v, c0) / np.where(v < 1e-150, 1.0, v))
    ref = (f[:, None] * cv).astype(np.float32)
    diff = np.abs(out.astype(np.float64) - ref)
    ulp = np.spacing(np.abs(ref)).astype(np.float64)
    assert np.all(diff <= ulp), f"max {np.max(diff / np.maximum(ulp, 1e-45))} ulp"
    assert np.mean(out == ref) > 0.999
