"""Numerics prototype (CPU, numpy) of the lane-group Panda step: forward
dynamics as base-frame CRBA + RNEA + Cholesky, evaluated in float32 (or with
selected stages in float64), against the fp64 oracle ABA.  Answers: is the
base-frame formulation accurate enough in float32 for the 1e-4 obs bound?

    python scripts/proto_group_crba.py [n_states]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import pyoracle  # noqa: E402
from mwstep import get_model_file  # noqa: E402


def rot_axis(a, q, F):
    c, s = np.cos(q).astype(F), np.sin(q).astype(F)
    v = F(1) - c
    ax, ay, az = a
    return np.array([[c + ax * ax * v, ax * ay * v - az * s, ax * az * v + ay * s],
                     [ay * ax * v + az * s, c + ay * ay * v, ay * az * v - ax * s],
                     [az * ax * v - ay * s, az * ay * v + ax * s, c + az * az * v]], dtype=F)


def crba_fd(m, q, qd, tau, F=np.float32, FM=np.float32):
    """Forward dynamics of one world: base-frame poses (F), body inertias in the
    base frame and composites, M, h and the Cholesky solve in FM."""
    n = m.n
    par = [m.parent[i] for i in range(n)]
    R0, p0 = [None] * n, [None] * n
    S0 = np.zeros((n, 6), F)
    for i in range(n):
        E = np.array(m.E[i], F).reshape(3, 3)
        r = np.array(m.r[i], F)
        a = np.array(m.axis[i], F)
        if m.jtype[i] == 0:
            R = E @ rot_axis(a, F(q[i]), F)
            p = r
        else:
            R = E
            p = r + F(q[i]) * (E @ a)
        if par[i] >= 0:
            R0[i] = (R0[par[i]] @ R).astype(F)
            p0[i] = (R0[par[i]] @ p + p0[par[i]]).astype(F)
        else:
            R0[i], p0[i] = R, p
        ax0 = R0[i] @ a
        if m.jtype[i] == 0:
            S0[i, :3] = ax0
            S0[i, 3:] = np.cross(p0[i], ax0)
        else:
            S0[i, 3:] = ax0
    # rigid inertias in the base frame about the base origin: (mass, h = m c0, J)
    mass = np.array([m.mass[i] for i in range(n)], FM)
    hh = np.zeros((n, 3), FM)
    JJ = np.zeros((n, 3, 3), FM)
    for i in range(n):
        c = np.array(m.com[i], F)
        c0 = (R0[i] @ c + p0[i]).astype(FM)
        Ic = np.array(m.Ic[i], FM)
        Icm = np.array([[Ic[0], Ic[3], Ic[4]], [Ic[3], Ic[1], Ic[5]], [Ic[4], Ic[5], Ic[2]]], FM)
        Rm = R0[i].astype(FM)
        hh[i] = mass[i] * c0
        JJ[i] = Rm @ Icm @ Rm.T + mass[i] * (np.dot(c0, c0) * np.eye(3, dtype=FM) - np.outer(c0, c0))
    # composites: subtree sums
    cm_, ch, cJ = mass.copy(), hh.copy(), JJ.copy()
    for i in range(n - 1, -1, -1):
        if par[i] >= 0:
            cm_[par[i]] += cm_[i]
            ch[par[i]] += ch[i]
            cJ[par[i]] += cJ[i]

    def imul(mm, h, J, V):
        w, v = V[:3], V[3:]
        return np.concatenate([J @ w + np.cross(h, v), mm * v - np.cross(h, w)])

    S0m = S0.astype(FM)
    M = np.zeros((n, n), FM)
    for i in range(n):
        Fi = imul(cm_[i], ch[i], cJ[i], S0m[i])
        M[i, i] = S0m[i] @ Fi
        j = par[i]
        while j >= 0:
            M[i, j] = M[j, i] = S0m[j] @ Fi
            j = par[j]
    # RNEA bias with qdd = 0, base acceleration = -g
    g = np.array(m.gravity_base, FM)
    V = np.zeros((n, 6), FM)
    A = np.zeros((n, 6), FM)
    f = np.zeros((n, 6), FM)
    for i in range(n):
        Sq = S0m[i] * FM(qd[i])
        if par[i] >= 0:
            Vp, Ap = V[par[i]], A[par[i]]
        else:
            Vp, Ap = np.zeros(6, FM), np.concatenate([np.zeros(3, FM), -g])
        V[i] = Vp + Sq
        # c = V_parent x_m (S qd)
        w, v = Vp[:3], Vp[3:]
        c = np.concatenate([np.cross(w, Sq[:3]), np.cross(w, Sq[3:]) + np.cross(v, Sq[:3])])
        A[i] = Ap + c
        IV = imul(mass[i], hh[i], JJ[i], V[i])
        IA = imul(mass[i], hh[i], JJ[i], A[i])
        w, v = V[i][:3], V[i][3:]
        f[i] = IA + np.concatenate([np.cross(w, IV[:3]) + np.cross(v, IV[3:]), np.cross(w, IV[3:])])
    fs = f.copy()
    for i in range(n - 1, -1, -1):
        if par[i] >= 0:
            fs[par[i]] += fs[i]
    h = np.array([S0m[i] @ fs[i] for i in range(n)], FM)
    b = (np.asarray(tau, FM) - h).astype(FM)
    # Cholesky
    L = np.zeros_like(M)
    Mw = M.copy()
    for k in range(n):
        L[k, k] = np.sqrt(Mw[k, k])
        for i in range(k + 1, n):
            L[i, k] = Mw[i, k] / L[k, k]
        for i in range(k + 1, n):
            for j in range(k + 1, i + 1):
                Mw[i, j] -= L[i, k] * L[j, k]
    y = np.zeros(n, FM)
    for k in range(n):
        y[k] = (b[k] - L[k, :k] @ y[:k]) / L[k, k]
    x = np.zeros(n, FM)
    for k in range(n - 1, -1, -1):
        x[k] = (y[k] - L[k + 1:, k] @ x[k + 1:]) / L[k, k]
    return x, M, h


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    cm = pyoracle.load_urdf(get_model_file("panda"))
    m = cm.model
    n = m.n
    rng = np.random.default_rng(0)
    lo = np.array([m.lower[i] for i in range(n)])
    hi = np.array([m.upper[i] for i in range(n)])
    eff = np.array([m.effort[i] for i in range(n)])
    res = {}
    for label, F, FM in (("f32/f32", np.float32, np.float32), ("f32 poses / f64 M,h", np.float32, np.float64),
                         ("f64", np.float64, np.float64)):
        worst = 0.0
        worstM = 0.0
        for _ in range(ns):
            q = rng.uniform(lo, hi)
            qd = rng.uniform(-1, 1, n)
            tau = rng.uniform(-0.3, 0.3, n) * eff
            ref = pyoracle.aba(cm, q, qd, tau)
            Mref = pyoracle.crba(cm, q)
            x, M, _ = crba_fd(m, q, qd, tau, F, FM)
            worst = max(worst, float(np.abs(x.astype(np.float64) - ref).max()))
            worstM = max(worstM, float(np.abs(M.astype(np.float64) - Mref).max()))
        res[label] = {"qdd_err": worst, "qd_err_per_step(dt=1e-3)": worst * 1e-3, "M_err": worstM}
    for k, v in res.items():
        print(f"{k:24s} {v}")


if __name__ == "__main__":
    main()
