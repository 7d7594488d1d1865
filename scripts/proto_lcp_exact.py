"""Prototype (numpy, float32 arithmetic) of the wave kernel's exact boxed-LCP
solve, checked against the fp64 oracle's converged solution on LCPs captured
from iCub-class (models/icub.urdf) drops / slides (pyoracle.lcp_last).  Mirrors the device
algorithm step by step so the iteration counts and fp32 errors seen here are
the kernel's:
  PGS warm-up (K sweeps) -> active-set Newton rounds: classify rows (held at a
  bound with a correctly signed gradient, else free; friction boxes
  [-mu x_n, mu x_n] from the current normals), solve A_FF d = -g_F by a masked
  Cholesky, x += d, project (normals, then frictions on the new normals), and
  one PGS sweep; stop when the complementarity residual is <= tol.
    python scripts/proto_lcp_exact.py [n_worlds] [steps]"""
import os
import sys

import numpy as np
BPP = int(__import__('os').environ.get('BPP', '0'))
SKIP = int(__import__('os').environ.get('SKIP', '0'))
STATS = [0, 0, 0]  # solves in phase 0, phase 1; phase-1 rounds (instrumentation)
LOOSE = float(__import__('os').environ.get('LOOSE', '10'))
BEST = int(__import__('os').environ.get('BEST', '0'))

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
import pyoracle  # noqa: E402

f32 = np.float32
BIG = f32(3.4e38)
LSNORM = os.environ.get("LSNORM", "max")
LSMODE = os.environ.get("LSMODE", "max")
BAND = float(os.environ.get("BAND", "0"))
SSN_MAX = int(os.environ.get("SSN_MAX", "6"))
PGS_ON_FAIL = int(os.environ.get("PGS_ON_FAIL", "0"))


def capture(n_worlds=8, steps=60, seed=21, every=1):
    from mwstep import get_model_file
    from mwstep.models import icub_pid_gains, icub_posture
    cm = pyoracle.load_urdf(get_model_file("icub"), pose_xyz=(0, 0, 0.572), pose_wxyz=(0, 0, 0, 1))
    post = np.array(icub_posture(cm.joint_names))
    n = cm.n
    rng = np.random.default_rng(seed)
    stiff = [any(k in nm for k in ("hip", "knee", "ankle", "torso")) for nm in cm.joint_names]
    kp = np.array([500.0 if s else 50.0 for s in stiff])
    kd = np.array([5.0 if s else 0.5 for s in stiff])
    lo, hi = np.array(cm.model.lower[:n]), np.array(cm.model.upper[:n])
    probs = []
    for w in range(n_worlds):
        ow = pyoracle.FloatWorld(cm, ground=True, mu=1.0, pgs_iters=pyoracle.PGS_CONVERGED)
        ang = rng.uniform(0, 0.08)
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        c, s = np.cos(ang), np.sin(ang)
        K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = np.eye(3) + s * K + (1 - c) * K @ K
        ow.set_pose([0, 0, 0.572 + rng.uniform(0, 0.09)], R)
        ow.set_twist(R.T @ rng.uniform(-0.3, 0.3, 3),
                     R.T @ np.array([*rng.uniform(-0.8, 0.8, 2), rng.uniform(-0.5, 0)]))
        ow.set_joints(np.clip(post + rng.uniform(-0.1, 0.1, n), lo, hi), rng.uniform(-0.5, 0.5, n))
        mode = np.full(n, pyoracle.FORCE, np.int32)
        for k in range(steps):
            tau = np.clip(-kp * (ow.q - post) - kd * ow.qd, -80, 80)
            ow.step(mode, tau)
            p = pyoracle.lcp_last()
            if p is not None and len(p["b"]) > 0 and k % every == 0:
                probs.append(p)
            pyoracle.lib()  # keep
    return probs


def residual(A, b, lo_, hi_, kind, mu, x, norm="max"):
    """oracle lcp_residual (velocity units)"""
    s = b - A @ x
    n = len(b)
    L, U = lo_.copy(), hi_.copy()
    for r in range(n):
        if kind[r] == 1:
            u = mu * x[r - r % 3]
            L[r], U[r] = -u, u
    xm = np.abs(x).max()
    tol = 1e-6 * (1 + xm)
    e = np.zeros(n)
    for r in range(n):
        if x[r] < L[r] - tol or x[r] > U[r] + tol:
            e[r] = (L[r] - x[r] if x[r] < L[r] else x[r] - U[r]) * A[r, r]
        elif U[r] - L[r] <= tol:
            e[r] = 0
        elif x[r] <= L[r] + tol:
            e[r] = max(s[r], 0)
        elif x[r] >= U[r] - tol:
            e[r] = max(-s[r], 0)
        else:
            e[r] = abs(s[r])
    return e.max() if norm == "max" else float(np.sqrt((e * e).sum()))


def bounds32(lo_, hi_, kind, mu, x):
    L, U = lo_.copy(), hi_.copy()
    for r in range(len(x)):
        if kind[r] == 1:
            u = f32(mu) * max(x[r - r % 3], f32(0))
            L[r], U[r] = -u, u
    return L, U


def pgs_sweep(A, b, L0, U0, kind, mu, x):
    for r in range(len(x)):
        v = f32(x[r] + (b[r] - A[r] @ x) / A[r, r])
        if kind[r] == 1:
            u = f32(mu) * x[r - r % 3]
            v = min(max(v, -u), u)
        else:
            v = min(max(v, L0[r]), U0[r])
        x[r] = v
    return x


def chol_solve_masked(A, free, rhs):
    """K = A on free x free, identity elsewhere; right-looking Cholesky in fp32."""
    n = len(rhs)
    K = np.where(np.outer(free, free), A, f32(0)).astype(f32)
    K[~free, ~free] = f32(1)  # diag of held rows
    for r in range(n):
        if not free[r]:
            K[r, :] = 0
            K[:, r] = 0
            K[r, r] = 1
    y = np.where(free, rhs, 0).astype(f32)
    Lf = np.zeros((n, n), f32)
    for k in range(n):
        d = max(K[k, k], f32(1e-30))
        inv = f32(1) / np.sqrt(d, dtype=f32)
        l = (K[k:, k] * inv).astype(f32)
        Lf[k:, k] = l
        y[k] = y[k] * inv
        y[k + 1:] -= l[1:] * y[k]
        K[k + 1:, k + 1:] -= np.outer(l[1:], l[1:]).astype(f32)
    d = np.zeros(n, f32)
    for k in range(n - 1, -1, -1):
        d[k] = (y[k] - Lf[k + 1:, k] @ d[k + 1:]) / Lf[k, k]
    return d


def solve32(p, warm_sweeps=20, rounds=12, tol=1e-6, smooth=1, x0=None):
    A = p["A"].astype(f32)
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    n = len(b)
    lo0 = np.where(np.isfinite(p["lo"]), p["lo"], -BIG).astype(f32)
    hi0 = np.where(np.isfinite(p["hi"]), p["hi"], BIG).astype(f32)
    x = np.zeros(n, f32) if x0 is None else x0.astype(f32)
    for _ in range(warm_sweeps):
        pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    used = 0
    for it in range(rounds):
        L, U = bounds32(lo0, hi0, kind, mu, x)
        g = (A @ x - b).astype(f32)
        # residual in f32
        res = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
        if res <= tol:
            break
        used += 1
        held = ((x <= L) & (g >= 0)) | ((x >= U) & (g <= 0)) | (L == U)
        free = ~held
        d = chol_solve_masked(A, free, -g)
        x = (x + d).astype(f32)
        # project: normals, then frictions with the new normals, box rows
        for r in range(n):
            if kind[r] == 0:
                x[r] = max(x[r], f32(0))
            elif kind[r] == 2:
                x[r] = min(max(x[r], lo0[r]), hi0[r])
        for r in range(n):
            if kind[r] == 1:
                u = mu * x[r - r % 3]
                x[r] = min(max(x[r], -u), u)
        for _ in range(smooth):
            pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    res = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
    return x, used, res


def ge_solve(K, rhs):
    """Gaussian elimination with partial pivoting in fp32 (lane = row on the device)."""
    n = len(rhs)
    K = K.astype(f32).copy()
    y = rhs.astype(f32).copy()
    used = np.zeros(n, bool)
    perm = []
    for j in range(n):
        cand = np.where(~used, np.abs(K[:, j]), -1)
        p = int(np.argmax(cand))
        perm.append(p)
        used[p] = True
        piv = K[p, j]
        if piv == 0:
            piv = f32(1e-30)
        for r in range(n):
            if not used[r]:
                f = f32(K[r, j] / piv)
                K[r, j + 1:] -= f * K[p, j + 1:]
                y[r] -= f * y[p]
    d = np.zeros(n, f32)
    acc = y.copy()
    for j in range(n - 1, -1, -1):
        p = perm[j]
        d[j] = acc[p] / (K[p, j] if K[p, j] != 0 else f32(1e-30))
        acc -= K[:, j] * d[j]
    return d


def solve_ssn(p, warm_sweeps=20, rounds=12, tol=1e-6, smooth=0, x0=None, linesearch=0):
    """semismooth Newton on the coupled conditions (friction rows at their
    bound move with their normal: d_t = s mu d_n)"""
    A = p["A"].astype(f32)
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    n = len(b)
    lo0 = np.where(np.isfinite(p["lo"]), p["lo"], -BIG).astype(f32)
    hi0 = np.where(np.isfinite(p["hi"]), p["hi"], BIG).astype(f32)
    x = np.zeros(n, f32) if x0 is None else x0.astype(f32)
    for _ in range(warm_sweeps):
        pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    used = 0
    best, bestres = x.copy(), 1e30
    for it in range(rounds + 1):
        res = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
        if res < bestres:
            best, bestres = x.copy(), res
        if res <= tol or it == rounds:
            break
        used += 1
        g = (A @ x - b).astype(f32)
        # status: 0 free, 1 fixed (d = 0), 2 coupled (d_t = s mu d_n)
        st = np.zeros(n, int)
        sgn = np.zeros(n, f32)
        for r in range(n):
            if kind[r] == 0:
                st[r] = 1 if (x[r] <= 0 and g[r] >= 0) else 0
            elif kind[r] == 2:
                st[r] = 1 if ((x[r] <= lo0[r] and g[r] >= 0) or (x[r] >= hi0[r] and g[r] <= 0)) else 0
        for r in range(n):
            if kind[r] == 1:
                nr = r - r % 3
                u = mu * x[nr]
                if st[nr] == 1 or u <= 0:
                    st[r] = 1
                elif x[r] >= u and g[r] <= 0:
                    st[r], sgn[r] = 2, f32(1)
                elif x[r] <= -u and g[r] >= 0:
                    st[r], sgn[r] = 2, f32(-1)
        K = np.eye(n, dtype=f32)
        rhs = np.zeros(n, f32)
        for r in range(n):
            if st[r] != 0:
                continue
            row = np.where(st == 0, A[r], 0).astype(f32)
            for t in range(n):
                if st[t] == 2:
                    row[t - t % 3] += sgn[t] * mu * A[r, t]
            K[r] = row
            rhs[r] = -g[r]
        d = ge_solve(K, rhs)
        for t in range(n):
            if st[t] == 2:
                d[t] = sgn[t] * mu * d[t - t % 3]
            elif st[t] == 1:
                d[t] = 0
        xs = x
        for ls in range(linesearch + 1):
            step = f32(0.5 ** ls)
            x = (xs + step * d).astype(f32)
            for r in range(n):
                if kind[r] == 0:
                    x[r] = max(x[r], f32(0))
                elif kind[r] == 2:
                    x[r] = min(max(x[r], lo0[r]), hi0[r])
            for r in range(n):
                if kind[r] == 1:
                    u = mu * x[r - r % 3]
                    x[r] = min(max(x[r], -u), u)
            if linesearch == 0:
                break
            r1 = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64), LSNORM)
            r0 = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], xs.astype(np.float64), LSNORM)
            if r1 < r0:
                break
        for _ in range(smooth):
            pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    return best, used, bestres


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    every = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    probs = capture(nw, steps, every=every)
    print(f"{len(probs)} LCPs, rows {min(len(p['b']) for p in probs)}..{max(len(p['b']) for p in probs)}")
    for fn, cfg in [(solve32, dict(warm_sweeps=50, rounds=0)), (solve_ssn, dict(warm_sweeps=10, rounds=8)),
                    (solve_ssn, dict(warm_sweeps=20, rounds=8)), (solve_ssn, dict(warm_sweeps=10, rounds=8, smooth=1)),
                    (solve_ssn, dict(warm_sweeps=0, rounds=12)), (solve_ssn, dict(warm_sweeps=10, rounds=8, linesearch=3)),
                    (solve_ssn, dict(warm_sweeps=0, rounds=12, linesearch=3)), (solve_ssn, dict(warm_sweeps=20, rounds=8, linesearch=3))]:
        ev, its, res_ = [], [], []
        for p in probs:
            x, used, res = fn(p, **cfg)
            dx = x.astype(np.float64) - p["x"]
            ev.append(np.abs(p["A"] @ dx).max())
            its.append(used)
            res_.append(res)
        ev, its, res_ = np.array(ev), np.array(its), np.array(res_)
        print(f"{fn.__name__} {cfg}: |A dx| median {np.median(ev):.2e} p99 {np.percentile(ev, 99):.2e} max {ev.max():.2e}; "
              f"rounds mean {its.mean():.2f} max {its.max()}; residual max {res_.max():.2e}")


if __name__ == "__main__" and len(sys.argv) <= 4:
    main()


def boxqp32(A, b, L, U, x, max_it=200, count=None):
    """the oracle's primal active-set box QP (boxqp_solve) in fp32; masked
    Cholesky for the Newton steps; returns iterations (-1 on budget)"""
    n = len(b)
    ws = np.zeros(n, int)
    for r in range(n):
        if x[r] <= L[r]:
            x[r], ws[r] = L[r], 1
        elif x[r] >= U[r]:
            x[r], ws[r] = U[r], 2
        if L[r] == U[r]:
            ws[r] = 1
    at_min = False
    for it in range(max_it):
        g = (A @ x - b).astype(f32)
        free = ws == 0
        if not at_min and free.any():
            d = chol_solve_masked(A, free, -g)
            if count is not None:
                count[0] += 1
            dn = np.abs(d).max()
        else:
            d, dn = np.zeros(n, f32), 0.0
        xm = np.abs(x).max()
        if at_min or dn <= 1e-7 * (1 + xm):
            at_min = False
            gm = np.abs(g).max()
            tol = 1e-6 * (1 + gm)
            v = np.where(ws == 1, -g, np.where(ws == 2, g, 0))
            v = np.where(L == U, 0, v)
            worst = int(np.argmax(v))
            if v[worst] <= tol:
                return it
            ws[worst] = 0
            continue
        alpha, block, bside = f32(1), -1, 0
        for r in range(n):
            if not free[r]:
                continue
            if d[r] < 0 and x[r] + d[r] < L[r]:
                a = (L[r] - x[r]) / d[r]
                if a < alpha:
                    alpha, block, bside = a, r, 1
            elif d[r] > 0 and x[r] + d[r] > U[r]:
                a = (U[r] - x[r]) / d[r]
                if a < alpha:
                    alpha, block, bside = a, r, 2
        alpha = max(alpha, 0)
        x[free] += f32(alpha) * d[free]
        if block >= 0:
            x[block] = L[block] if bside == 1 else U[block]
            ws[block] = bside
        else:
            at_min = True
    return -1


def solve_stag(p, warm_sweeps=20, rounds=30, tol=1e-6, x0=None):
    A = p["A"].astype(f32)
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    n = len(b)
    lo0 = np.where(np.isfinite(p["lo"]), p["lo"], -BIG).astype(f32)
    hi0 = np.where(np.isfinite(p["hi"]), p["hi"], BIG).astype(f32)
    x = np.zeros(n, f32) if x0 is None else x0.astype(f32)
    for _ in range(warm_sweeps):
        pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    count = [0]
    for rnd in range(rounds):
        L, U = bounds32(lo0, hi0, kind, mu, x)
        prev = x.copy()
        boxqp32(A, b, L, U, x, count=count)
        if np.abs(x - prev).max() <= 1e-6 * (1 + np.abs(x).max()):
            break
    res = residual(A.astype(np.float64), b.astype(np.float64), p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
    return x, count[0], res


if __name__ == "__main__" and len(sys.argv) > 4:
    import pickle
    probs = pickle.load(open(sys.argv[4], "rb"))
    for ws_ in (0, 10, 20):
        ev, its, res_ = [], [], []
        for p in probs:
            x, used, res = solve_stag(p, warm_sweeps=ws_)
            dx = x.astype(np.float64) - p["x"]
            ev.append(np.abs(p["A"] @ dx).max())
            its.append(used)
            res_.append(res)
        ev, its, res_ = np.array(ev), np.array(its), np.array(res_)
        print(f"staggered warm {ws_}: |A dx| median {np.median(ev):.2e} p99 {np.percentile(ev, 99):.2e} max {ev.max():.2e}; "
              f"solves mean {its.mean():.2f} p99 {np.percentile(its, 99)} max {its.max()}; residual max {res_.max():.2e}")


def solve_hybrid(p, warm_sweeps=20, ssn_rounds=4, tol=1e-6):
    x, used, res = solve_ssn(p, warm_sweeps=warm_sweeps, rounds=ssn_rounds, linesearch=3, tol=tol)
    if res <= tol:
        return x, used, res, 0
    x2, cnt, res2 = solve_stag(p, warm_sweeps=0, x0=x)
    return x2, used + cnt, res2, 1


if __name__ == "__main__" and len(sys.argv) > 5:
    for ws_ in (10, 20):
        ev, its, fb = [], [], 0
        for p in probs:
            x, used, res, f = solve_hybrid(p, warm_sweeps=ws_)
            dx = x.astype(np.float64) - p["x"]
            ev.append(np.abs(p["A"] @ dx).max())
            its.append(used)
            fb += f
        ev, its = np.array(ev), np.array(its)
        print(f"hybrid warm {ws_}: |A dx| median {np.median(ev):.2e} p99 {np.percentile(ev, 99):.2e} max {ev.max():.2e}; "
              f"solves mean {its.mean():.2f} p99 {np.percentile(its, 99)} max {its.max()}; fallbacks {fb}/{len(probs)}")


def device_solve(p, warm_sweeps=20, ssn_rounds=int(os.environ.get('SSN', '4')), max_solves=16, tol=1e-6):
    """the kernel's algorithm: PGS warm-up, semismooth Newton rounds with a
    monotone line search (stop when it fails), then the staggered active-set
    fallback within a total solve budget"""
    A = p["A"].astype(f32)
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    n = len(b)
    lo0 = np.where(np.isfinite(p["lo"]), p["lo"], -BIG).astype(f32)
    hi0 = np.where(np.isfinite(p["hi"]), p["hi"], BIG).astype(f32)
    x = np.zeros(n, f32)
    for _ in range(warm_sweeps):
        pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    A64, b64 = A.astype(np.float64), b.astype(np.float64)
    res = residual(A64, b64, p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
    solves = 0
    for it in range(ssn_rounds):
        if res <= tol:
            return x, solves, res, 0
        x1, used, r1 = solve_ssn(p, warm_sweeps=0, rounds=1, linesearch=3, tol=tol, x0=x)
        solves += 1
        if r1 >= res:
            if PGS_ON_FAIL:
                for _ in range(PGS_ON_FAIL):
                    pgs_sweep(A, b, lo0, hi0, kind, mu, x)
                res = residual(A64, b64, p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
                continue
            break
        x, res = x1, r1
    if res <= tol:
        return x, solves, res, 0
    # staggered fallback within the budget
    count = [0]
    for rnd in range(30):
        L, U = bounds32(lo0, hi0, kind, mu, x)
        prev = x.copy()
        boxqp32(A, b, L, U, x, max_it=max(max_solves - solves - count[0], 0) * 2, count=count)
        if np.abs(x - prev).max() <= 1e-6 * (1 + np.abs(x).max()) or solves + count[0] >= max_solves:
            break
    res = residual(A64, b64, p["lo"], p["hi"], kind, p["mu"], x.astype(np.float64))
    return x, solves + count[0], res, 1


if __name__ == "__main__" and len(sys.argv) > 6:
    for ms in (8, 16, 32):
        ev, its, fb = [], [], 0
        for p in probs:
            x, used, res, f = device_solve(p, max_solves=ms)
            dx = x.astype(np.float64) - p["x"]
            ev.append(np.abs(p["A"] @ dx).max())
            its.append(used)
            fb += f
        ev, its = np.array(ev), np.array(its)
        print(f"device max_solves {ms}: |A dx| median {np.median(ev):.2e} p99 {np.percentile(ev, 99):.2e} max {ev.max():.2e}; "
              f"solves mean {its.mean():.2f} p99 {np.percentile(its, 99)} max {its.max()}; fallbacks {fb}/{len(probs)}")


def wave_exact(p, pgs_sweeps=20, max_solves=16, x0=None):
    """numpy emulation of wave_lcp.hpp wave_lcp_exact (fp32, lane-vectorised)"""
    A = p["A"].astype(f32)
    n = len(p["b"])
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    lo0 = np.where(np.isfinite(p["lo"]), p["lo"], -BIG).astype(f32)
    hi0 = np.where(np.isfinite(p["hi"]), p["hi"], BIG).astype(f32)
    lo0 = np.where(kind == 0, f32(0), lo0)
    hi0 = np.where(kind == 0, BIG, hi0)
    nrow = np.array([r - r % 3 if kind[r] == 1 else r for r in range(n)])
    x = np.zeros(n, f32) if x0 is None else x0.astype(f32).copy()
    for _ in range(pgs_sweeps):
        pgs_sweep(A, b, lo0, hi0, kind, mu, x)
    arr = np.diag(A).copy()
    RT, AT = f32(float(__import__('os').environ.get('RT', '4e-6'))), f32(float(__import__('os').environ.get('AT', '1e-7')))

    def bounds(xl):
        u = mu * np.maximum(xl[nrow], 0)
        return np.where(kind == 1, -u, lo0), np.where(kind == 1, u, hi0)

    def res(xl, w, mag, L, U, tolx):
        s = b - w
        e = np.where((xl < L - tolx) | (xl > U + tolx), np.where(xl < L, L - xl, xl - U) * arr,
                     np.where(U - L <= tolx, 0, np.where(xl <= L + tolx, np.maximum(s, 0),
                                                         np.where(xl >= U - tolx, np.maximum(-s, 0), np.abs(s)))))
        return e.astype(f32), (e / (RT * (np.abs(b) + mag) + AT)).max()

    solves, phase, at_min, new_round = 0, 0, False, True
    ssn_n, best_e, best_x = 0, np.inf, x.copy()
    bpp_best, bpp_strikes = 1 << 30, 0
    ws = np.zeros(n, int)
    Lf = Uf = prev = None
    conv = False
    polish, polish_at = False, 0
    for it in range(4 * max_solves + 8):
        w = (A @ x).astype(f32)
        mag = (np.abs(A) @ np.abs(x)).astype(f32)
        g = w - b
        L, U = bounds(x)
        xmax = np.abs(x).max()
        tolx = f32(2e-6) * (1 + xmax)
        e_abs, rel = res(x, w, mag, L, U, tolx)
        if rel <= 1 or (polish and rel <= LOOSE and solves > polish_at):
            conv = True
            break
        if rel > LOOSE:
            polish = False
        elif not polish:
            polish, polish_at = True, solves
        if rel < best_e:
            best_e, best_x = rel, x.copy()
        if solves >= max_solves:
            break
        if phase == 1 and new_round:
            STATS[2] += 1
            bpp_best, bpp_strikes = 1 << 30, 0
            new_round = False
            Lf, Uf, prev = L.copy(), U.copy(), x.copy()
            ws = np.where(x <= Lf, 1, np.where(x >= Uf, 2, 0))
            x = np.where(x <= Lf, Lf, np.where(x >= Uf, Uf, x)).astype(f32)
            ws = np.where(Lf == Uf, 1, ws)
            at_min = False
            continue
        if phase == 1 and BPP and not new_round and at_min:
            # block principal pivoting on the round's box QP (x: the subspace
            # minimiser of the current partition)
            at_min = False
            gm = np.abs(g).max()
            tg = RT * (1 + gm)
            live = Lf != Uf
            inf_lo = (ws == 0) & (x < Lf) & live
            inf_hi = (ws == 0) & (x > Uf) & live
            inf_bl = (ws == 1) & (g < -tg) & live
            inf_bu = (ws == 2) & (g > tg) & live
            inf = inf_lo | inf_hi | inf_bl | inf_bu
            ninf = int(inf.sum())
            if ninf == 0:
                if np.abs(x - prev).max() <= tolx:
                    break
                new_round = True
                continue
            if ninf < bpp_best:
                bpp_best, bpp_strikes = ninf, 0
                flip = inf
            elif bpp_strikes < 3:
                bpp_strikes += 1
                flip = inf
            else:
                flip = np.zeros(n, bool)
                flip[int(np.nonzero(inf)[0].max())] = True
            ws = np.where(flip & inf_lo, 1, np.where(flip & inf_hi, 2, np.where(flip & (inf_bl | inf_bu), 0, ws)))
            x = np.where(ws == 1, Lf, np.where(ws == 2, Uf, x)).astype(f32)
            continue
        if phase == 1 and at_min:
            at_min = False
            v = np.where(ws == 1, -g, np.where(ws == 2, g, 0))
            v = np.where(Lf == Uf, 0, v)
            gm = np.abs(g).max()
            worst = int(np.argmax(v))
            if v[worst] <= RT * (1 + gm):
                if np.abs(x - prev).max() <= tolx:
                    break
                new_round = True
            else:
                ws[worst] = 0
            continue
        emax = e_abs.max()
        if phase == 0:
            band = BAND * (1 + xmax)
            fixed = np.zeros(n, bool)
            fixed |= (kind == 0) & (x <= band) & (g >= 0)
            fixed |= (kind == 2) & (((x <= lo0 + band) & (g >= 0)) | ((x >= hi0 - band) & (g <= 0)))
            nfixed = fixed[nrow]
            cpos = np.zeros(n, bool)
            cneg = np.zeros(n, bool)
            for r in range(n):
                if kind[r] == 1 and not fixed[r]:
                    if nfixed[r]:
                        fixed[r] = True
                    elif U[r] <= 0:
                        # a contact opening from x_n = 0: its frictions start on the
                        # pyramid edge they push towards (sliding), 0 if g_t = 0
                        if g[r] < 0:
                            cpos[r] = True
                        elif g[r] > 0:
                            cneg[r] = True
                        else:
                            fixed[r] = True
                    elif x[r] >= U[r] - band and g[r] <= 0:
                        cpos[r] = True
                    elif x[r] <= L[r] + band and g[r] >= 0:
                        cneg[r] = True
            fr = ~fixed & ~cpos & ~cneg
            coup = np.where(cpos, mu, np.where(cneg, -mu, 0)).astype(f32)
            K = np.where(np.outer(fr, fr), A, 0).astype(f32)
            K[~fr] = 0
            K[~fr, ~fr] = 1
            for c in range(0, n - 2, 3):
                s1 = f32(cpos[c + 1]) - f32(cneg[c + 1])
                s2 = f32(cpos[c + 2]) - f32(cneg[c + 2])
                K[fr, c] += mu * (s1 * A[fr, c + 1] + s2 * A[fr, c + 2])
        else:
            fr = ws == 0
            if SKIP and np.abs(np.where(fr & (Lf != Uf), g, 0)).max() <= RT * (1 + np.abs(g).max()):
                # the free rows are already stationary: the working set's minimiser
                at_min = True
                continue
            K = np.where(np.outer(fr, fr), A, 0).astype(f32)
            K[~fr] = 0
            K[~fr, ~fr] = 1
        d = ge_solve(K, np.where(fr, -g, 0).astype(f32))
        solves += 1
        STATS[phase] += 1
        x_prev = x.copy()
        if phase == 0:
            d = np.where(fr, d, coup * d[nrow]).astype(f32)
            acc = False
            step = f32(1)
            for ls in range(4):
                xt = (x + step * d).astype(f32)
                xt = np.where(kind == 0, np.maximum(xt, 0), xt)
                xt = np.where(kind == 2, np.minimum(np.maximum(xt, lo0), hi0), xt)
                Lt, Ut = bounds(xt)
                xt = np.where(kind == 1, np.minimum(np.maximum(xt, Lt), Ut), xt).astype(f32)
                wt = (A @ xt).astype(f32)
                mt = (np.abs(A) @ np.abs(xt)).astype(f32)
                et, _ = res(xt, wt, mt, Lt, Ut, f32(2e-6) * (1 + np.abs(xt).max()))
                if LSMODE == "none" or ((et.max() < emax) if LSMODE == "max" else ((et * et).sum() < (e_abs * e_abs).sum())):
                    x, acc = xt, True
                    break
                step *= f32(0.5)
            if LSMODE == "none":
                ssn_n += 1
                if emax < best_e:
                    best_e, best_x = emax, x_prev
                if ssn_n >= SSN_MAX:
                    # back to the best point seen, then the staggered phase
                    wtmp = (A @ x).astype(f32)
                    mtmp = (np.abs(A) @ np.abs(x)).astype(f32)
                    Lb, Ub = bounds(x)
                    et2, _ = res(x, wtmp, mtmp, Lb, Ub, f32(2e-6) * (1 + np.abs(x).max()))
                    if et2.max() > best_e:
                        x = best_x
                    phase, new_round = 1, True
                continue
            if not acc:
                phase, new_round = 1, True
            continue
        if BPP:
            x = np.where(fr, x + d, x).astype(f32)
            at_min = True
            continue
        if np.abs(d).max() <= 1e-7 * (1 + xmax):
            at_min = True
            continue
        al = np.ones(n, f32)
        side = np.zeros(n, int)
        m1 = fr & (d < 0) & (x + d < Lf)
        m2 = fr & (d > 0) & (x + d > Uf) & ~m1
        al = np.where(m1, (Lf - x) / np.where(d == 0, 1, d), np.where(m2, (Uf - x) / np.where(d == 0, 1, d), al))
        side = np.where(m1, 1, np.where(m2, 2, 0))
        al = np.maximum(al, 0).astype(f32)
        amin = al.min()
        if amin < 1:
            blk = int(np.argmax(-al))
            x = np.where(fr, x + amin * d, x).astype(f32)
            x[blk] = Lf[blk] if side[blk] == 1 else Uf[blk]
            ws[blk] = side[blk]
        else:
            x = np.where(fr, x + d, x).astype(f32)
            at_min = True
    if not conv and BEST:
        x = best_x
    if not conv and BPP and phase == 1 and Lf is not None:
        x = np.minimum(np.maximum(x, Lf), Uf).astype(f32)
    return x, solves, conv


if __name__ == "__main__" and len(sys.argv) > 7:
    for ps, ms in ((20, 16), (20, 24), (10, 24), (50, 24)):
        ev, its, nc = [], [], 0
        for p in probs:
            x, used, conv = wave_exact(p, pgs_sweeps=ps, max_solves=ms)
            dx = x.astype(np.float64) - p["x"]
            ev.append(np.abs(p["A"] @ dx).max())
            its.append(used)
            nc += not conv
        ev, its = np.array(ev), np.array(its)
        print(f"wave_exact pgs {ps} max_solves {ms}: |A dx| median {np.median(ev):.2e} p99 {np.percentile(ev, 99):.2e} "
              f"max {ev.max():.2e}; solves mean {its.mean():.2f} p99 {np.percentile(its, 99)} max {its.max()}; "
              f"unconverged {nc}/{len(probs)}")
