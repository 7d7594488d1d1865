"""Prototype (numpy, float32 arithmetic) of the wave kernel's exact boxed-LCP
solve in DART's two stages (wave_lcp.hpp, oracle.c lcp_dantzig), run on LCPs
captured from iCub-class (models/icub.urdf) drops / slides (pyoracle.lcp_last).  Mirrors the
device algorithm so the linear-solve counts and fp32 errors seen here are the
kernel's:  per stage, PGS sweeps on the stage's box problem (tolerance exit
1e-6 on the constraint velocities), then semismooth Newton (held rows: at a
bound with the gradient pushing out), a monotone line search on the largest
residual, the primal active-set method when a step fails, refinement solves
on a working set whose minimiser misses the tolerance.

    python scripts/proto_dantzig.py [n_worlds] [steps]      (env: MODE, SWEEPS, BUDGET, REFINE, F64)

MODE was (the kernel's method since r04d): the primal active-set method from
the previous step's working set (rows without a record take the PGS point's
class); ssn / tol / as: the r04c starts measured against it on a standing
humanoid (3 x 150 steps; stage-2 solves per LCP, unconverged of 450):
ssn 6.7 / 78, as 6.1 / 78 (3.2 / 0 with the release test on each row's own
tolerance), was 1.2 / 0 with 10 sweeps.  F64=1 solves in float64: no change,
the stall was never the fp32 elimination.
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
import pyoracle  # noqa: E402


def capture(n_worlds=8, steps=60, seed=21):
    """iCub-class (models/icub.urdf) drops / slides under a PD hold in the fp64 oracle (DART's LCP):
    [((world, step), lcp)] (proto_lcp_exact.capture with the world index)"""
    from mwstep import get_model_file
    from mwstep.models import icub_pid_gains, icub_posture
    cm = pyoracle.load_urdf(get_model_file("icub"), pose_xyz=(0, 0, 0.572), pose_wxyz=(0, 0, 0, 1))
    post = np.array(icub_posture(cm.joint_names))
    n = cm.n
    rng = np.random.default_rng(seed)
    kp, kd = np.array(icub_pid_gains(cm.joint_names)).T
    lo, hi = np.array(cm.model.lower[:n]), np.array(cm.model.upper[:n])
    out = []
    for w in range(n_worlds):
        ow = pyoracle.FloatWorld(cm, ground=True, mu=1.0, pgs_iters=pyoracle.PGS_CONVERGED)
        ang = rng.uniform(0, 0.08)
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        c, s_ = np.cos(ang), np.sin(ang)
        K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = np.eye(3) + s_ * K + (1 - c) * K @ K
        ow.set_pose([0, 0, 0.572 + rng.uniform(0, 0.09)], R)
        ow.set_twist(R.T @ rng.uniform(-0.3, 0.3, 3),
                     R.T @ np.array([*rng.uniform(-0.8, 0.8, 2), rng.uniform(-0.5, 0)]))
        ow.set_joints(np.clip(post + rng.uniform(-0.1, 0.1, n), lo, hi), rng.uniform(-0.5, 0.5, n))
        mode = np.full(n, pyoracle.FORCE, np.int32)
        for k in range(steps):
            tau = np.clip(-kp * (ow.q - post) - kd * ow.qd, -80, 80)
            ow.step(mode, tau)
            p = pyoracle.lcp_last()
            if p is not None and len(p["b"]) > 0:
                out.append(((w, k), p))
    return out

f32 = np.float32
REL, ABS = float(os.environ.get("REL", "1e-6")), float(os.environ.get("ABS", "1e-7"))
FLOOR = os.environ.get("FLOOR", "1") != "0"
MINSOLVE = os.environ.get("MINSOLVE", "0") != "0"
SWEEPS = int(os.environ.get("SWEEPS", "50"))
BUDGET = int(os.environ.get("BUDGET", "24"))
REFINE = int(os.environ.get("REFINE", "1"))
# MODE ssn: semismooth Newton first (held: at a bound, gradient outward);
#      tol: the same with bound / gradient tests within the tolerance;
#      as: the primal active-set method from the start (working set = rows at a bound)
MODE = os.environ.get("MODE", "ssn")


def matvec(A, x):
    """compensated fp32 matvec ~ the fp64 sum rounded once"""
    w = (A.astype(np.float64) @ x.astype(np.float64)).astype(f32)
    mag = (np.abs(A.astype(np.float64) * x.astype(np.float64)[None, :]).sum(axis=1)).astype(f32)
    return w, mag


def residual(A, b, x, L, U, arr):
    w, mag = matvec(A, x)
    s = b - w
    tolx = f32(2e-6) * (f32(1) + np.abs(x).max(initial=0))
    e = np.zeros_like(x)
    out = (x < L - tolx) | (x > U + tolx)
    e[out] = np.where(x[out] < L[out], L[out] - x[out], x[out] - U[out]) * arr[out]
    pin = ~out & (U - L <= tolx)
    lo = ~out & ~pin & (x <= L + tolx)
    hi = ~out & ~pin & ~lo & (x >= U - tolx)
    fr = ~out & ~pin & ~lo & ~hi
    e[lo] = np.maximum(s[lo], 0)
    e[hi] = np.maximum(-s[hi], 0)
    e[fr] = np.abs(s[fr])
    rel = e / (REL * (np.abs(b) + mag) + ABS)
    return rel.max(initial=0), e, w


def pgs(A, b, L, U, x, sweeps):
    n = len(b)
    for _ in range(sweeps):
        w0 = A @ x
        for r in range(n):
            v = x[r] + (b[r] - A[r] @ x) / A[r, r]
            x[r] = min(max(v, L[r]), U[r])
        if np.abs(A @ x - w0).max(initial=0) <= 1e-6:
            break
    return x


def ge_nopivot(K, r):
    """fp32 Gaussian elimination in row order without pivoting (the kernel's
    lcp_ge_solve with pivot = false), back substitution"""
    K = K.astype(f32).copy()
    r = r.astype(f32).copy()
    n = len(r)
    for j in range(n):
        piv = K[j, j] if abs(K[j, j]) >= 1e-30 else f32(1e-30)
        f = (K[j + 1:, j] / piv).astype(f32)
        K[j + 1:, j:] = (K[j + 1:, j:] - np.outer(f, K[j, j:])).astype(f32)
        r[j + 1:] = (r[j + 1:] - f * r[j]).astype(f32)
    d = np.zeros(n, f32)
    for j in range(n - 1, -1, -1):
        d[j] = (r[j] - np.dot(K[j, j + 1:], d[j + 1:]).astype(f32)) / K[j, j]
    return d


def boxqp(A, b, L, U, x, budget, stats, ws0=None):
    n = len(b)
    arr = np.diag(A).copy()
    pinned = (U - L) <= 0
    phase, ws, at_min = 0, np.zeros(n, int), False
    if ws0 is not None:
        phase = 1
        tolx0 = f32(2e-6) * (f32(1) + np.abs(x).max(initial=0))
        wpgs = np.where(x <= L + tolx0, 1, np.where(x >= U - tolx0, 2, 0))
        ws = np.where(pinned, 1, np.where(ws0 < 0, wpgs, ws0))
        x = np.where(ws == 1, L, np.where(ws == 2, U, x)).astype(f32)
    elif MODE == "as":
        tolx0 = f32(2e-6) * (f32(1) + np.abs(x).max(initial=0))
        phase = 1
        ws = np.where(pinned, 1, np.where(x <= L + tolx0, 1, np.where(x >= U - tolx0, 2, 0)))
        x = np.where(ws == 1, L, np.where(ws == 2, U, x)).astype(f32)
    solves = 0
    for _ in range(4 * budget + 8):
        rel, e, w = residual(A, b, x, L, U, arr)
        g = w - b
        if rel <= 1 and (solves > 0 or not MINSOLVE or not (~pinned & (ws == 0)).any()):
            return x, solves, True
        if phase == 1 and at_min:
            at_min = False
            tiny_last_ = stats.get("_tiny", False)
            v = np.where(ws == 1, -g, np.where(ws == 2, g, 0)).astype(f32)
            v[pinned] = 0
            v = v / (REL * (np.abs(b) + matvec(A, x)[1]) + ABS)
            if v.max(initial=0) > 1:
                if os.environ.get("MULTI", "0") != "0":
                    ws[v > 1] = 0   # every wrongly signed multiplier at once
                else:
                    ws[int(np.argmax(v))] = 0
                stats["_tiny"] = False
                continue
            if tiny_last_ and FLOOR:
                # the last solve on this working set was a refinement that moved
                # nothing: the fp32 floor
                stats["floor"] = stats.get("floor", 0) + 1
                return x, solves, rel <= 64
            if not REFINE:
                return x, solves, False
        if solves >= budget:
            return x, solves, False
        if phase == 0 and MODE == "tol":
            tolx = f32(2e-6) * (f32(1) + np.abs(x).max(initial=0))
            tg = REL * (np.abs(b) + matvec(A, x)[1]) + ABS
            held = pinned | ((x <= L + tolx) & (g >= -tg)) | ((x >= U - tolx) & (g <= tg))
        elif phase == 0:
            held = pinned | ((x <= L) & (g >= 0)) | ((x >= U) & (g <= 0))
        else:
            held = pinned | (ws != 0)
        fr = ~held
        d = np.zeros(n, f32)
        if fr.any():
            dt = np.float64 if os.environ.get("F64", "0") != "0" else f32
            if os.environ.get("NOPIV", "0") != "0":
                d[fr] = ge_nopivot(A[np.ix_(fr, fr)], -g[fr])
            else:
                d[fr] = np.linalg.solve(A[np.ix_(fr, fr)].astype(dt), (-g[fr]).astype(dt)).astype(f32)
        solves += 1
        stats["solve_rows"].append(int(fr.sum()))
        if phase == 0:
            emax = e.max(initial=0)
            ok = False
            step = f32(1)
            for _ls in range(4):
                xt = np.clip(x + step * d, L, U).astype(f32)
                _, et, _ = residual(A, b, xt, L, U, arr)
                if et.max(initial=0) < emax:
                    x, ok = xt, True
                    break
                step *= f32(0.5)
            if not ok:
                stats["fallback"] += 1
                phase = 1
                ws = np.where(pinned, 1, np.where(x <= L, 1, np.where(x >= U, 2, 0)))
                at_min = False
            continue
        if np.abs(d).max(initial=0) <= 1e-7 * (1 + np.abs(x).max(initial=0)):
            at_min = True
            stats["_tiny"] = True
            continue
        stats["_tiny"] = False
        al = np.ones(n, f32)
        lo_hit = fr & (d < 0) & (x + d < L)
        hi_hit = fr & (d > 0) & (x + d > U)
        al[lo_hit] = (L[lo_hit] - x[lo_hit]) / d[lo_hit]
        al[hi_hit] = (U[hi_hit] - x[hi_hit]) / d[hi_hit]
        al = np.maximum(al, 0)
        amin = al.min(initial=1)
        if amin < 1 and os.environ.get("PROJ", "0") != "0":
            # projected full step: every row the full step pushes past a bound
            # joins the working set there, if the objective still decreases
            obj = lambda v: float(0.5 * v.astype(np.float64) @ (A.astype(np.float64) @ v.astype(np.float64))
                                  - b.astype(np.float64) @ v.astype(np.float64))
            xp = np.where(fr, np.clip(x + d, L, U), x).astype(f32)
            if obj(xp) < obj(x):
                hit = lo_hit | hi_hit
                ws = np.where(lo_hit, 1, np.where(hi_hit, 2, ws))
                x = xp
                stats["proj"] = stats.get("proj", 0) + 1
                continue
            blk = int(np.argmin(al))
            x = np.where(fr, x + amin * d, x).astype(f32)
            x[blk] = L[blk] if lo_hit[blk] else U[blk]
            ws[blk] = 1 if lo_hit[blk] else 2
        elif amin < 1:
            blk = int(np.argmin(al))
            x = np.where(fr, x + amin * d, x).astype(f32)
            x[blk] = L[blk] if lo_hit[blk] else U[blk]
            ws[blk] = 1 if lo_hit[blk] else 2
        else:
            x = np.where(fr, x + d, x).astype(f32)
            at_min = True
    return x, solves, False


def solve(p, x_final_prev, x1_prev, stats, prev_active=False):
    A = p["A"].astype(f32)
    b = p["b"].astype(f32)
    kind = p["kind"]
    mu = f32(p["mu"])
    n = len(b)
    fric = kind == 1
    nrow = np.array([r - r % 3 if kind[r] == 1 else r for r in range(n)])
    big = f32(3.4e38)
    lo = np.where(kind == 0, 0, np.where(kind == 2, p["lo"], 0)).astype(f32)
    hi = np.where(kind == 0, big, np.where(kind == 2, p["hi"], 0)).astype(f32)
    # stage 1
    L1, U1 = np.where(fric, 0, lo).astype(f32), np.where(fric, 0, hi).astype(f32)
    warm = MODE in ("was", "was2")
    # was2: the record marks rows active last step (a zero impulse included):
    # a zero normal starts held at 0, a zero friction row free; PGS only when
    # some row has no record (a new contact)
    marked = MODE == "was2" and prev_active
    tolc = lambda v: f32(2e-6) * (f32(1) + np.abs(v).max(initial=0))
    x = np.clip(x1_prev, L1, U1).astype(f32)
    ws1 = None
    if warm:
        t = tolc(x1_prev)
        ws1 = np.where(x1_prev <= L1 + t, 1, np.where(x1_prev >= U1 - t, 2, 0))
        ws1 = np.where(x1_prev == 0, (np.where(fric, 0, 1) if marked else -1), ws1)
    if SWEEPS and not marked:
        x = pgs(A, b, L1, U1, x, SWEEPS).astype(f32)
    x, s1, ok1 = boxqp(A, b, L1, U1, x, BUDGET, stats, ws1)
    x1 = x.copy()
    # stage 2
    u = mu * np.maximum(x[nrow], 0)
    L2 = np.where(fric, -u, L1).astype(f32)
    U2 = np.where(fric, u, U1).astype(f32)
    ws2 = None
    if warm:
        x = np.clip(x_final_prev, L2, U2).astype(f32)
        up = mu * np.maximum(x1_prev[nrow], 0)
        Lp, Up = np.where(fric, -up, L1), np.where(fric, up, U1)
        t = tolc(x_final_prev)
        ws2 = np.where(x_final_prev <= Lp + t, 1, np.where(x_final_prev >= Up - t, 2, 0))
        ws2 = np.where((x_final_prev == 0) | (Up - Lp <= 0), (np.where(fric, 0, 1) if marked else -1), ws2)
    else:
        x = np.where(fric, np.clip(x_final_prev, L2, U2), x).astype(f32)
    if SWEEPS and not marked:
        x = pgs(A, b, L2, U2, x, SWEEPS).astype(f32)
    x, s2, ok2 = boxqp(A, b, L2, U2, x, BUDGET - s1, stats, ws2)
    return x, x1, s1, s2, ok1 and ok2


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    probs = capture(W, T)
    stats = {"solve_rows": [], "fallback": 0}
    s1s, s2s, bad, errs = [], [], 0, []
    prev = {}
    for (w, k), p in probs:
        n = len(p["b"])
        xf, x1p = prev.get(w, (np.zeros(n, f32), np.zeros(n, f32)))
        if len(xf) != n:
            xf, x1p = np.zeros(n, f32), np.zeros(n, f32)
        x, x1, s1, s2, ok = solve(p, xf, x1p, stats)
        prev[w] = (x, x1)
        s1s.append(s1)
        s2s.append(s2)
        bad += not ok
        errs.append(np.abs(x - p["x"]).max() / (1 + np.abs(p["x"]).max()))
    s1s, s2s = np.array(s1s), np.array(s2s)
    print(f"{len(probs)} LCPs: solves stage 1 mean {s1s.mean():.2f} max {s1s.max()}, stage 2 mean {s2s.mean():.2f} "
          f"max {s2s.max()}; > 4 total: {(s1s + s2s > 4).sum()}; unconverged {bad}; fallbacks {stats['fallback']}; "
          f"max rel impulse err vs oracle {max(errs):.2e}")


if __name__ == "__main__":
    main()
