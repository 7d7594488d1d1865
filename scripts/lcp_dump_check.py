#!/usr/bin/env python3
"""Why did a dumped exact LCP count as unconverged?  

Reads gpurun_out/{wave,scene}_dump.npz (scripts/wave_prof.py on a debug build
with -DMW_WAVE_PROF -DMW_DUMP_FAIL) and, for every dumped world-step:
  * re-solves both of DART's stages in fp64 (a textbook primal active-set
    method; the Delassus matrix as the kernel held it, CFM included),
  * evaluates the kernel's own convergence measure (wave_lcp.hpp
    lcp_row_residual: residual / (kLcpRelTol (|b| + sum |A_rc x_c|) + kLcpAbsTol))
    for the kernel's answer, for the fp64 answer, and for the fp64 answer
    rounded to fp32 -- the best any fp32 iterate can do,
  * prints cond(A) and the distance between the kernel's and the fp64 answer.
A world-step whose fp32-rounded exact answer already misses the measure is
beyond fp32 (a tolerance question), one whose kernel answer is far from the
fp64 answer is a solver failure.
"""
import sys

import numpy as np

REL, ABS = 1e-6, 1e-8


def row_measure(A, b, x, lo, hi):
    w = A @ x
    mag = np.abs(A) @ np.abs(x)
    s = b - w
    tolx = 2e-6 * (1 + np.max(np.abs(x)))
    e = np.zeros_like(b)
    for r in range(len(b)):
        L, U = lo[r], hi[r]
        if x[r] < L - tolx or x[r] > U + tolx:
            e[r] = ((L - x[r]) if x[r] < L else (x[r] - U)) * A[r, r]
        elif U - L <= tolx:
            e[r] = 0
        elif x[r] <= L + tolx:
            e[r] = max(s[r], 0)
        elif x[r] >= U - tolx:
            e[r] = max(-s[r], 0)
        else:
            e[r] = abs(s[r])
    return e / (REL * (np.abs(b) + mag) + ABS)


def boxqp64(A, b, lo, hi, x0=None):
    """min 1/2 x'Ax - b'x on the box, primal active set in fp64"""
    n = len(b)
    x = np.clip(np.zeros(n) if x0 is None else x0.astype(np.float64), lo, hi)
    ws = np.where(hi - lo <= 0, 1, np.where(x <= lo, 1, np.where(x >= hi, 2, 0)))
    x = np.where(ws == 1, lo, np.where(ws == 2, hi, x))
    for _ in range(20 * n + 50):
        F = ws == 0
        g = A @ x - b
        xs = x.copy()
        if F.any():
            xs[F] = np.linalg.solve(A[np.ix_(F, F)], b[F] - A[np.ix_(F, ~F)] @ x[~F])
        d = xs - x
        al, blk, side = 1.0, -1, 0
        for r in np.nonzero(F)[0]:
            if d[r] < 0 and xs[r] < lo[r]:
                a = (lo[r] - x[r]) / d[r]
                if a < al: al, blk, side = a, r, 1
            elif d[r] > 0 and xs[r] > hi[r]:
                a = (hi[r] - x[r]) / d[r]
                if a < al: al, blk, side = a, r, 2
        x = x + max(al, 0) * d
        if blk >= 0:
            ws[blk] = side
            x[blk] = lo[blk] if side == 1 else hi[blk]
            continue
        g = A @ x - b
        v = np.where(ws == 1, -g, np.where(ws == 2, g, 0))
        v[hi - lo <= 0] = 0
        r = int(np.argmax(v))
        if v[r] <= 1e-13 * (1 + np.abs(b).max()):
            return x
        ws[r] = 0
    return x


def stages(A, b, lo, hi, kind, mu):
    n = len(b)
    fric = kind == 1
    L1, U1 = np.where(fric, 0, lo), np.where(fric, 0, hi)
    x1 = boxqp64(A, b, L1, U1)
    nrow = np.array([r - r % 3 if fric[r] else r for r in range(n)])
    U2 = np.where(fric, mu * np.maximum(x1[nrow], 0), hi)
    L2 = np.where(fric, -U2, lo)
    x2 = boxqp64(A, b, L2, U2, x1)
    return (L1, U1, x1), (L2, U2, x2), nrow


def main(path):
    d = np.load(path)
    scene = str(d["layout"]) == "scene"
    for k in range(d["A"].shape[0]):
        H, V = d["head"][k], d["V"][k]
        n = int(H[0])
        A = d["A"][k][:n, :n].astype(np.float64)
        A = 0.5 * (A + A.T)
        b, lo, hi = (V[i][:n].astype(np.float64) for i in range(3))
        if scene:
            kind, xg, x1g = V[6][:n], V[5][:n], V[7][:n]
        else:
            kind, xg, x1g = V[3][:n], V[6][:n], V[7][:n]
        mu = float(H[3])
        (L1, U1, x1), (L2, U2, x2), nrow = stages(A, b, lo, hi, kind.astype(int), mu)
        # the kernel's stage-2 boxes come from its own stage-1 normals
        fr = kind.astype(int) == 1
        U2g = np.where(fr, mu * np.maximum(x1g[nrow].astype(np.float64), 0), hi)
        L2g = np.where(fr, -U2g, lo)
        m1g = row_measure(A, b, x1g.astype(np.float64), L1, U1)
        m2g = row_measure(A, b, xg.astype(np.float64), L2g, U2g)
        m1e = row_measure(A, b, x1.astype(np.float32).astype(np.float64), L1, U1)
        m2e = row_measure(A, b, x2.astype(np.float32).astype(np.float64), L2, U2)
        ev = np.linalg.eigvalsh(A)
        print(f"[{k}] n={n} solves={int(H[1])} stage2={int(H[2])} ok={int(H[4])} mu={mu:g} "
              f"cond={ev[-1] / max(ev[0], 1e-300):.2e} kinds n/f/j={np.sum(kind == 0)}/{np.sum(kind == 1)}/{np.sum(kind == 2)}")
        print(f"    stage 1: kernel measure max {m1g.max():.3g} (row {int(m1g.argmax())}), fp64->fp32 {m1e.max():.3g}; "
              f"|x1_gpu - x1_64| {np.abs(x1g - x1).max():.3g} of |x1| {np.abs(x1).max():.3g}")
        print(f"    stage 2: kernel measure max {m2g.max():.3g} (row {int(m2g.argmax())}), fp64->fp32 {m2e.max():.3g}; "
              f"|x_gpu - x_64| {np.abs(xg - x2).max():.3g} of |x| {np.abs(x2).max():.3g}")


if __name__ == "__main__":
    for p in sys.argv[1:] or ["gpurun_out/wave_dump.npz"]:
        print(p)
        main(p)
