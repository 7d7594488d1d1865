"""Is a GPU contact answer a solution of the fp64 LCP?  (test helper)

VERDICT r5 item 1: a world whose GPU velocities differ from the fp64
oracle's is accepted only when the GPU's own impulses -- read back from the
warm-start record (mw_get_state: per contact slot / joint row the final
impulses, then DART's stage-1 impulses) -- are themselves a solution of the
oracle's fp64 two-stage problem (pyoracle.lcp_last: A with DART's CFM, b,
boxes, row identities), i.e. of DART's boxed LCP as the oracle restates it
(oracle.c lcp_dantzig; DantzigBoxedLcpSolver / ODE dSolveLCP with the
friction index [EXT], called from Physics.cpp:1824-1835):

  stage 1: rows S without a friction index (contact normals in [0, inf),
           joint rows in their boxes), friction impulses 0;
  stage 2: every row, each friction box [-mu x1_n, mu x1_n] built from its
           contact's STAGE-1 normal impulse.

For each stage and row the complementarity error e_r is measured in velocity
units exactly as the oracle's lcp_residual does (free rows |s_r|, rows on a
bound the wrongly signed part of s_r, a bound violation times A_rr;
s = b - A x), and compared with the kernel's own convergence tolerance
(wave_lcp.hpp: 1e-6 (|b_r| + sum_c |A_rc x_c|) + 1e-8, MW_LCP_REL_TOL /
MW_LCP_ABS_TOL) widened by the same 1e-6 of the terms b_r is formed from
(bscale_r = sum_e |J_re nu_e| + the bias velocity, or_lcp_last_rows): the
GPU's b comes out of an fp32 articulated-body pass, so its rounding error
scales with those terms, not with |b_r| (a joint-limit row's b = -qd + bias
nearly cancels).  ratio = max_r e_r / tol_r.  ratio <= 1 means the GPU
impulses are the exact DART solution of an LCP whose A and b differ from the
fp64 ones by at most 1e-6 relative to their terms, entry by entry (the
componentwise backward error of an fp32 computation: 17 roundings of 6e-8)
-- where the fp64 LCP's answer itself moves by more than the north star's
1e-4 under such a perturbation (cond(A) ~ 1e7 on redundant contacts) the two
answers are both valid and the velocity gap is not a bug.  The friction boxes
use mu in fp32, as the kernel does.
"""

import numpy as np

REL_TOL, ABS_TOL = 1e-6, 1e-8        # wave_lcp.hpp MW_LCP_REL_TOL / MW_LCP_ABS_TOL
# Acceptance: ratio <= 4, i.e. a componentwise backward error of at most
# 4e-6 relative -- 64 fp32 roundings (gamma_64 = 64 u), the error budget of
# the articulated-body recursion that forms A and b in fp32 over the
# humanoid's 38 coordinates and 10 tree levels.  The kernel's own residual
# test (1e-6, on its own fp32 A and b) cannot see the forward error of A and
# b themselves; measured on the r06 probes (scripts/lcp_validity_probe.py),
# worlds whose GPU answer equals the oracle's to five digits reach ratio 3.0
# on joint-limit rows, and every other GPU answer stays below 1.
ACCEPT = 4.0
SLOTS, JOINT_ROWS = 32, 3 * 48       # kMaxFloatSlots, 3 kMaxBodies (wave_tree.hpp warm record)
WORDS = 3 * SLOTS + JOINT_ROWS
OR_WARM_JOINT0 = 3 * 128             # oracle.h OR_WARM_JOINT0 (3 OR_MAXFC)


def warm_records(state_row):
    """(final, stage-1) impulses by the kernels' row identity from one world's
    mw_get_state record (the warm record is its last 2 WORDS floats)."""
    rec = np.asarray(state_row[-2 * WORDS:], dtype=np.float64)
    return rec[:WORDS], rec[WORDS:]


def gpu_index(wid):
    """oracle row identity -> index into the kernels' warm record (-1: none)."""
    if wid < 0:
        return -1
    if wid < OR_WARM_JOINT0:
        return wid if wid < 3 * SLOTS else -1
    j = wid - OR_WARM_JOINT0
    return 3 * SLOTS + j if j < JOINT_ROWS else -1


def _complementarity(A, b, L, U, x, bscale=0.0):
    """Per-row complementarity error (velocity units, as oracle.c
    lcp_residual) and the row's tolerance scale
    |b_r| + sum_c |A_rc x_c| + bscale_r."""
    s = b - A @ x
    scale = np.abs(b) + np.abs(A) @ np.abs(x) + bscale
    tx = 5e-7 * np.maximum(np.abs(L), np.abs(U), where=np.isfinite(L) & np.isfinite(U),
                           out=np.abs(x).copy()) + 1e-12
    e = np.zeros(len(b))
    for r in range(len(b)):
        if x[r] < L[r] - tx[r] or x[r] > U[r] + tx[r]:
            e[r] = (L[r] - x[r] if x[r] < L[r] else x[r] - U[r]) * A[r, r]
        elif U[r] - L[r] <= tx[r]:
            e[r] = 0.0              # a pinned row (friction of an unloaded contact)
        elif x[r] <= L[r] + tx[r]:
            e[r] = max(s[r], 0.0)
        elif x[r] >= U[r] - tx[r]:
            e[r] = max(-s[r], 0.0)
        else:
            e[r] = abs(s[r])
    return e, scale


def stage_boxes(p, x1):
    """Stage-1 bounds of every row and stage-2 bounds from the stage-1 normals
    (friction row r belongs to the contact whose normal is row r - r % 3:
    contact rows come first, three per contact, oracle.c or_float_step_warm)."""
    kind = p["kind"]
    L1 = np.where(kind == 0, 0.0, p["lo"])
    U1 = np.where(kind == 0, np.inf, p["hi"])
    mu32 = float(np.float32(p["mu"]))
    L2, U2 = L1.copy(), U1.copy()
    for r in np.flatnonzero(kind == 1):
        u = mu32 * max(x1[r - r % 3], 0.0)
        L2[r], U2[r] = -u, u
    return (L1, U1), (L2, U2)


# Contact detection (a box corner or sphere point below z = 0 at the start of
# the step, Physics.cpp -> ODE/DART [EXT]) is a threshold: a point grazing
# the plane within the fp32 resolution of its world position (~1e-7 m) can be
# a contact for one precision and not the other.  GRAZE bounds that window.
GRAZE = 1e-6


def contact_set_gap(or_contacts, gpu_contacts, tol=1e-5):
    """Contacts of the oracle's step that the GPU did not detect and the
    GPU's that the oracle did not, matched by world point: ([oracle contact
    index, depth], [GPU contact index, depth]).  or_contacts: FloatWorld
    .contacts (point, force, depth, body); gpu_contacts: Simulator.contacts
    rows (point 3, normal 3, force 3, depth)."""
    gp = [np.asarray(r[:3], dtype=float) for r in gpu_contacts]
    op = [np.asarray(c[0], dtype=float) for c in or_contacts]
    only_or = [(i, float(c[2])) for i, c in enumerate(or_contacts)
               if not any(np.abs(op[i] - g).max() <= tol for g in gp)]
    only_gpu = [(i, float(r[9])) for i, r in enumerate(gpu_contacts)
                if not any(np.abs(gp[i] - o).max() <= tol for o in op)]
    return only_or, only_gpu


def drop_contacts(p, contacts):
    """The oracle's problem without the rows of the given contacts (contact
    c owns rows 3c .. 3c + 2: contact rows come first, in detection order)."""
    keep = np.ones(len(p["b"]), bool)
    for c in contacts:
        keep[3 * c:3 * c + 3] = False
    q = {k: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == keep.shape else v) for k, v in p.items()}
    q["A"] = p["A"][np.ix_(keep, keep)]
    return q


def validity(p, state_row):
    """dict(ratio1, ratio2, ratio, missing) for one world: the GPU's stage-1
    and final impulses in the oracle's fp64 problem p (pyoracle.lcp_last
    right after the oracle's step from the same start).  `missing` = the
    largest GPU impulse on a row the oracle's problem does not have (a
    contact the fp64 detection did not produce), 0 if none."""
    fin, st1 = warm_records(state_row)
    idx = np.array([gpu_index(int(w)) for w in p["wid"]])
    assert (idx >= 0).all(), "an oracle row outside the kernels' warm record"
    x = fin[idx]
    x1 = st1[idx]
    extra = np.ones(WORDS, bool)
    extra[idx] = False
    missing = float(np.abs(np.concatenate([fin[extra], st1[extra]])).max()) if extra.any() else 0.0
    (L1, U1), (L2, U2) = stage_boxes(p, x1)
    S = p["kind"] != 1
    A, b = p["A"], p["b"]
    bs = p["bscale"]
    e1, s1 = _complementarity(A[np.ix_(S, S)], b[S], L1[S], U1[S], x1[S], bs[S])
    e2, s2 = _complementarity(A, b, L2, U2, x, bs)
    r1 = float((e1 / (REL_TOL * s1 + ABS_TOL)).max()) if S.any() else 0.0
    r2 = float((e2 / (REL_TOL * s2 + ABS_TOL)).max())
    return dict(ratio1=r1, ratio2=r2, ratio=max(r1, r2), missing=missing, x=x, x1=x1, e1=e1, e2=e2,
                tol1=REL_TOL * s1 + ABS_TOL, tol2=REL_TOL * s2 + ABS_TOL)


def oracle_ratio(p):
    """The same measure of the oracle's own fp64 answer (p["x"], p["x1"])."""
    (L1, U1), (L2, U2) = stage_boxes(p, p["x1"])
    S = p["kind"] != 1
    A, b = p["A"], p["b"]
    bs = p["bscale"]
    e1, s1 = _complementarity(A[np.ix_(S, S)], b[S], L1[S], U1[S], p["x1"][S], bs[S])
    e2, s2 = _complementarity(A, b, L2, U2, p["x"], bs)
    r1 = float((e1 / (REL_TOL * s1 + ABS_TOL)).max()) if S.any() else 0.0
    return max(r1, float((e2 / (REL_TOL * s2 + ABS_TOL)).max()))


def judge(p, or_contacts, gpu_contacts, state_row):
    """Is the GPU's step, which differs from the oracle's, a valid fp64 LCP
    answer?  (ok, ratio, grazing): the contact sets may differ only by points
    within GRAZE of the ground; an oracle-only grazing point's rows are
    dropped from the problem before the GPU impulses are checked in it; a
    GPU-only grazing point has no row in the oracle's problem (ok, ratio
    nan: the callers count these, they cannot be checked); any other
    difference of the contact sets is not ok."""
    only_or, only_gpu = contact_set_gap(or_contacts, gpu_contacts)
    grazing = [("oracle", dep) for _, dep in only_or] + [("GPU", dep) for _, dep in only_gpu]
    if any(dep > GRAZE for _, dep in grazing):
        return False, float("nan"), grazing
    if only_gpu:
        return True, float("nan"), grazing
    if p is None:
        return not only_or, 0.0, grazing
    if only_or:
        p = drop_contacts(p, [c for c, _ in only_or])
    v = validity(p, state_row)
    return v["ratio"] <= ACCEPT and v["missing"] == 0.0, v["ratio"], grazing
