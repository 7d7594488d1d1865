"""GPU tests of the scene kernel's large-contact world-steps
(scene_kernel.hip sc_big_constraints): more contact points than the LDS
record holds (32) or more constraint rows than the 64-lane register LCP --
the workspace in HBM, DART's two-stage boxed LCP by block Gauss-Seidel over
64-row exact box QPs -- against the fp64 scene oracle (oracle.c
or_scene_step; exact mode = DART's Dantzig LCP, PGS mode = the same
sweeps).  The reference has no contact cap (World::insertModel,
cpp/scenario/gazebo/src/World.cpp:70-180; DART's step at
cpp/scenario/plugins/Physics/Physics.cpp:1824-1835).

  * eight cubes side by side in face contact on the ground (32 ground
    corners + the box-box face points, 60+ points, 180+ rows), every world a
    different small tilt / velocity: one step in exact mode within 1e-5 (pose,
    contact points) and 1e-4 (velocities) of DART's LCP, unless the fp64
    oracle itself moves as much under an fp32-size perturbation of its inputs;
  * the same row at rest for 300 steps: no drift, 0 unconverged world-steps;
  * PGS mode: the big path's sweeps against the oracle's PGS-50;
  * beyond the large-contact capacity (a 4 x 4 grid of cubes in face
    contact: 152 points) the run still fails loudly (MW_ECAPACITY).
"""

import ctypes

import numpy as np
import pytest

import lcp_validity as LV

from scene_models import cube_urdf, plank_urdf
from test_gpu_scene import _compare, _oracle_from_gpu, _rand_quat, _scene, _Snapshot

pytestmark = pytest.mark.gpu


def _row_scene(W, rng, exact, tilt=0.0, vel=0.05, pgs=50, mu=0.8):
    # (axis-aligned: with near-parallel faces -- tilts of a few mrad -- the
    # box-box SAT's reference face is a near-tie that fp32 and fp64 may break
    # differently, a different but equally valid manifold)
    n = 8
    models = [(cube_urdf(), (0.1999 * k, 0.0, 0.0999, 1, 0, 0, 0), f"c{k}") for k in range(n)]
    sc = _scene(models, W, pgs, mu, exact=exact)
    for m in range(n):
        poses = np.array([np.concatenate([[0.1999 * m + rng.uniform(-2e-4, 2e-4), rng.uniform(-1e-3, 1e-3),
                                           0.0999 + rng.uniform(-2e-4, 1e-4)],
                                          _rand_quat(rng, tilt) if tilt else [1.0, 0.0, 0.0, 0.0]])
                          for _ in range(W)])
        sc.reset_base_pose(m, poses)
        sc.reset_base_velocity(m, np.column_stack([rng.uniform(-vel, vel, (W, 3)), rng.uniform(-10 * vel, 10 * vel, (W, 3))]))
    sc.run(paused=True)
    return sc, n


def _big_ws(sc, w):
    """(final impulses [c][3], stage-1 impulses of the rows) of world w's last
    large-contact step (test hook mw_debug_scene_big_ws)"""
    from mwstep import native as N
    out = np.zeros(20 * 128 + 11 * 512, np.float32)
    cmax, rows = ctypes.c_int32(), ctypes.c_int32()
    assert N.lib().mw_debug_scene_big_ws(sc.handle, w, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(out),
                                         ctypes.byref(cmax), ctypes.byref(rows)) == 0
    ct = out[:20 * cmax.value].reshape(cmax.value, 20).astype(np.float64)
    x1 = out[20 * cmax.value + 4 * rows.value:20 * cmax.value + 5 * rows.value].astype(np.float64)
    return ct[:, 16:19], x1


def _validity(p, x, x1):
    """the GPU's impulses in the oracle's fp64 two-stage problem p
    (pyoracle.lcp_last), as tests/lcp_validity.py measures them: the largest
    complementarity error over the tolerance, stage 1 and stage 2"""
    (L1, U1), (L2, U2) = LV.stage_boxes(p, x1)
    S = p["kind"] != 1
    A, b, bs = p["A"], p["b"], p["bscale"]
    e1, s1 = LV._complementarity(A[np.ix_(S, S)], b[S], L1[S], U1[S], x1[S], bs[S])
    e2, s2 = LV._complementarity(A, b, L2, U2, x, bs)
    return max(float((e1 / (LV.REL_TOL * s1 + LV.ABS_TOL)).max()), float((e2 / (LV.REL_TOL * s2 + LV.ABS_TOL)).max()))


def _one_step(oracle, sc, n, W, pgs, mu, vel_tol):
    cms = [oracle.load_urdf(cube_urdf(), pose_xyz=(0.1999 * k, 0, 0.0999)) for k in range(n)]
    orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
    before = [_Snapshot(sc, w, n) for w in range(W)]
    sc.run()
    unconv = sc.lcp_unconverged()
    print(f"unconverged world-steps {unconv}")
    worst = dict(pose=0.0, vel=0.0, point=0.0)
    ill, ncs, valid = [], [], []
    for w in range(W):
        ow = orcs[w]
        ow.step()
        p = oracle.lcp_last() if pgs < 0 else None
        e = _compare(oracle, cms, sc, ow, w)
        gc = sc.contacts(w)
        ncs.append(len(gc))
        assert len(gc) == len(ow.contacts), (w, len(gc), len(ow.contacts))
        for row, (oc, who) in zip(gc, ow.contacts):
            assert tuple(int(v) for v in row[10:14]) == who
            e["point"] = max(e.get("point", 0.0), float(np.abs(row[0:3] - oc[0:3]).max()))
        if e["vel"] > vel_tol and p is not None:
            # exact mode: a different answer is accepted only as a solution of
            # the fp64 LCP (tests/lcp_validity.py) -- the
            # stage-1 normals of redundant contacts (cond(A) ~ 1e6) are set
            # to within the tolerance only, and the friction boxes follow them
            xg, x1g = _big_ws(sc, w)
            nr = len(p["b"])
            x = xg[:nr // 3].reshape(-1)
            ratio, ratio_or = _validity(p, x, x1g[:nr]), LV.oracle_ratio(p)
            valid.append((w, round(e["vel"], 6), round(ratio, 2), round(ratio_or, 2)))
            assert ratio <= LV.ACCEPT, f"world {w}: {e}, GPU LCP residual ratio {ratio:.2f} (oracle {ratio_or:.2f})"
            e["vel"] = 0.0
        elif e["vel"] > vel_tol:
            sens = 0.0
            for k in range(4):
                ow2 = _oracle_from_gpu(oracle, cms, before[w], 0, pgs, mu, 3e-7, k)
                ow2.step()
                for m in range(n):
                    sens = max(sens, float(np.abs(ow2.V(m) - ow.V(m)).max()))
            ill.append((w, round(e["vel"], 6), round(sens, 6)))
            if sens < 0.05 * e["vel"]:
                # diagnostics: impulses per contact row, GPU (from the contact forces) vs oracle
                for c, (row, (oc, who)) in enumerate(zip(gc, ow.contacts)):
                    n = row[3:6]
                    fg, fo = row[6:9] * 1e-3, oc[6:9] * 1e-3
                    if np.abs(fg - fo).max() > 1e-4:
                        print(f"  contact {c} who {who} depth {row[9]:.2e} x_gpu {fg} x_or {fo} n {n}")
            assert sens >= 0.05 * e["vel"], f"world {w}: {e}, oracle sensitivity {sens:.2e}"
            e["vel"] = 0.0
        for k in worst:
            worst[k] = max(worst[k], e.get(k, 0.0))
    print(f"different velocities accepted as fp64 LCP solutions (world, gap, GPU ratio, oracle ratio): {valid}")
    return worst, ill, ncs


def test_eight_cubes_in_a_row_one_step_exact(require_gpu, oracle):
    W, mu = 32, 0.8
    rng = np.random.default_rng(11)
    sc, n = _row_scene(W, rng, exact=True, mu=mu)
    worst, ill, ncs = _one_step(oracle, sc, n, W, -1, mu, 1e-4)
    print(f"8 cubes x{W} exact: contacts {min(ncs)}..{max(ncs)}, one-step " +
          ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) + f", ill {ill[:6]}")
    assert min(ncs) > 32                     # every world took the large-contact path
    assert len(ill) <= W // 8
    assert worst["pose"] <= 1e-5 and worst["point"] <= 1e-5 and worst["vel"] <= 1e-4
    assert sc.overflow() == 0 and sc.lcp_unconverged() == 0
    sc.close()


def test_eight_cubes_in_a_row_one_step_pgs(require_gpu, oracle):
    W, mu, pgs = 16, 0.8, 50
    rng = np.random.default_rng(12)
    sc, n = _row_scene(W, rng, exact=False, mu=mu, pgs=pgs)
    worst, ill, ncs = _one_step(oracle, sc, n, W, pgs, mu, 2e-3)
    print(f"8 cubes x{W} PGS-{pgs}: contacts {min(ncs)}..{max(ncs)}, one-step " +
          ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) + f", ill {ill[:6]}")
    assert min(ncs) > 32
    assert len(ill) <= W // 8
    assert worst["pose"] <= 1e-5 and worst["point"] <= 1e-5 and worst["vel"] <= 2e-3
    assert sc.overflow() == 0
    sc.close()


def test_eight_cubes_in_a_row_rest(require_gpu, oracle):
    """The row settling for 300 steps (exact mode) next to the fp64 oracle's
    run of world 0: the overlapping faces push the cubes apart at DART's
    capped contact correction (1e-3 m/s: the oracle's |v| is 0.96e-3 to
    1.22e-3 over the run), nothing sinks, 0 unconverged world-steps."""
    W, n = 4, 8
    rng = np.random.default_rng(13)
    sc, n = _row_scene(W, rng, exact=True, vel=0.0)
    cms = [oracle.load_urdf(cube_urdf(), pose_xyz=(0.1999 * k, 0, 0.0999)) for k in range(n)]
    ow = _oracle_from_gpu(oracle, cms, sc, 0, -1, 0.8)
    for _ in range(300):
        sc.run()
        ow.step()
    z = np.array([sc.base_pose(m, 0, W)[:, 2] for m in range(n)])
    v = np.array([sc.base_velocity(m, 0, W) for m in range(n)])
    dp = max(float(np.abs(sc.base_pose(m, 0, 1)[0][:3] - ow.p(m)).max()) for m in range(n))
    vo = max(float(np.abs(ow.V(m)).max()) for m in range(n))
    print(f"8 cubes settling, 300 steps: z {z.min():.6f}..{z.max():.6f}, |v| max {np.abs(v).max():.2e} "
          f"(oracle {vo:.2e}), world 0 position vs oracle {dp:.2e}, contacts {len(sc.contacts(0))}")
    assert len(sc.contacts(0)) > 32
    assert np.abs(z - 0.1).max() <= 2e-4
    assert np.abs(v).max() <= 2e-3 and dp <= 1e-4
    assert sc.overflow() == 0 and sc.lcp_unconverged() == 0
    sc.close()


def test_beyond_large_contact_capacity_fails_loudly(require_gpu):
    """Eight planks of two cubes tiling a 4 x 4 grid flat on the ground, every
    cube in face contact with its neighbours (64 ground points + 88 box-box
    points in the fp64 oracle, above the 128 of the large-contact workspace):
    points are dropped and the synchronous run reports it (MW_ECAPACITY ->
    RuntimeError) instead of stepping on silently."""
    from mwstep import native as N
    sp = 0.1999
    models = [(plank_urdf(2), ((2 * (p % 2) + 0.5) * sp, (p // 2) * sp, 0.0999, 1, 0, 0, 0), f"p{p}")
              for p in range(8)]
    sc = _scene(models, 2)
    with pytest.raises(RuntimeError, match="capacity"):
        sc.run()
    assert sc.overflow() > 0
    assert "dropped" in N.lib().mw_last_error().decode()
    sc.close()
