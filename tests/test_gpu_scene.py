"""GPU tests of scenes (several models per world; csrc/scene_kernel.hip via
include/mwscene.h) against the fp64 scene oracle (oracle.c or_scene_step)
and the reference's multi-model KATs:

  * teacher-forced one-step parity over 256 worlds, each a different random
    arrangement of cubes, a ball and a floating 3-link chain dropped onto
    each other and the ground (box-box face / edge contacts, box-sphere,
    sphere-ground, random torques): poses within 1e-5, velocities within 2e-3
    (the contact tolerance of test_gpu_float_tree.py, same ill-conditioning
    probe), contact points within 1e-5;
  * a welded (fixed-base) Panda next to a falling cube: the Panda's joints
    follow the oracle;
  * the three-cube KAT of tests/test_scenario/test_contacts.py:125-236, both
    collision variants, cube3 inserted after 50 steps (mid-run insertion);
  * world wrenches (Link::applyWorldForce, Link.cpp:484-560): v = F t / m
    for exactly max(1, ceil(duration / dt)) steps;
  * batching: a model present in a subset of worlds only; every world of a
    batched scene equals the same world simulated alone, bit for bit.
"""

import numpy as np
import pytest

from scene_models import cube_urdf, sphere_urdf
from test_float_tree_oracle import chain_urdf

pytestmark = pytest.mark.gpu
G = 9.8


def _quat_to_R(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _rand_quat(rng, max_angle):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    a = rng.uniform(0, max_angle)
    return np.concatenate([[np.cos(a / 2)], axis * np.sin(a / 2)])


def _scene(models, W, pgs=50, mu=0.8, exact=False):
    """A scene of `models` in W worlds.  exact=False: the PGS sweeps alone, so
    the kernel is compared with the oracle running the same algorithm (the
    exact solve is covered by the KATs and the exact-mode tests)."""
    from mwstep.scene import Scene
    sc = Scene(n_worlds=W, pgs_iters=pgs)
    assert sc.lcp_solver() == (True, 48)
    sc.set_lcp_solver(exact)
    sc.set_ground_plane(True, mu)
    for text, pose, name in models:
        sc.insert_model(text, pose, name)
    return sc


def _oracle_from_gpu(oracle, cms, sc, w, pgs, mu, eps=0.0, seed=0):
    r = np.random.default_rng(seed)
    jig = (lambda a: np.asarray(a) * (1.0 + eps * r.uniform(-1, 1, np.shape(a)))) if eps else (lambda a: np.asarray(a))
    ow = oracle.SceneWorld(cms, pgs_iters=pgs, mu=mu)
    for m, cm in enumerate(cms):
        if cm.floating:
            pose = sc.base_pose(m, w, 1)[0]
            vel = sc.base_velocity(m, w, 1)[0]
            R = _quat_to_R(pose[3:])
            ow.set_pose(m, jig(pose[:3]), R)
            ow.set_twist(m, jig(R.T @ vel[3:]), jig(R.T @ vel[:3]))
        if cm.n:
            ow.set_joints(m, jig(sc.get("q", m, w, 1)[0]), jig(sc.get("qd", m, w, 1)[0]))
    return ow


class _Snapshot:
    """the start state of one world (base_pose / base_velocity / get of a Scene)"""

    def __init__(self, sc, w, K):
        self._p = [sc.base_pose(m, w, 1) for m in range(K)]
        self._v = [sc.base_velocity(m, w, 1) for m in range(K)]
        self._j = {(f, m): sc.get(f, m, w, 1) for f in ("q", "qd") for m in range(K)}

    def base_pose(self, m, w, nw):
        return self._p[m]

    def base_velocity(self, m, w, nw):
        return self._v[m]

    def get(self, f, m, w, nw):
        return self._j[(f, m)]


def _compare(oracle, cms, sc, ow, w):
    e = dict(pose=0.0, q=0.0, vel=0.0, qd=0.0)
    for m, cm in enumerate(cms):
        if cm.floating:
            pose = sc.base_pose(m, w, 1)[0]
            vel = sc.base_velocity(m, w, 1)[0]
            e["pose"] = max(e["pose"], float(np.abs(pose[:3] - ow.p(m)).max()),
                            float(np.abs(_quat_to_R(pose[3:]) - ow.R(m)).max()))
            R = ow.R(m)
            e["vel"] = max(e["vel"], float(np.abs(vel - np.concatenate([R @ ow.V(m)[3:], R @ ow.V(m)[:3]])).max()))
        if cm.n:
            e["q"] = max(e["q"], float(np.abs(sc.get("q", m, w, 1)[0] - ow.q(m)).max()))
            e["qd"] = max(e["qd"], float(np.abs(sc.get("qd", m, w, 1)[0] - ow.qd(m)).max()))
    return e


def test_one_step_parity_random_piles(require_gpu, oracle):
    W, pgs, mu = 256, 50, 0.8
    rng = np.random.default_rng(7)
    texts = [cube_urdf(), cube_urdf(double_collision=True, mass=2.0, edge=0.15), sphere_urdf(1.0, 0.08),
             chain_urdf(3)]
    names = ["cube1", "cube2", "ball", "chain"]
    base_z = [0.1, 0.28, 0.45, 0.6]
    cms = [oracle.load_urdf(t, pose_xyz=(0, 0, z)) for t, z in zip(texts, base_z)]
    sc = _scene([(t, (0, 0, z, 1, 0, 0, 0), nm) for t, z, nm in zip(texts, base_z, names)], W, pgs, mu)
    assert [m["floating"] for m in sc.models] == [True, True, True, True]
    # random piles: every body near the ones below it, tilted, moving
    for m, z in enumerate(base_z):
        poses = np.array([np.concatenate([rng.uniform(-0.06, 0.06, 2) + (0.0 if m else 0.0),
                                          [z + rng.uniform(-0.03, 0.02)], _rand_quat(rng, 0.4)]) for _ in range(W)])
        sc.reset_base_pose(m, poses)
        sc.reset_base_velocity(m, np.column_stack([rng.uniform(-0.5, 0.5, (W, 3)), rng.uniform(-1, 1, (W, 3))]))
    nj = cms[3].n
    sc.set("reset_q", rng.uniform(-1, 1, (W, nj)), m=3)
    sc.set("reset_qd", rng.uniform(-2, 2, (W, nj)), m=3)
    sc.run(paused=True)
    from mwstep import native as N
    sc.set_control_mode(N.MODE_FORCE, m=3)
    tau = rng.uniform(-5, 5, (W, nj)).astype(np.float32).astype(np.float64)
    sc.set("force_target", tau, m=3)
    orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
    sc_before = [_Snapshot(sc, w, len(cms)) for w in range(W)]
    sc.run()
    worst = dict(pose=0.0, q=0.0, vel=0.0, qd=0.0, point=0.0)
    ill, n_pairs, n_contact = [], 0, 0
    for w in range(W):
        ow = orcs[w]
        ow.mode[3, :nj] = oracle.FORCE
        ow.cmd[3, :nj] = tau[w]
        ow.step()
        e = _compare(oracle, cms, sc, ow, w)
        gc = sc.contacts(w)
        assert len(gc) == len(ow.contacts), (w, len(gc), len(ow.contacts))
        n_contact += len(gc) > 0
        for row, (oc, who) in zip(gc, ow.contacts):
            assert tuple(int(v) for v in row[10:14]) == who
            n_pairs += who[2] >= 0
            e["point"] = max(e.get("point", 0.0), float(np.abs(row[0:3] - oc[0:3]).max()))
        if e["vel"] > 2e-3 or e["qd"] > 2e-3:
            # ill-conditioned contact LCP: accept only if the oracle itself moves
            # as much under an fp32-size perturbation of its inputs
            sens = 0.0
            for k in range(4):
                ow2 = _oracle_from_gpu(oracle, cms, sc_before[w], 0, pgs, mu, 3e-7, k)
                ow2.mode[3, :nj] = oracle.FORCE
                ow2.cmd[3, :nj] = tau[w]
                ow2.step()
                for m in range(len(cms)):
                    sens = max(sens, float(np.abs(ow2.V(m) - ow.V(m)).max()) if cms[m].floating else 0.0,
                               float(np.abs(ow2.qd(m) - ow.qd(m)).max()) if cms[m].n else 0.0)
            ill.append((w, round(max(e["vel"], e["qd"]), 5), round(sens, 5)))
            assert sens >= 0.05 * max(e["vel"], e["qd"]), f"world {w}: {e}, oracle sensitivity {sens:.2e}"
            e.update(vel=0.0, qd=0.0)
        for k in worst:
            worst[k] = max(worst[k], e.get(k, 0.0))
    print(f"scene piles x{W}: one-step " + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) +
          f", {n_contact} worlds in contact, {n_pairs} body-body contact points, ill: {ill[:6]}")
    assert n_contact > W // 2 and n_pairs > W // 4
    assert len(ill) <= W // 20
    assert worst["pose"] <= 1e-5 and worst["q"] <= 1e-5 and worst["point"] <= 1e-5
    assert worst["vel"] <= 2e-3 and worst["qd"] <= 2e-3
    assert sc.overflow() == 0
    sc.close()


def test_cylinders_on_the_ground_one_step(require_gpu, oracle):
    """Cylinder collisions (ground plane only in this build: 4 rim points per
    cap from the deepest one, chain_dyn.hpp shape_slot_point / oracle.c
    or_slot_point) on the scene kernel: a free cylinder at random tilts and
    heights next to a cube, one step vs the fp64 scene oracle over 256 worlds
    (poses 1e-5, velocities 2e-3, contact points 1e-5; the can-cube pair
    contacts are checked in test_cylinder_pairs_one_step)."""
    from test_cylinder_oracle import cylinder_urdf
    W, pgs, mu = 256, 50, 0.8
    rng = np.random.default_rng(9)
    texts = [cylinder_urdf(), cube_urdf()]
    base = [(0.0, 0.0, 0.2), (0.05, 0.0, 0.3)]
    cms = [oracle.load_urdf(t, pose_xyz=b) for t, b in zip(texts, base)]
    sc = _scene([(t, (*b, 1, 0, 0, 0), nm) for t, b, nm in zip(texts, base, ["can", "cube"])], W, pgs, mu)
    poses = np.array([np.concatenate([[0, 0, rng.uniform(0.08, 0.22)], _rand_quat(rng, np.pi)]) for _ in range(W)])
    sc.reset_base_pose(0, poses)
    sc.reset_base_velocity(0, np.column_stack([rng.uniform(-0.5, 0.5, (W, 3)), rng.uniform(-2, 2, (W, 3))]))
    sc.run(paused=True)
    orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
    sc.run()
    worst = dict(pose=0.0, vel=0.0, point=0.0)
    n_contact = 0
    for w in range(W):
        ow = orcs[w]
        ow.step()
        e = _compare(oracle, cms, sc, ow, w)
        gc = sc.contacts(w)
        assert len(gc) == len(ow.contacts), (w, len(gc), len(ow.contacts))
        for row, (oc, who) in zip(gc, ow.contacts):
            assert tuple(int(v) for v in row[10:14]) == who
            if who[2] >= 0:   # cylinder-box pair (test_cylinder_pairs_one_step)
                continue
            n_contact += who[0] == 0
            worst["point"] = max(worst["point"], float(np.abs(row[0:3] - oc[0:3]).max()))
        worst["pose"] = max(worst["pose"], e["pose"])
        worst["vel"] = max(worst["vel"], e["vel"])
    print(f"cylinders x{W}: one-step " + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) +
          f", {n_contact} cylinder-ground contact points")
    assert n_contact > W
    assert worst["pose"] <= 1e-5 and worst["point"] <= 1e-5 and worst["vel"] <= 2e-3
    sc.close()


@pytest.mark.parametrize("double", [False, True])
def test_three_cubes_kat(require_gpu, double):
    """tests/test_scenario/test_contacts.py:125-236 through the scene API."""
    from mwstep.scene import Scene
    sc = Scene(n_worlds=1, pgs_iters=50)
    sc.set_ground_plane(True, 1.0)
    c = cube_urdf(double)
    sc.insert_model(c, (0, -0.15, 0.101, 1, 0, 0, 0), "cube1")
    sc.insert_model(c, (0, 0.15, 0.101, 1, 0, 0, 0), "cube2")
    sc.run(paused=True)
    assert len(sc.contacts(0)) == 0
    for _ in range(50):
        sc.run()
    rows = sc.contacts(0)
    assert {int(r[10]) for r in rows} == {0, 1} and all(r[12] == -1 for r in rows)
    z12 = sc.base_pose(0)[0, 2], sc.base_pose(1)[0, 2]
    sc.insert_model(c, (0, 0, 0.301, 1, 0, 0, 0), "cube3")
    sc.run(paused=True)
    assert sc.base_pose(0)[0, 2] == z12[0] and sc.base_pose(1)[0, 2] == z12[1]   # state kept
    for _ in range(50):
        sc.run()
    rows = sc.contacts(0)

    def wrench(m):
        f = np.zeros(3)
        for r in rows:
            if int(r[10]) == m:
                f += r[6:9]
            elif int(r[12]) == m:
                f -= r[6:9]
        return f

    partners = sorted({int(r[10]) for r in rows if int(r[12]) == 2})
    assert partners == [0, 1]
    assert wrench(2)[2] == pytest.approx(50, abs=1.1)
    assert wrench(0)[2] == pytest.approx(50, abs=1.1)
    assert wrench(1)[2] == pytest.approx(50, abs=1.1)
    for r in rows:
        if int(r[12]) == 2:
            assert np.allclose(r[3:6], [0, 0, -1], atol=1e-3) and r[8] < 0
    assert sc.overflow() == 0
    sc.close()


def test_world_wrench_duration(require_gpu):
    """A floating cube far from the ground, F = 30 N along x for 10.5 ms at
    dt = 1 ms: applied on 11 steps (expiry = now + duration, removed after
    the step whose time reaches it; Physics.cpp:1446-1525): v_x = 30/5 *
    0.011; a second wrench of 0 s still acts on one step."""
    from mwstep.scene import Scene
    sc = Scene(n_worlds=2, pgs_iters=50)
    sc.insert_model(cube_urdf(), (0, 0, 5.0, 1, 0, 0, 0), "cube")
    sc.run(paused=True)
    sc.apply_world_wrench(0, -1, [30.0, 0, 0, 0, 0, 0], 0.0105, w0=0, nw=1)
    sc.apply_world_wrench(0, -1, [0, 20.0, 0, 0, 0, 0], 0.0, w0=1, nw=1)
    for _ in range(40):
        sc.run()
    v = sc.base_velocity(0)
    assert v[0, 0] == pytest.approx(30.0 / 5.0 * 0.011, rel=1e-5)
    assert v[1, 1] == pytest.approx(20.0 / 5.0 * 0.001, rel=1e-5)
    assert v[0, 2] == pytest.approx(-G * 0.04, rel=1e-5) and v[1, 0] == 0.0
    sc.close()


def test_welded_panda_and_cube(require_gpu, oracle):
    """A fixed-base Panda (URDF root welded to "world") and a cube dropped
    onto the ground next to it: one world, 200 steps free-running against
    the oracle scene (no contact between them)."""
    from mwstep import get_model_file
    from mwstep import native as N
    panda = get_model_file("panda")
    cms = [oracle.load_urdf(panda), oracle.load_urdf(cube_urdf(), pose_xyz=(0.8, 0, 0.3))]
    sc = _scene([(panda, (0, 0, 0, 1, 0, 0, 0), "panda"), (cube_urdf(), (0.8, 0, 0.3, 1, 0, 0, 0), "cube")], 1)
    assert sc.models[0]["floating"] is False and sc.models[0]["dofs"] == 9
    q0 = np.array([0.1, -0.5, 0.2, -2.0, 0.1, 1.5, 0.5, 0.02, 0.02])
    sc.set("reset_q", q0[None], m=0)
    sc.run(paused=True)
    sc.set_control_mode(N.MODE_FORCE, m=0)
    ow = oracle.SceneWorld(cms, pgs_iters=50, mu=0.8)
    ow.set_joints(0, q0, np.zeros(9))
    rng = np.random.default_rng(3)
    worst = 0.0
    for k in range(200):
        tau = rng.uniform(-5, 5, 9).astype(np.float32).astype(np.float64)
        sc.set("force_target", tau[None], m=0)
        sc.run()
        ow.mode[0, :9] = oracle.FORCE
        ow.cmd[0, :9] = tau
        ow.step()
        worst = max(worst, float(np.abs(sc.get("q", 0)[0] - ow.q(0)).max()))
    zc = sc.base_pose(1)[0, 2]
    print(f"welded panda + cube, 200 steps: max|dq| {worst:.2e}, cube z {zc:.4f} (oracle {ow.p(1)[2]:.4f})")
    assert worst <= 1e-4 and abs(zc - ow.p(1)[2]) <= 1e-5
    sc.close()


def test_partial_presence_and_batch_identity(require_gpu):
    """Worlds 0..3 hold cube + ball, the ball is inserted only into worlds 2
    and 3; a world of the batched scene equals the same world run alone."""
    from mwstep.scene import Scene
    W = 4
    sc = Scene(n_worlds=W, pgs_iters=50)
    sc.set_ground_plane(True, 1.0)
    sc.insert_model(cube_urdf(), (0, 0, 0.3, 1, 0, 0, 0), "cube")
    sc.insert_model(sphere_urdf(), (0.02, 0, 0.6, 1, 0, 0, 0), "ball", worlds=(2, 2))
    assert [sc.present(1, w) for w in range(W)] == [False, False, True, True]
    solo = []
    for w in range(W):
        s1 = Scene(n_worlds=1, pgs_iters=50)
        s1.set_ground_plane(True, 1.0)
        s1.insert_model(cube_urdf(), (0, 0, 0.3, 1, 0, 0, 0), "cube")
        if w >= 2:
            s1.insert_model(sphere_urdf(), (0.02, 0, 0.6, 1, 0, 0, 0), "ball")
        solo.append(s1)
    vel = np.array([[0.1 * w, 0, 0, 0, 0, 0.5] for w in range(W)])
    sc.reset_base_velocity(0, vel)
    for w in range(W):
        solo[w].reset_base_velocity(0, vel[w:w + 1])
    for _ in range(300):
        sc.run()
        for s1 in solo:
            s1.run()
    for w in range(W):
        assert np.array_equal(sc.base_pose(0, w, 1), solo[w].base_pose(0)), w
        if w >= 2:
            assert np.array_equal(sc.base_pose(1, w, 1), solo[w].base_pose(1)), w
    # the ball rests on the cube in worlds 2, 3
    assert sc.base_pose(1, 2, 1)[0, 2] > 0.25
    for s1 in solo:
        s1.close()
    sc.close()


def _fixed_tree_urdf(n=16, seed=9):
    """A random branched tree of n revolute / prismatic joints welded to the
    world (the fixed-base generalisation of test_gpu_float_tree.tree_urdf):
    models of this shape are refused by the single-model chain kernels
    (serial chains of <= 9 dofs and the Panda only) and run on the scene kernel."""
    rng = np.random.default_rng(seed)
    parents = [-1] + [int(rng.integers(-1, i)) for i in range(1, n)]
    parts = ['<robot name="ftree"><link name="world"/><joint name="weld" type="fixed"><parent link="world"/>'
             '<child link="base"/><origin xyz="0 0 1.5"/></joint><link name="base"><inertial><mass value="3"/>'
             '<inertia ixx="0.1" iyy="0.1" izz="0.1" ixy="0" ixz="0" iyz="0"/></inertial></link>']
    for i, pa in enumerate(parents):
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        prismatic = i % 6 == 5
        lim = ('<limit lower="-0.2" upper="0.2" effort="80" velocity="10"/>' if prismatic else
               '<limit lower="-1.2" upper="1.2" effort="50" velocity="30"/>')
        xyz = " ".join(f"{v:.3f}" for v in rng.uniform(-0.15, 0.15, 3))
        rpy = " ".join(f"{v:.3f}" for v in rng.uniform(-0.5, 0.5, 3))
        m = rng.uniform(0.2, 1.0)
        parent = "base" if pa < 0 else f"l{pa}"
        parts.append(f'<joint name="j{i}" type="{"prismatic" if prismatic else "revolute"}">'
                     f'<parent link="{parent}"/><child link="l{i}"/><origin xyz="{xyz}" rpy="{rpy}"/>'
                     f'<axis xyz="{axis[0]:.4f} {axis[1]:.4f} {axis[2]:.4f}"/>{lim}'
                     f'<dynamics damping="{0.3 * (i % 3):.2f}" friction="{0.2 if i % 4 == 1 else 0.0}"/></joint>'
                     f'<link name="l{i}"><inertial><origin xyz="0 0.01 -0.05"/><mass value="{m:.3f}"/>'
                     f'<inertia ixx="{0.004 * m:.5f}" iyy="{0.005 * m:.5f}" izz="{0.002 * m:.5f}" ixy="0.0001" '
                     f'ixz="0" iyz="0"/></inertial></link>')
    return "".join(parts) + "</robot>"


def test_generic_fixed_base_tree_one_step(require_gpu, oracle):
    """A welded random 16-joint branched tree (damping, Coulomb friction,
    joints beyond their limits, random torques): one step against the fp64
    tree oracle or_step (ABA + joint LCP) for 256 worlds of random states, on
    the scene kernel and through mw_sim (the world-per-wavefront kernel with a
    welded base, FloatF::fixed): q within 1e-5, qd within 1e-4."""
    from mwstep import native as N
    from mwstep.sim import Simulator
    text = _fixed_tree_urdf()
    W = 256
    rng = np.random.default_rng(4)
    cm = oracle.load_urdf(text)
    n = cm.n
    assert n == 16 and not cm.floating
    lo, hi = np.array(cm.model.lower[:n]), np.array(cm.model.upper[:n])
    q = rng.uniform(lo, hi, (W, n))
    beyond = rng.uniform(size=(W, n)) < 0.1
    q[beyond] = np.where(rng.uniform(size=(W, n)) < 0.5, lo - 1e-3, hi + 1e-3)[beyond]
    qd = rng.uniform(-1, 1, (W, n))
    tau = rng.uniform(-10, 10, (W, n))
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    q, qd, tau = f32(q), f32(qd), f32(tau)
    from mwstep.scene import Scene
    sc = Scene(n_worlds=W, pgs_iters=50)
    sc.set_lcp_solver(False)  # vs the oracle's PGS-50 step
    sc.insert_model(text, (0, 0, 0, 1, 0, 0, 0), "ftree")
    assert sc.models[0]["floating"] is False and sc.models[0]["dofs"] == n
    sc.set("reset_q", q, m=0)
    sc.set("reset_qd", qd, m=0)
    sc.run(paused=True)
    sc.set_control_mode(N.MODE_FORCE, m=0)
    sc.set("force_target", tau, m=0)
    sc.run()
    gq, gqd = sc.get("q", 0), sc.get("qd", 0)
    wq = wqd = 0.0
    for w in range(W):
        oq, oqd, *_ = oracle.step(cm, 1e-3, q[w], qd[w], np.full(n, oracle.FORCE, np.int32), tau[w], 50)
        wq = max(wq, float(np.abs(gq[w] - oq).max()))
        wqd = max(wqd, float(np.abs(gqd[w] - oqd).max()))
    print(f"fixed 16-joint tree on the scene kernel, one step x{W}: max|dq| {wq:.2e}, max|dqd| {wqd:.2e}")
    assert wq <= 1e-5 and wqd <= 1e-4
    sc.close()
    sim = Simulator(text, n_worlds=W, pgs_iters=50)
    assert not sim.floating and sim.float_kernel() == 2
    sim.set("reset_q", q)
    sim.set("reset_qd", qd)
    sim.run(paused=True)
    sim.set_control_mode(N.MODE_FORCE)
    sim.set("force_target", tau)
    sim.run()
    sq, sqd = sim.get("q"), sim.get("qd")
    wq = wqd = 0.0
    for w in range(W):
        # mw_sim's wave kernel solves the joint-row LCP exactly (wave_lcp.hpp)
        oq, oqd, *_ = oracle.step(cm, 1e-3, q[w], qd[w], np.full(n, oracle.FORCE, np.int32), tau[w],
                                  oracle.PGS_CONVERGED)
        wq = max(wq, float(np.abs(sq[w] - oq).max()))
        wqd = max(wqd, float(np.abs(sqd[w] - oqd).max()))
    print(f"fixed 16-joint tree through mw_sim (wave kernel, welded base): max|dq| {wq:.2e}, max|dqd| {wqd:.2e}")
    assert wq <= 1e-5 and wqd <= 1e-4
    # the welded base stays where the model was inserted (Model::basePosition)
    assert np.allclose(sim.base_pose()[:, :3], cm.base_p) and np.allclose(sim.base_velocity(), 0.0)
    assert sim.constraint_overflow() == 0
    sim.close()


def test_cylinder_sphere_contacts(require_gpu, oracle):
    """Cylinder-sphere contacts on the scene kernel (sc_cylinder_sphere, the
    float32 restatement of oracle.c cylinder_sphere): one step over 256 worlds
    of a tilted floating cylinder with a ball pressed against its cap, side or
    rim (poses 1e-5, velocities 2e-3, contact points 1e-5 vs the fp64 scene
    oracle), and a ball dropped on a welded pillar resting on its top cap
    (closed loop within 1e-4 m of the oracle)."""
    from test_cylinder_oracle import PILLAR, ball_urdf, cylinder_urdf
    W, pgs, mu = 256, 50, 0.8
    rng = np.random.default_rng(21)
    texts = [cylinder_urdf(), ball_urdf(1.0, 0.06)]
    base = [(0.0, 0.0, 0.5), (0.0, 0.0, 0.8)]
    cms = [oracle.load_urdf(t, pose_xyz=b) for t, b in zip(texts, base)]
    sc = _scene([(t, (*b, 1, 0, 0, 0), nm) for t, b, nm in zip(texts, base, ["can", "ball"])], W, pgs, mu)
    qc = np.array([_rand_quat(rng, 1.2) for _ in range(W)])
    pc = np.column_stack([np.zeros((W, 2)), np.full(W, 0.5)])
    # ball centre: a point on the cylinder surface (cap, side or rim) pushed in by up to 1 cm
    pts = []
    for w in range(W):
        R = _quat_to_R(qc[w])
        kind = w % 3
        ang = rng.uniform(0, 2 * np.pi)
        if kind == 0:
            local = np.array([0.05 * np.cos(ang), 0.05 * np.sin(ang), 0.2 + 0.06 - rng.uniform(0, 0.01)])
        elif kind == 1:
            rr = 0.1 + 0.06 - rng.uniform(0, 0.01)
            local = np.array([rr * np.cos(ang), rr * np.sin(ang), rng.uniform(-0.15, 0.15)])
        else:
            dirn = np.array([0.6 * np.cos(ang), 0.6 * np.sin(ang), 0.8])
            local = np.array([0.1 * np.cos(ang), 0.1 * np.sin(ang), 0.2]) + (0.06 - rng.uniform(0, 0.01)) * dirn
        pts.append(pc[w] + R @ local)
    sc.reset_base_pose(0, np.column_stack([pc, qc]))
    sc.reset_base_pose(1, np.column_stack([np.array(pts), np.ones(W), np.zeros((W, 3))]))
    for m in range(2):
        sc.reset_base_velocity(m, np.column_stack([rng.uniform(-0.3, 0.3, (W, 3)), rng.uniform(-1, 1, (W, 3))]))
    sc.run(paused=True)
    orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
    sc.run()
    worst = dict(pose=0.0, vel=0.0, point=0.0)
    n_pairs = 0
    for w in range(W):
        ow = orcs[w]
        ow.step()
        e = _compare(oracle, cms, sc, ow, w)
        gc = sc.contacts(w)
        assert len(gc) == len(ow.contacts), (w, len(gc), len(ow.contacts))
        for row, (oc, who) in zip(gc, ow.contacts):
            assert tuple(int(v) for v in row[10:14]) == who
            n_pairs += who[2] >= 0
            worst["point"] = max(worst["point"], float(np.abs(row[0:3] - oc[0:3]).max()))
        worst["pose"] = max(worst["pose"], e["pose"])
        worst["vel"] = max(worst["vel"], e["vel"])
    print(f"cylinder-sphere x{W}: one-step " + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) +
          f", {n_pairs} cylinder-sphere contact points")
    assert n_pairs > W // 2
    assert worst["pose"] <= 1e-5 and worst["point"] <= 1e-5 and worst["vel"] <= 2e-3
    sc.close()
    # the pillar KAT through the scene kernel
    texts = [PILLAR, ball_urdf()]
    cms = [oracle.load_urdf(PILLAR), oracle.load_urdf(texts[1], pose_xyz=(0.02, 0, 0.75))]
    sc = _scene([(PILLAR, (0, 0, 0, 1, 0, 0, 0), "pillar"), (texts[1], (0.02, 0, 0.75, 1, 0, 0, 0), "ball")],
                2, pgs, 1.0)
    ow = oracle.SceneWorld(cms, pgs_iters=pgs, mu=1.0)
    worst = 0.0
    for k in range(600):
        sc.run()
        ow.step()
        if k % 50 == 49:
            worst = max(worst, float(np.abs(sc.base_pose(1, 0, 1)[0, :3] - ow.p(1)).max()))
    z = sc.base_pose(1, 0, 1)[0, 2]
    print(f"ball on a pillar: z {z:.5f} (0.6 + 0.05), max |dp| vs oracle {worst:.2e}")
    assert z == pytest.approx(0.65, abs=2e-3) and worst <= 1e-4
    sc.close()


def test_cylinder_pairs_one_step(require_gpu, oracle):
    """Cylinder-box and cylinder-cylinder contacts between models (oracle.c
    cylinder_pair, scene_kernel.hip sc_cylinder_pair: least-overlap axis,
    sampled features): a tilted cylinder and a smaller one dropped on a welded
    table and on each other, one step vs the fp64 scene oracle over 256
    worlds (poses 1e-5, velocities 2e-3, contact points 1e-5; at most 2 % of
    the pair points may differ where fp32 picks another axis of near-equal
    overlap, with the dynamics still within the bounds)."""
    from test_cylinder_oracle import TABLE, cylinder_urdf
    W, pgs, mu = 256, 50, 0.8
    rng = np.random.default_rng(21)
    texts = [TABLE, cylinder_urdf(2.0, 0.1, 0.4, name="can"), cylinder_urdf(1.0, 0.06, 0.2, name="cup")]
    base = [(0, 0, 0), (0.0, 0.0, 0.5), (0.05, 0.0, 0.8)]
    cms = [oracle.load_urdf(t, pose_xyz=b) for t, b in zip(texts, base)]
    sc = _scene([(t, (*b, 1, 0, 0, 0), nm) for t, b, nm in zip(texts, base, ["table", "can", "cup"])], W, pgs, mu)
    can = np.array([np.concatenate([rng.uniform(-0.1, 0.1, 2), [rng.uniform(0.36, 0.5)], _rand_quat(rng, np.pi)])
                    for _ in range(W)])
    cup = np.array([np.concatenate([can[w, :2] + rng.uniform(-0.08, 0.08, 2), [can[w, 2] + rng.uniform(0.1, 0.3)],
                                    _rand_quat(rng, np.pi)]) for w in range(W)])
    sc.reset_base_pose(1, can)
    sc.reset_base_pose(2, cup)
    for m in (1, 2):
        sc.reset_base_velocity(m, np.column_stack([rng.uniform(-0.5, 0.5, (W, 3)), rng.uniform(-2, 2, (W, 3))]))
    sc.run(paused=True)
    orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
    sc.run()
    worst = dict(pose=0.0, vel=0.0, point=0.0)
    n_cb, n_cc, moved, ill = 0, 0, [], []
    for w in range(W):
        ow = orcs[w]
        ow.step()
        e = _compare(oracle, cms, sc, ow, w)
        gc = sc.contacts(w)
        assert len(gc) == len(ow.contacts), (w, len(gc), len(ow.contacts))
        for row, (oc, who) in zip(gc, ow.contacts):
            assert tuple(int(v) for v in row[10:14]) == who
            n_cb += who[0] == 0 and who[2] >= 1
            n_cc += who[0] == 1 and who[2] == 2
            err = float(np.abs(row[0:3] - oc[0:3]).max())
            if err > 1e-5 and who[2] >= 0:
                moved.append((w, who, round(err, 5)))
                continue
            worst["point"] = max(worst["point"], err)
        if e["vel"] > 2e-3:
            ill.append((w, round(e["vel"], 5)))
            continue
        worst["pose"] = max(worst["pose"], e["pose"])
        worst["vel"] = max(worst["vel"], e["vel"])
    print(f"cylinder pairs x{W}: one-step " + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) +
          f", {n_cb} cylinder-table and {n_cc} cylinder-cylinder points, moved {moved[:6]}, ill {ill[:6]}")
    assert n_cb > W // 4 and n_cc > W // 16
    assert len(moved) <= (n_cb + n_cc) // 50 and len(ill) <= W // 50
    assert worst["pose"] <= 1e-5 and worst["point"] <= 1e-5 and worst["vel"] <= 2e-3
    assert sc.overflow() == 0
    sc.close()


def test_cylinder_stack_on_a_table(require_gpu):
    """a can standing on the welded table, a cup standing on the can: both
    come to rest at their stacked heights and the table carries both weights"""
    from test_cylinder_oracle import TABLE, cylinder_urdf
    W = 8
    sc = _scene([(TABLE, (0, 0, 0, 1, 0, 0, 0), "table"),
                 (cylinder_urdf(2.0, 0.1, 0.4, name="can"), (0.02, 0, 0.52, 1, 0, 0, 0), "can"),
                 (cylinder_urdf(1.0, 0.06, 0.2, name="cup"), (0.03, 0, 0.82, 1, 0, 0, 0), "cup")], W)
    for _ in range(1500):
        sc.run()
    can, cup = sc.base_pose(1, 0, W), sc.base_pose(2, 0, W)
    np.testing.assert_allclose(can[:, 2], 0.3 + 0.2, atol=2e-3)
    np.testing.assert_allclose(cup[:, 2], 0.7 + 0.1, atol=3e-3)
    for w in range(W):
        # force on the table (always model A of its pairs: lower index)
        on_table = sum(r[8] for r in sc.contacts(w) if int(r[10]) == 0 and int(r[12]) >= 0)
        assert abs(on_table) == pytest.approx(3.0 * G, abs=0.1)
    sc.close()


def test_direct_runs_match_device_runs(require_gpu):
    """Small scenes run direct (mw_scene_run: the kernel reads the command
    block out of the pinned mirror and writes q / qd / qdd into it, no
    copies).  A mix of direct runs and device runs (mw_scene_run_device, which
    must first upload the command block the direct runs left stale: control
    modes, targets) steps exactly like direct runs alone."""
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.scene import Scene
    scenes = []
    for _ in range(2):
        sc = Scene(n_worlds=2, step_size=1e-3, steps_per_run=1)
        sc.insert_model(get_model_file("cartpole"))
        sc.set_control_mode(N.MODE_POSITION, m=0)
        for d in range(sc._nd):
            sc.set_pid(d, [100.0, 0.0, 5.0, -50.0, 50.0, 0.0, 0.0, -1.0])
        sc.set("position_target", np.full((2, sc._nd), 0.2), m=0)
        sc.run(paused=True)
        scenes.append(sc)
    a, b = scenes
    for k in range(30):
        a.run()
        if k % 3 == 2:
            b.run_device(1)
            b.get("q")  # pulls the joint planes
        else:
            b.run()
        if k == 10:
            for sc in scenes:
                sc.set("position_target", np.full((2, sc._nd), -0.1), m=0)
        qa, qb = a.get("q"), b.get("q")
        assert np.array_equal(qa, qb), (k, qa, qb)
        assert np.array_equal(a.get("qd"), b.get("qd"))
    assert np.abs(a.get("q")).max() > 1e-3  # the targets moved the joints
    for sc in scenes:
        sc.close()
