"""CPU tests of the scene oracle (oracle.c or_scene_step: several models in
one world, shape-pair contacts, world wrenches), pinned by:

  * the single-model oracles it generalises: one floating humanoid equals
    or_float_step, one fixed-base Panda equals or_step (the chain ABA), step
    for step;
  * the reference's contact KATs (tests/test_scenario/test_contacts.py):
    a cube on the ground carries its weight (:58-122); three cubes, the third
    resting across the gap of the other two, both collision variants
    (:125-236: contact wrench of cube3 = its weight within 1.1 N, the lower
    cubes 1.5x from below and 0.5x from above, normals / force signs);
  * the narrow phase against closed forms (box-box face and edge contacts,
    box-sphere, sphere-sphere);
  * a world wrench on a floating cube in free fall: v = (F/m + g) t.
"""

import numpy as np
import pytest

from scene_models import cube_urdf, sphere_urdf

G = 9.8


def _cubes(oracle, poses, double=False, pgs=50):
    cms = [oracle.load_urdf(cube_urdf(double), pose_xyz=p) for p in poses]
    return oracle.SceneWorld(cms, pgs_iters=pgs)


def test_single_floating_model_equals_float_step(oracle):
    from mwstep import get_model_file
    cm = oracle.load_urdf(get_model_file("icub"), pose_xyz=(0, 0, 0.66), pose_wxyz=(0, 0, 0, 1))
    sw = oracle.SceneWorld([cm], pgs_iters=50)
    fw = oracle.FloatWorld(cm, pgs_iters=50)
    for w in (sw,):
        w.set_twist(0, [0.2, 0.1, 0.0], [0.3, 0.0, -0.2])
    fw.set_twist([0.2, 0.1, 0.0], [0.3, 0.0, -0.2])
    n = cm.n
    rng = np.random.default_rng(0)
    for _ in range(200):
        tau = rng.uniform(-5, 5, n)
        sw.mode[0, :n] = oracle.FORCE
        sw.cmd[0, :n] = tau
        nc = sw.step()
        fw.step(np.full(n, oracle.FORCE, np.int32), tau)
        assert nc == len(fw.contacts)
    assert np.abs(sw.q(0) - fw.q).max() < 1e-9 and np.abs(sw.V(0) - fw.V).max() < 1e-8
    assert np.abs(sw.p(0) - fw.p).max() < 1e-10
    assert nc > 0


def test_single_fixed_model_equals_chain_step(oracle):
    from mwstep import get_model_file
    cm = oracle.load_urdf(get_model_file("panda"))
    sw = oracle.SceneWorld([cm], ground=False, pgs_iters=50)
    n = cm.n
    rng = np.random.default_rng(1)
    q = rng.uniform(-1, 1, n)
    qd = rng.uniform(-1, 1, n)
    q[3] = cm.model.upper[3] + 0.01       # a limit row
    sw.set_joints(0, q, qd)
    qc, qdc = q.copy(), qd.copy()
    for _ in range(100):
        tau = rng.uniform(-10, 10, n)
        sw.mode[0, :n] = oracle.FORCE
        sw.cmd[0, :n] = tau
        sw.step()
        qc, qdc = oracle.step(cm, 1e-3, qc, qdc, np.full(n, oracle.FORCE, np.int32), tau, pgs_iters=50)[:2]
    assert np.abs(sw.q(0) - qc).max() < 1e-9 and np.abs(sw.qd(0) - qdc).max() < 1e-7


def test_cube_on_ground_kat(oracle):
    sw = _cubes(oracle, [(0, 0, 0.15)])
    for _ in range(150):
        nc = sw.step()
    assert nc == 4
    fz = sum(c[6:9][2] for c, who in sw.contacts)
    assert fz == pytest.approx(5 * G, abs=0.1)
    for c, who in sw.contacts:
        assert np.allclose(c[3:6], [0, 0, 1]) and who == (0, -1, -1, -1)


@pytest.mark.parametrize("double", [False, True])
def test_three_cubes_kat(oracle, double):
    """test_contacts.py:125-236 on the oracle: cube3 falls onto the gap
    between cube1 and cube2 (all in one world)."""
    cms = [oracle.load_urdf(cube_urdf(double), pose_xyz=p) for p in [(0, -0.15, 0.101), (0, 0.15, 0.101)]]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(50):
        sw.step()
    # insert cube3 with the lower cubes' state carried over
    cm3 = oracle.load_urdf(cube_urdf(double), pose_xyz=(0, 0, 0.301))
    sw2 = oracle.SceneWorld(cms + [cm3], pgs_iters=50)
    for m in range(2):
        sw2.set_pose(m, sw.p(m), sw.R(m))
        sw2.set_twist(m, sw.V(m)[:3], sw.V(m)[3:])
    for _ in range(50):
        sw2.step()

    def wrench(m):
        f = np.zeros(3)
        for c, (ma, ba, mb, bb) in sw2.contacts:
            if ma == m:
                f += c[6:9]
            elif mb == m:
                f -= c[6:9]
        return f

    def partners(m):
        return sorted({(mb if ma == m else ma) for c, (ma, ba, mb, bb) in sw2.contacts if m in (ma, mb)})

    assert partners(2) == [0, 1]                 # cube3 touches cube1 and cube2 only
    assert wrench(2)[2] == pytest.approx(50, abs=1.1)
    assert wrench(0)[2] == pytest.approx(50, abs=1.1)
    assert wrench(1)[2] == pytest.approx(50, abs=1.1)
    for c, (ma, ba, mb, bb) in sw2.contacts:
        if mb == -1:
            assert np.allclose(c[3:6], [0, 0, 1]) and c[8] > 0
        else:   # cube3 (model 2) is always B in its pairs: the force on the lower cube points down
            assert mb == 2 and np.allclose(c[3:6], [0, 0, -1], atol=1e-3) and c[8] < 0


def test_narrow_phase_closed_forms(oracle):
    I = np.eye(3)
    h = [0.1, 0.1, 0.1]
    # face-face: B 0.19 below A, offset in y: 4 points, depth 0.01, normal +z (B into A)
    n, pts, dep = oracle.collide(0, h, [0, 0, 0.19], I, 0, h, [0, 0.05, 0], I)
    assert np.allclose(n, [0, 0, 1]) and len(pts) == 4 and np.allclose(dep, 0.01)
    assert np.allclose(sorted(pts[:, 1]), [-0.05, -0.05, 0.1, 0.1])
    # edge-edge: A rotated 45 deg about x, B rotated 45 deg about y, A above B
    c, s = np.cos(np.pi / 4), np.sin(np.pi / 4)
    Rx = np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    Ry = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    d = 0.1 * np.sqrt(2)
    n, pts, dep = oracle.collide(0, h, [0, 0, 2 * d - 0.004], Rx, 0, h, [0, 0, 0], Ry)
    assert len(pts) == 1 and np.allclose(n, [0, 0, 1], atol=1e-9) and dep[0] == pytest.approx(0.004)
    assert np.allclose(pts[0], [0, 0, d - 0.002])
    # box-sphere and sphere-sphere
    n, pts, dep = oracle.collide(1, [0.05], [0, 0, 0.14], I, 0, h, [0, 0, 0], I)
    assert np.allclose(n, [0, 0, 1]) and dep[0] == pytest.approx(0.01) and np.allclose(pts[0], [0, 0, 0.1])
    n, pts, dep = oracle.collide(1, [0.05], [0.09, 0, 0], I, 1, [0.05], [0, 0, 0], I)
    assert np.allclose(n, [1, 0, 0]) and dep[0] == pytest.approx(0.01)
    assert len(oracle.collide(0, h, [0, 0, 0.21], I, 0, h, [0, 0, 0], I)[1]) == 0


def test_world_wrench_on_free_cube(oracle):
    """A floating cube away from the ground, 30 N along x at its origin (=
    its COM) for 200 steps: v = (F / m) t, z falls with g; a torque about z
    alone spins it at (tau / I) t."""
    cm = oracle.load_urdf(cube_urdf(), pose_xyz=(0, 0, 5.0))
    sw = oracle.SceneWorld([cm], pgs_iters=50)
    sw.wrench[0, 0] = [30.0, 0.0, 0.0, 0.0, 0.0, 0.0]
    for _ in range(200):
        sw.step()
    v = sw.R(0) @ sw.V(0)[3:]
    assert v[0] == pytest.approx(30.0 / 5.0 * 0.2, rel=1e-9)
    assert v[2] == pytest.approx(-G * 0.2, rel=1e-9)
    sw = oracle.SceneWorld([cm], pgs_iters=50)
    sw.wrench[0, 0] = [0.0, 0.0, 0.0, 0.0, 0.0, 0.2]
    for _ in range(200):
        sw.step()
    w = sw.R(0) @ sw.V(0)[:3]
    I = 1 / 12 * 5.0 * (0.04 + 0.04)
    assert w[2] == pytest.approx(0.2 / I * 0.2, rel=1e-9)


def test_sphere_rolls_on_fixed_box(oracle):
    """A fixed-base model (a static box on a 'world' joint) is a collider for
    a floating ball: the ball comes to rest on the box top."""
    box = ('<robot name="table"><link name="world"/><joint name="fix" type="fixed"><parent link="world"/>'
           '<child link="top"/><origin xyz="0 0 0.25"/></joint><link name="top"><inertial><mass value="10"/>'
           '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision><geometry>'
           '<box size="1 1 0.5"/></geometry></collision></link></robot>')
    cms = [oracle.load_urdf(box), oracle.load_urdf(sphere_urdf(), pose_xyz=(0, 0, 0.62))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    assert not cms[0].floating
    for _ in range(400):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.6, abs=2e-3)
    fz = sum(c[8] for c, who in sw.contacts if who[2] == 1 or who[0] == 1)
    assert abs(fz) == pytest.approx(1.0 * G, abs=0.05)
