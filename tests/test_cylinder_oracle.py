"""Cylinder collisions (Physics.cpp:687-1219 builds box, sphere and
cylinder collision shapes) in the fp64 oracle, pinned before the kernels are
compared with it (CPU):

  * the slot geometry (or_slot_point): a standing cylinder touches on a square
    of its bottom rim, a lying one at the two exact ends of its contact line,
    a tilted one first at the deepest rim point;
  * a standing cylinder carries its weight (the contact KAT shape of
    tests/test_scenario/test_contacts.py:58-122) at rest at half its length;
  * a lying cylinder released with spin about its axis rolls without slipping:
    v = omega r, and the final speed is omega0 r / 3 (a solid cylinder,
    I = m r^2 / 2, angular momentum about the contact line conserved);
  * the URDF and SDF cylinder geometry compile alike in the product's C++
    compiler and the oracle's reader;
  * cylinder-sphere closed forms, a ball on a pillar; cylinder-box and
    cylinder-cylinder pairs (sampled features): closed forms, a cylinder
    standing and lying on a welded table, a two-cylinder stack.
"""

import ctypes
import math

import numpy as np
import pytest

G = 9.8


def cylinder_urdf(mass=2.0, r=0.1, length=0.4, name="can", rpy="0 0 0"):
    ixx = mass * (3 * r * r + length * length) / 12.0
    izz = 0.5 * mass * r * r
    return (f'<robot name="{name}"><link name="{name}"><inertial><mass value="{mass}"/>'
            f'<inertia ixx="{ixx}" iyy="{ixx}" izz="{izz}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><origin rpy="{rpy}" xyz="0 0 0"/><geometry><cylinder radius="{r}" length="{length}"/>'
            f'</geometry></collision></link></robot>')


def _Rx(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _slot(oracle, RS, c, h=(0.1, 0.2, 0.0)):
    lib = oracle.lib()
    l = np.zeros(3)
    hh = np.array(h, dtype=np.float64)
    RSa = np.ascontiguousarray(RS, dtype=np.float64).ravel()
    lib.or_slot_point(2, hh.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                      RSa.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), c,
                      l.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return l


def test_slot_geometry(oracle):
    lib = oracle.lib()
    lib.or_slot_point.restype = None
    # standing: the 4 points of each cap at 90 degrees, radius r
    pts = np.array([_slot(oracle, np.eye(3), c) for c in range(8)])
    np.testing.assert_allclose(np.linalg.norm(pts[:, :2], axis=1), 0.1)
    np.testing.assert_allclose(pts[:4, 2], -0.2)
    np.testing.assert_allclose(pts[4:, 2], 0.2)
    np.testing.assert_allclose(pts[0], [0.1, 0, -0.2], atol=1e-15)
    # lying (axis along world y after Rx(90 deg)): slot 0 / 4 are the lowest
    # points of the two caps, exactly on the contact line
    R = _Rx(math.pi / 2)
    for c in (0, 4):
        w = R @ _slot(oracle, R, c)
        assert w[2] == pytest.approx(-0.1, abs=1e-15)
    w = np.array([R @ _slot(oracle, R, c) for c in range(8)])
    assert w[:, 2].min() == pytest.approx(-0.1)
    # tilted: slot 0 of the lower cap is the deepest of all rim points
    R = _Rx(0.3)
    w0 = R @ _slot(oracle, R, 0)
    ang = np.linspace(0, 2 * np.pi, 721)
    rim = np.stack([0.1 * np.cos(ang), 0.1 * np.sin(ang), np.full_like(ang, -0.2)], 1) @ R.T
    assert w0[2] == pytest.approx(rim[:, 2].min(), abs=1e-6)


def test_standing_cylinder_carries_its_weight(oracle):
    cm = oracle.load_urdf(cylinder_urdf(), pose_xyz=(0, 0, 0.25))
    w = oracle.FreeWorld(cm, mu=1.0)
    for _ in range(600):
        w.step()
    assert w.p[2] == pytest.approx(0.2, abs=2e-3)
    assert len(w.contacts) == 4
    fz = sum(c[2][2] for c in w.contacts)
    assert fz == pytest.approx(2.0 * G, abs=0.05)
    for p, n, f, d in w.contacts:
        assert list(n) == [0, 0, 1]


def test_lying_cylinder_rolls_without_slipping(oracle):
    r, m = 0.1, 2.0
    # the collision cylinder lies along the body x axis (rpy: pitch 90 deg)
    ixx = m * (3 * r * r + 0.16) / 12.0
    text = (f'<robot name="roll"><link name="roll"><inertial><mass value="{m}"/>'
            f'<inertia ixx="{0.5 * m * r * r}" iyy="{ixx}" izz="{ixx}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><origin rpy="0 {math.pi / 2} 0" xyz="0 0 0"/><geometry>'
            f'<cylinder radius="{r}" length="0.4"/></geometry></collision></link></robot>')
    cm = oracle.load_urdf(text, pose_xyz=(0, 0, r))
    w = oracle.FreeWorld(cm, mu=1.0, pgs_iters=100)
    for _ in range(100):
        w.step()
    assert len(w.contacts) == 2
    w0 = -10.0   # spin about +x: rolls towards +y
    w.set_twist([w0, 0, 0], [0, 0, 0])
    for _ in range(1500):
        w.step()
    om, v = w.twist
    vw = w.R @ v
    omw = w.R @ om
    assert vw[1] == pytest.approx(-omw[0] * r, rel=0.02)           # rolling: v = omega r
    assert vw[1] == pytest.approx(-w0 * r / 3.0, rel=0.03)          # I = m r^2 / 2
    assert w.p[2] == pytest.approx(r, abs=2e-3) and abs(vw[0]) < 1e-3
    assert len(w.contacts) == 2


def test_cylinder_geometry_compiles_alike(oracle):
    from mwstep import native as N
    from test_sdf_models import _compile, _compare
    N.lib()
    rc, got = _compile(N, cylinder_urdf(rpy="0.3 0.2 0.1"), (0, 0, 1, 1, 0, 0, 0))
    assert rc == 0
    sh = got["shapes"][-1]
    assert len(sh) == 1 and sh[0, 0] == 2 and list(sh[0, 1:3]) == [0.1, 0.2]
    _compare(got, oracle.load_urdf(cylinder_urdf(rpy="0.3 0.2 0.1"), pose_xyz=(0, 0, 1)))
    sdf = ("<sdf version='1.6'><model name='c'><link name='l'><collision name='k'><pose>0 0 0.1 0 0.5 0</pose>"
           "<geometry><cylinder><radius>0.05</radius><length>0.3</length></cylinder></geometry></collision>"
           "</link></model></sdf>")
    rc, got = _compile(N, sdf)
    assert rc == 0 and got["shapes"][-1][0, 0] == 2
    np.testing.assert_allclose(got["shapes"][-1][0, 1:3], [0.05, 0.15])
    _compare(got, oracle.load_urdf(sdf))


def test_cylinder_sphere_closed_forms(oracle):
    """or_collide cylinder (type 2, size {r, half length}) vs sphere: normal
    from B into A, the point on the cylinder surface; outside the solid
    (cap face, side, rim) and with the sphere centre inside it."""
    I = np.eye(3)
    cyl = [0.1, 0.2, 0.0]
    # sphere B above the top cap of cylinder A: n from B into A = -z
    n, pts, dep = oracle.collide(2, cyl, [0, 0, 0], I, 1, [0.05], [0.03, 0, 0.24], I)
    assert np.allclose(n, [0, 0, -1]) and dep[0] == pytest.approx(0.01) and np.allclose(pts[0], [0.03, 0, 0.2])
    # sphere A beside the side of cylinder B (rotated: axis along x)
    Ry = np.array([[0, 0, 1], [0, 1, 0], [-1, 0, 0]])
    n, pts, dep = oracle.collide(1, [0.05], [0.1, 0.14, 0], I, 2, cyl, [0, 0, 0], Ry)
    assert np.allclose(n, [0, 1, 0]) and dep[0] == pytest.approx(0.01) and np.allclose(pts[0], [0.1, 0.1, 0])
    # beyond the rim: the closest point is on the rim circle
    c = np.array([0.1 + 0.03, 0, 0.2 + 0.04])
    n, pts, dep = oracle.collide(2, cyl, [0, 0, 0], I, 1, [0.06], c, I)
    assert dep[0] == pytest.approx(0.06 - 0.05) and np.allclose(pts[0], [0.1, 0, 0.2])
    np.testing.assert_allclose(n, -np.array([0.6, 0, 0.8]))
    # centre inside, nearer the side than the caps
    n, pts, dep = oracle.collide(2, cyl, [0, 0, 0], I, 1, [0.05], [0.08, 0, 0.0], I)
    assert np.allclose(n, [-1, 0, 0]) and dep[0] == pytest.approx(0.07) and np.allclose(pts[0], [0.1, 0, 0])
    # apart
    assert len(oracle.collide(2, cyl, [0, 0, 0], I, 1, [0.05], [0, 0, 0.3], I)[1]) == 0
    # cylinder-box (sampled features, below): the cylinder's top rim in the box above
    n, pts, dep = oracle.collide(2, cyl, [0, 0, 0], I, 0, [0.1, 0.1, 0.1], [0, 0, 0.25], I)
    assert np.allclose(n, [0, 0, -1]) and np.allclose(dep, 0.05)


PILLAR = ('<robot name="pillar"><link name="world"/><joint name="fix" type="fixed"><parent link="world"/>'
          '<child link="p"/><origin xyz="0 0 0.3"/></joint><link name="p"><inertial><mass value="10"/>'
          '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision><geometry>'
          '<cylinder radius="0.15" length="0.6"/></geometry></collision></link></robot>')


def ball_urdf(mass=1.0, r=0.05):
    i = 0.4 * mass * r * r
    return (f'<robot name="ball"><link name="ball"><inertial><mass value="{mass}"/>'
            f'<inertia ixx="{i}" iyy="{i}" izz="{i}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><geometry><sphere radius="{r}"/></geometry></collision></link></robot>')


def test_ball_rests_on_a_pillar(oracle):
    """A ball dropped on a welded cylinder (a pillar) rests on its top cap at
    0.6 + r, carried by the cylinder-sphere contact."""
    cms = [oracle.load_urdf(PILLAR), oracle.load_urdf(ball_urdf(), pose_xyz=(0.02, 0, 0.75))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(600):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.65, abs=2e-3)
    fz = sum(c[8] for c, who in sw.contacts if 0 in (who[0], who[2]) and 1 in (who[0], who[2]))
    assert abs(fz) == pytest.approx(1.0 * G, abs=0.05)


# ---------------------------------------------------------------- cylinder pairs
# cylinder-box and cylinder-cylinder contacts between models (oracle.c
# cylinder_pair: sampled features, 8 samples per shape, the deepest
# candidate's normal, <= 4 points)

TABLE = ('<robot name="table"><link name="world"/><joint name="fix" type="fixed"><parent link="world"/>'
         '<child link="t"/><origin xyz="0 0 0.25"/></joint><link name="t"><inertial><mass value="10"/>'
         '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision><geometry>'
         '<box size="0.8 0.8 0.1"/></geometry></collision></link></robot>')   # top face at z = 0.3


def _pair_force(sw, a, b):
    return sum(c[8] if who[0] == b else -c[8] for c, who in sw.contacts
               if {who[0], who[2]} == {a, b})


def test_cylinder_box_closed_forms(oracle):
    """cylinder A (r 0.1, half length 0.2) standing 0.01 deep in a box B top:
    4 bottom-rim points, normal +z (B into A), depth 0.01; lying 0.02 deep:
    the two rim points facing the box; apart: nothing"""
    I = np.eye(3)
    hb, cb = [0.4, 0.4, 0.05], [0.0, 0.0, 0.0]
    nrm, pts, dep = oracle.collide(2, [0.1, 0.2, 0], [0, 0, 0.24], I, 0, hb, cb, I)
    assert len(dep) == 4
    np.testing.assert_allclose(nrm, [0, 0, 1], atol=1e-12)
    np.testing.assert_allclose(dep, 0.01, atol=1e-12)
    np.testing.assert_allclose(pts[:, 2], 0.04, atol=1e-12)
    np.testing.assert_allclose(np.hypot(pts[:, 0], pts[:, 1]), 0.0999, atol=1e-12)
    Ry = np.array([[0, 0, 1], [0, 1, 0], [-1, 0, 0]], dtype=float)   # axis along x
    nrm, pts, dep = oracle.collide(2, [0.1, 0.2, 0], [0, 0, 0.13], Ry, 0, hb, cb, I)
    assert len(dep) == 2
    np.testing.assert_allclose(nrm, [0, 0, 1], atol=1e-12)
    np.testing.assert_allclose(sorted(pts[:, 0]), [-0.2, 0.2], atol=1e-12)
    np.testing.assert_allclose(dep, 0.05 - (0.13 - 0.0999), atol=1e-12)
    assert len(oracle.collide(2, [0.1, 0.2, 0], [0, 0, 0.26], I, 0, hb, cb, I)[2]) == 0
    # B into A is reversed when the box is A
    nrm, _, _ = oracle.collide(0, hb, cb, I, 2, [0.1, 0.2, 0], [0, 0, 0.24], I)
    np.testing.assert_allclose(nrm, [0, 0, -1], atol=1e-12)


def test_cylinder_stands_on_a_table(oracle):
    cms = [oracle.load_urdf(TABLE), oracle.load_urdf(cylinder_urdf(2.0, 0.1, 0.4), pose_xyz=(0.05, 0, 0.55))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(800):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.3 + 0.2, abs=2e-3)
    assert np.abs(sw.V(1)).max() < 1e-3
    assert _pair_force(sw, 0, 1) == pytest.approx(2.0 * G, abs=0.05)


def test_lying_cylinder_rests_on_a_table(oracle):
    cms = [oracle.load_urdf(TABLE),
           oracle.load_urdf(cylinder_urdf(2.0, 0.1, 0.4, rpy="1.5707963267948966 0 0"), pose_xyz=(0, 0, 0.45))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(800):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.3 + 0.1, abs=2e-3)
    assert np.abs(sw.V(1)).max() < 1e-3
    assert _pair_force(sw, 0, 1) == pytest.approx(2.0 * G, abs=0.05)


def test_two_cylinders_stack(oracle):
    """equal radii, coaxial: the rim samples sit at 0.999 r, so the stack
    holds; the lower one carries both weights on the ground"""
    cms = [oracle.load_urdf(cylinder_urdf(2.0, 0.1, 0.4, name="low"), pose_xyz=(0, 0, 0.2)),
           oracle.load_urdf(cylinder_urdf(1.0, 0.1, 0.2, name="high"), pose_xyz=(0.01, 0, 0.51))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(800):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.4 + 0.1, abs=2e-3)
    assert _pair_force(sw, 0, 1) == pytest.approx(1.0 * G, abs=0.05)
    ground = sum(c[8] for c, who in sw.contacts if who[2] < 0)
    assert ground == pytest.approx(3.0 * G, abs=0.05)
