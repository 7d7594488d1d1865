"""The mesh narrow phase against other models (CPU; VERDICT r5 missing #3).

The reference attaches a <mesh> collision to DART as its triangle mesh
(cpp/scenario/plugins/Physics/Physics.cpp:897-931) [EXT].  Rounds 2-5 let a
mesh collide with other models as its bounding box; now a mesh collides with
boxes and other meshes as the convex hull of its support points
(oracle.c hull_pair, scene_kernel.hip sc_hull_pair: separating axes over both
face-normal sets and the Gauss-map-pruned edge pairs, reference-face
clipping).  Pinned here:

  * the hull: the oracle's brute-force construction equals scipy's Qhull
    (scipy.spatial.ConvexHull, coplanar triangles merged) and the library's
    host build (csrc/hull.hpp, mw_debug_hull) face for face;
  * closed forms of the narrow phase: a regular tetrahedron resting on a box
    face (normal, depth, 3 points = its base corners), an upside-down one on
    its apex, two crossing edges (one point at the crossing, depth = the
    overlap);
  * scene KATs: a tetrahedron mesh comes to rest ON ITS FACE with its
    centroid h/4 above the table, and carries its weight; a cube resting
    across a slanted edge of a hexagonal mesh platform with its centre over
    the platform stays put; one placed with its centre beyond that edge but
    over the platform's bounding box tips off (the bounding box held it).
"""

import ctypes

import numpy as np
import pytest

from mesh_models import write_obj
from scene_models import cube_urdf

G = 9.8


def _tetra(edge=0.2):
    """regular tetrahedron with a horizontal base face, centroid at the origin"""
    h = edge * np.sqrt(2.0 / 3.0)
    r = edge / np.sqrt(3.0)
    base = [[r * np.cos(a), r * np.sin(a), -h / 4] for a in (0.0, 2 * np.pi / 3, 4 * np.pi / 3)]
    return np.array(base + [[0.0, 0.0, 3 * h / 4]]), [(0, 2, 1), (0, 1, 3), (1, 2, 3), (2, 0, 3)], h


def _hexprism(r=0.15, half_h=0.05):
    v = [[r * np.cos(k * np.pi / 3), r * np.sin(k * np.pi / 3), z] for z in (-half_h, half_h) for k in range(6)]
    tris = []
    for k in range(6):
        a, b = k, (k + 1) % 6
        tris += [(a, b, 6 + b), (a, 6 + b, 6 + a)]
    tris += [(0, k + 1, k) for k in range(1, 5)] + [(6, 6 + k, 6 + k + 1) for k in range(1, 5)]
    return np.array(v), tris


def _scipy_planes(pts):
    from scipy.spatial import ConvexHull
    hull = ConvexHull(pts)
    planes = []
    for eq in hull.equations:   # n . x + c <= 0 inside
        n, d = eq[:3], -eq[3]
        if not any(np.abs(n - q[:3]).max() < 1e-9 and abs(d - q[3]) < 1e-9 for q in planes):
            planes.append(np.concatenate([n, [d]]))
    return np.array(planes)


def _same_planes(a, b, tol=1e-9):
    return len(a) == len(b) and all(np.abs(b - p).max(axis=1).min() < tol for p in a)


@pytest.mark.parametrize("case", ["ellipsoid", "cube", "hexprism", "tetra", "rock"])
def test_hull_equals_qhull_and_the_library(oracle, case):
    from mesh_models import rock_vertices
    from mwstep import native as N
    rng = np.random.default_rng(3)
    if case == "ellipsoid":
        d = rng.normal(size=(16, 3))
        pts = d / np.linalg.norm(d, axis=1, keepdims=True) * [0.2, 0.1, 0.07]
    elif case == "cube":
        pts = np.array([[sx, sy, sz] for sx in (-0.1, 0.1) for sy in (-0.1, 0.1) for sz in (-0.1, 0.1)])
    elif case == "hexprism":
        pts = _hexprism()[0]
    elif case == "tetra":
        pts = _tetra()[0]
    else:
        pts = rock_vertices(2)[0]
    h = oracle.hull(pts)
    ours = np.column_stack([h["n"], h["d"]])
    assert _same_planes(ours, _scipy_planes(pts))
    # every face polygon lies on its plane, counter-clockwise seen from outside
    for n, d, face in zip(h["n"], h["d"], h["faces"]):
        P = pts[face]
        assert np.abs(P @ n - d).max() < 1e-12
        c = P.mean(axis=0)
        for k in range(len(face)):
            assert np.dot(np.cross(P[k] - c, P[(k + 1) % len(face)] - c), n) > 0
    # Euler: V - E + F = 2; every edge between two distinct faces
    assert len(pts) - len(h["edges"]) + len(h["n"]) == 2
    assert (h["edge_faces"][:, 0] != h["edge_faces"][:, 1]).all()
    # the library's host build (the scene kernel's hull) is the same hull
    p = np.ascontiguousarray(pts, dtype=float)
    planes, faces = np.zeros(32 * 4), np.zeros(32 * 17, np.int32)
    edges, counts = np.zeros(48 * 4, np.int32), np.zeros(2, np.int32)
    ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    assert N.lib().mw_debug_hull(N.dptr(p), len(p), N.dptr(planes), ip(faces), ip(edges), ip(counts)) == 0
    nf, ne = counts
    assert nf == len(h["n"]) and ne == len(h["edges"])
    np.testing.assert_allclose(planes.reshape(32, 4)[:nf], ours, atol=1e-12)
    f17 = faces.reshape(32, 17)
    assert [list(f17[f, 1:1 + f17[f, 0]]) for f in range(nf)] == h["faces"]
    e4 = edges.reshape(48, 4)[:ne]
    assert np.array_equal(e4[:, :2], h["edges"]) and np.array_equal(e4[:, 2:], h["edge_faces"])


def test_flat_point_sets_have_no_hull(oracle):
    pts = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0.0]])
    assert oracle.hull(pts) is None


def test_tetrahedron_on_a_box_face_closed_form(oracle):
    v, _, h = _tetra(0.2)
    box, top = np.array([0.3, 0.3, 0.05]), 0.05
    I = np.eye(3).reshape(-1)
    pen = 1e-3
    c = np.array([0.02, -0.01, top + h / 4 - pen])   # base face 1 mm into the box top
    n, pts, dep = oracle.collide_hull(3, np.abs(v).max(axis=0), v, c, I, 0, box, None, [0, 0, 0], I)
    np.testing.assert_allclose(n, [0, 0, 1], atol=1e-12)   # from the box into the tetrahedron
    assert len(pts) == 3
    np.testing.assert_allclose(dep, pen, atol=1e-12)
    np.testing.assert_allclose(np.sort(pts[:, 0]), np.sort(v[:3, 0] + c[0]), atol=1e-12)
    # apex down: one point at the apex
    Rx = np.diag([1.0, -1.0, -1.0]).reshape(-1)
    c2 = np.array([0.0, 0.0, top + 3 * h / 4 - pen])
    n, pts, dep = oracle.collide_hull(3, np.abs(v).max(axis=0), v, c2, Rx, 0, box, None, [0, 0, 0], I)
    assert len(pts) == 1
    np.testing.assert_allclose(n, [0, 0, 1], atol=1e-9)
    np.testing.assert_allclose(pts[0], [0, 0, top - pen], atol=1e-12)
    np.testing.assert_allclose(dep, pen, atol=1e-12)


def test_crossing_edges_closed_form(oracle):
    """a wedge's ridge (along y) under a tetrahedron-like wedge's ridge along x
    (edge down): one point at the crossing, depth = the vertical overlap"""
    wedge = np.array([[-0.1, -0.2, 0.0], [0.1, -0.2, 0.0], [0.0, -0.2, 0.1],
                      [-0.1, 0.2, 0.0], [0.1, 0.2, 0.0], [0.0, 0.2, 0.1]])   # ridge at z = 0.1 along y
    wc = wedge - wedge.mean(axis=0)
    Rz = np.array([[0, -1.0, 0], [1.0, 0, 0], [0, 0, 1.0]])                  # ridge along x
    Rflip = Rz @ np.diag([1.0, -1.0, -1.0])                                  # and upside down
    pen = 2e-3
    ca = np.array([0.0, 0.0, 0.1 + (wc[:, 2].max()) - pen])   # upper wedge: its ridge 2 mm below z = 0.1
    cb = wedge.mean(axis=0)
    n, pts, dep = oracle.collide_hull(3, np.abs(wc).max(axis=0), wc, ca, Rflip.reshape(-1), 3,
                                      np.abs(wc).max(axis=0), wc, cb, np.eye(3).reshape(-1))
    assert len(pts) == 1
    np.testing.assert_allclose(n, [0, 0, 1], atol=1e-9)
    np.testing.assert_allclose(pts[0], [0.0, 0.0, 0.1 - pen / 2], atol=1e-9)
    np.testing.assert_allclose(dep, pen, atol=1e-9)


def _table(top=0.3, half=(0.3, 0.3, 0.05)):
    return ('<robot name="table"><link name="world"/><link name="top"><inertial><mass value="1"/>'
            '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision>'
            f'<geometry><box size="{2 * half[0]} {2 * half[1]} {2 * half[2]}"/></geometry></collision></link>'
            '<joint name="weld" type="fixed"><parent link="world"/><child link="top"/>'
            f'<origin xyz="0 0 {top - half[2]}"/></joint></robot>')


def test_tetrahedron_rests_on_its_face(oracle, tmp_path):
    from mesh_models import mesh_body_urdf
    v, tris, h = _tetra(0.2)
    path = str(tmp_path / "tetra.obj")
    write_obj(path, v, tris)
    m = 1.5
    cms = [oracle.load_urdf(_table()), oracle.load_urdf(mesh_body_urdf(path, mass=m, half=(0.06, 0.06, 0.06)),
                                                        pose_xyz=(0.0, 0.0, 0.3 + h / 4 + 0.01))]
    assert cms[1].base_shapes[0][0] == 3
    sw = oracle.SceneWorld(cms, pgs_iters=oracle.PGS_CONVERGED)
    for _ in range(800):
        sw.step()
    # the centroid sits h / 4 above the table (the bounding box would hold it at
    # half its height, 0.5 h above the box centre offset)
    assert sw.p(1)[2] == pytest.approx(0.3 + h / 4, abs=2e-4)
    assert np.abs(sw.V(1)).max() < 1e-3
    pair = [(c, who) for c, who in sw.contacts if who[0] == 0 and who[2] == 1 or who[0] == 1 and who[2] == 0]
    assert len(pair) == 3
    assert abs(sum(c[8] for c, _ in pair)) == pytest.approx(m * G, abs=0.05)


@pytest.mark.parametrize("dist, stays", [(0.10, True), (0.16, False)])
def test_cube_across_a_mesh_platform_edge(oracle, tmp_path, dist, stays):
    """a welded hexagonal-prism mesh platform (circumradius 0.15, vertices at
    0, 60, ... degrees: the slanted edge between the 0 and 60 degree vertices
    runs 0.13 from the centre along 30 degrees, while the bounding box reaches
    (0.15, 0.13)) and a 0.1 m cube placed along 30 degrees.  At 0.10 from the
    centre the cube hangs over the slanted edge with its centre over the
    platform: it rests there and the platform carries its weight.  At 0.16
    its centre is beyond the edge but still over the bounding box: it tips
    off the hull (the bounding box stand-in of rounds 2-5 held it)."""
    from mesh_models import mesh_body_urdf  # noqa: F401
    v, tris = _hexprism(0.15, 0.05)
    path = str(tmp_path / "hex.obj")
    write_obj(path, v, tris)
    platform = ('<robot name="platform"><link name="world"/><link name="top"><inertial><mass value="1"/>'
                '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision>'
                f'<geometry><mesh filename="{path}"/></geometry></collision></link>'
                '<joint name="weld" type="fixed"><parent link="world"/><child link="top"/>'
                '<origin xyz="0 0 0.25"/></joint></robot>')
    xy = dist * np.array([np.cos(np.pi / 6), np.sin(np.pi / 6)])
    assert xy[0] < 0.15 and xy[1] < 0.13            # over the bounding box either way
    cms = [oracle.load_urdf(platform), oracle.load_urdf(cube_urdf(mass=1.0, edge=0.1),
                                                        pose_xyz=(xy[0], xy[1], 0.3 + 0.05))]
    assert cms[0].base_shapes[0][0] == 3
    sw = oracle.SceneWorld(cms, pgs_iters=oracle.PGS_CONVERGED)
    p0 = sw.p(1).copy()
    for _ in range(600):
        sw.step()
    moved = float(np.abs(sw.p(1) - p0).max())
    if stays:
        assert moved < 2e-3
        pair = [c for c, who in sw.contacts if who[2] == 1 or who[0] == 1]
        assert abs(sum(c[8] for c in pair)) == pytest.approx(1.0 * G, abs=0.05)
    else:
        assert moved > 0.02 and sw.p(1)[2] < p0[2] - 0.01
