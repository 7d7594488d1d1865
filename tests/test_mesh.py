"""Mesh collisions (reference Physics.cpp:897-931: a <mesh> collision is loaded
from its URI and attached with the collision pose and the SDF <scale>), CPU
side:

  * the model compiler (gym-ignition_amd/csrc/mesh.cpp via mw_compile_collisions)
    and the oracle's independent numpy restatement (pyoracle.mesh_shape) give
    the same shape: bounding box, pose, support points -- for binary STL, ASCII
    STL, OBJ and COLLADA files (node transforms, units), URDF and SDF front-ends, scales and collision poses,
    relative / file:// / model:// URIs;
  * a box-shaped mesh IS the box: its support points are the 8 corners in the
    box's slot order, so a scene with the mesh cube steps bit-identically to
    the same scene with the box cube;
  * KATs on the fp64 scene oracle: an irregular mesh dropped on the ground
    comes to rest with its weight carried by its support points, and a mesh
    body rests on a box of another model (the hull narrow phase against other
    models is pinned in tests/test_mesh_hull.py);
  * loud failures: unsupported formats, missing files, a free body with more
    shape entries than mw_sim's free-body kernel holds.

Mesh-vs-plane contact in DART (FCL / ODE collision detectors [EXT]) generates
points from the triangles; the support-point restatement is pinned by the
box identity and the weight KATs, not by DART itself (parity unpinned).
"""

import ctypes
import os

import numpy as np
import pytest

from mesh_models import (CUBE_TRIS, cube_vertices, mesh_body_sdf, mesh_body_urdf, rock_vertices, write_obj,
                         write_stl_ascii, write_stl_binary)
from scene_models import cube_urdf

G = 9.8
IDENT = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)


@pytest.fixture(scope="module")
def N():
    from mwstep import native
    native.lib()
    return native


WORDS = 66   # MW_COLLISION_WORDS (include/mwstep.h)


def _collisions(N, text, pose=IDENT):
    out, c = np.zeros(64 * WORDS), ctypes.c_int32()
    rc = N.lib().mw_compile_collisions(text.encode(), N.dptr(np.asarray(pose, dtype=np.float64)), N.dptr(out), 64,
                                       ctypes.byref(c))
    if rc:
        return rc, N.last_error()
    return 0, out[:WORDS * c.value].reshape(c.value, WORDS)


def _check_against_oracle(got, cm, tol=1e-12):
    ref = [(-1, *s) for s in cm.base_shapes] + list(cm.body_shapes)
    assert len(got) == len(ref)
    for g, (b, t, sz, SR, sp) in zip(got, ref):
        assert int(g[0]) == b and int(g[1]) == t
        np.testing.assert_allclose(g[2:5], sz[:3], atol=tol)
        np.testing.assert_allclose(g[5:14].reshape(3, 3), SR, atol=tol)
        np.testing.assert_allclose(g[14:17], sp, atol=tol)
        if t == 3:
            pts = np.asarray(sz[3:]).reshape(-1, 3)
            assert int(g[17]) == len(pts)
            np.testing.assert_allclose(g[18:18 + 3 * len(pts)].reshape(-1, 3), pts, atol=tol)


def test_box_mesh_is_the_box(N, oracle, tmp_path):
    v = cube_vertices((0.1, 0.1, 0.1))
    for fmt, write in (("stl", write_stl_binary), ("ascii.stl", write_stl_ascii), ("obj", write_obj)):
        path = str(tmp_path / f"cube.{fmt}")
        write(path, v, CUBE_TRIS)
        rc, got = _collisions(N, mesh_body_urdf(path))
        assert rc == 0, got
        assert got.shape[0] == 1 and int(got[0, 1]) == 3 and int(got[0, 17]) == 8
        np.testing.assert_allclose(got[0, 2:5], [0.1, 0.1, 0.1], atol=1e-7)
        np.testing.assert_allclose(got[0, 18:42].reshape(8, 3), v, atol=1e-7)   # the box corner order
        cm = oracle.load_urdf(mesh_body_urdf(path))
        _check_against_oracle(got, cm)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_compiler_matches_oracle_restatement(N, oracle, tmp_path, seed):
    rng = np.random.default_rng(seed)
    v, f = rock_vertices(seed)
    write_stl_binary(str(tmp_path / "rock.stl"), v, f)
    write_obj(str(tmp_path / "rock.obj"), v, f)
    scale = tuple(rng.uniform(0.5, 2.0, 3).round(3))
    xyz = tuple(rng.uniform(-0.1, 0.1, 3).round(3))
    rpy = tuple(rng.uniform(-1, 1, 3).round(3))
    for uri in (str(tmp_path / "rock.stl"), "file://" + str(tmp_path / "rock.obj")):
        text = mesh_body_urdf(uri, scale=scale, xyz=xyz, rpy=rpy)
        rc, got = _collisions(N, text)
        assert rc == 0, got
        cm = oracle.load_urdf(text)
        _check_against_oracle(got, cm)
        assert int(got[0, 17]) == 12   # every hull vertex of the 12-vertex rock
        # every support point is a (scaled) vertex of the mesh
        pts = got[0, 18:18 + 3 * int(got[0, 17])].reshape(-1, 3) + (
            np.asarray(got[0, 14:17]) - np.asarray(xyz)) @ oracle._rpy(rpy)   # back to the mesh frame
        d = np.abs(pts[:, None, :] - v[None, :, :] * np.asarray(scale)).max(axis=2).min(axis=1)
        assert d.max() < 1e-9
    sdf = mesh_body_sdf(str(tmp_path / "rock.stl"), scale=scale, pose=" ".join(str(x) for x in xyz + rpy))
    rc, got = _collisions(N, sdf)
    assert rc == 0, got
    _check_against_oracle(got, oracle.load_urdf(sdf), tol=1e-10)


def test_relative_and_model_uris(N, oracle, tmp_path, monkeypatch):
    v, f = rock_vertices(5)
    d = tmp_path / "models" / "rock" / "meshes"
    d.mkdir(parents=True)
    write_stl_ascii(str(d / "rock.stl"), v, f)
    model_file = tmp_path / "models" / "rock" / "model.urdf"
    model_file.write_text(mesh_body_urdf("meshes/rock.stl"))
    rc, rel = _collisions(N, str(model_file))
    assert rc == 0, rel
    _check_against_oracle(rel, oracle.load_urdf(str(model_file)))
    monkeypatch.setenv("GZ_SIM_RESOURCE_PATH", str(tmp_path / "models"))
    rc, mod = _collisions(N, mesh_body_urdf("model://rock/meshes/rock.stl"))
    assert rc == 0, mod
    np.testing.assert_array_equal(rel, mod)
    # ScenarI/O insert_model(file): relative URIs resolve against the file's directory
    from scenario.gazebo import _absolute_mesh_uris
    assert str(d / "rock.stl") in _absolute_mesh_uris(model_file.read_text(), str(model_file.parent))


@pytest.mark.parametrize("text,needle", [
    (mesh_body_urdf("/nonexistent/rock.stl"), "cannot open mesh"),
    (mesh_body_urdf("/tmp/rock.ply"), "STL, OBJ and COLLADA"),
    (mesh_body_urdf("model://nowhere/rock.stl"), "cannot resolve"),
])
def test_bad_meshes_fail_loudly(N, text, needle):
    rc, msg = _collisions(N, text)
    assert rc == N.MW_EPARSE and needle in msg


@pytest.mark.parametrize("exact", [False, True])
def test_mw_sim_free_body_mesh_entries(N, tmp_path, exact):
    """mw_sim's PGS-only free-body kernel (MW_LCP_PGS chosen before the load)
    holds 2 shape entries of 8 slots: a mesh takes one entry per 8 support
    points; beyond 2 entries the model fails loudly.  With the exact LCP (the
    default) a joint-less body steps on the world-per-wavefront kernel, where
    a mesh is one zero-radius sphere per support point (16 shapes, 32 slots):
    all three bodies load."""
    path = str(tmp_path / "cube.stl")
    write_stl_binary(path, cube_vertices(), CUBE_TRIS)
    v, f = rock_vertices(7)
    rock = str(tmp_path / "rock.stl")
    write_stl_binary(rock, v, f)
    cfg = N.MwConfig(1e-3, 1.0, 1, 2, 0, 0)
    for uri, extra, ok in ((path, "", True), (rock, "", True), (rock, '<collision><geometry><box size="0.1 0.1 0.1"/>'
                                                                     '</geometry></collision>', exact)):
        h = ctypes.c_void_p()
        N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
        try:
            if not exact:
                N.check(N.lib().mw_set_lcp_solver(h, N.LCP_PGS, 0))
            text = mesh_body_urdf(uri).replace("</link>", extra + "</link>")
            rc = N.lib().mw_load_model(h, text.encode(), N.dptr(IDENT), b"")
            assert (rc == 0) == ok, N.last_error()
            if not ok:
                assert rc == N.MW_EPARSE and "entries" in N.last_error()
            else:
                m, k = ctypes.c_int32(), ctypes.c_int32()
                N.check(N.lib().mw_lcp_solver(h, ctypes.byref(m), ctypes.byref(k)))
                assert (m.value == N.LCP_EXACT) == exact
        finally:
            N.lib().mw_destroy(h)


def test_mesh_cube_scene_equals_box_scene(oracle, tmp_path):
    """The mesh cube's slots are the box's corners in the box's order, so the
    whole scene (drop, tumble, a box cube landing on it) is bit-identical."""
    path = str(tmp_path / "cube.stl")
    write_stl_binary(path, cube_vertices((0.125, 0.125, 0.125)), CUBE_TRIS)   # exact in float32
    box = cube_urdf(mass=5.0, edge=0.25)
    mesh = box.replace('<box size="0.25 0.25 0.25"/>', f'<mesh filename="{path}"/>')
    assert mesh != box
    worlds = []
    for first in (box, mesh):
        cms = [oracle.load_urdf(first, pose_xyz=(0, 0, 0.3)), oracle.load_urdf(cube_urdf(), pose_xyz=(0.05, 0, 0.7))]
        sw = oracle.SceneWorld(cms, pgs_iters=50)
        sw.set_twist(0, [1.0, -2.0, 0.5], [0.2, 0.0, 0.0])
        worlds.append(sw)
    for _ in range(400):
        n = [sw.step() for sw in worlds]
        assert n[0] == n[1]
    a, b = worlds
    for m in range(2):
        np.testing.assert_array_equal(a.p(m), b.p(m))
        np.testing.assert_array_equal(a.V(m), b.V(m))
    assert any(who[2] == 0 or who[0] == 0 and who[2] == 1 for c, who in a.contacts)


def test_rock_comes_to_rest_on_its_support_points(oracle, tmp_path):
    v, f = rock_vertices(1)
    path = str(tmp_path / "rock.obj")
    write_obj(path, v, f)
    cm = oracle.load_urdf(mesh_body_urdf(path, mass=3.0, half=(0.12, 0.08, 0.06)), pose_xyz=(0, 0, 0.3))
    sw = oracle.SceneWorld([cm], pgs_iters=50, mu=0.8)
    rng = np.random.default_rng(0)
    sw.set_twist(0, rng.uniform(-2, 2, 3), [0.3, -0.2, 0.0])
    for _ in range(2500):
        nc = sw.step()
    assert nc >= 3
    fz = sum(c[8] for c, who in sw.contacts)
    assert fz == pytest.approx(3.0 * G, abs=0.1)
    assert np.abs(sw.V(0)).max() < 1e-3
    # every contact is one of the support points, in contact with the plane
    R, p = sw.R(0), sw.p(0)
    shape = cm.base_shapes[0]
    pts = np.asarray(shape[1][3:]).reshape(-1, 3)
    world = p + (shape[3] + pts @ shape[2].T) @ R.T
    assert world[:, 2].min() > -2e-3          # nothing sinks in
    for c, who in sw.contacts:
        assert np.abs(world - c[0:3]).max(axis=1).min() < 1e-9


def test_mesh_body_rests_on_a_box_of_another_model(oracle, tmp_path):
    """a cube-shaped mesh rests on a box of another model (a mesh whose support
    points are its bounding box corners keeps the box narrow phase; other
    meshes use their convex hull, tests/test_mesh_hull.py)"""
    path = str(tmp_path / "cube.stl")
    write_stl_binary(path, cube_vertices((0.05, 0.05, 0.05)), CUBE_TRIS)
    table = ('<robot name="table"><link name="world"/><link name="top"><inertial><mass value="1"/>'
             '<inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" iyz="0"/></inertial><collision>'
             '<geometry><box size="0.6 0.6 0.1"/></geometry></collision></link>'
             '<joint name="weld" type="fixed"><parent link="world"/><child link="top"/>'
             '<origin xyz="0 0 0.3"/></joint></robot>')
    cms = [oracle.load_urdf(table), oracle.load_urdf(mesh_body_urdf(path, mass=1.0, half=(0.05,) * 3),
                                                     pose_xyz=(0, 0, 0.45))]
    sw = oracle.SceneWorld(cms, pgs_iters=50)
    for _ in range(600):
        sw.step()
    assert sw.p(1)[2] == pytest.approx(0.35 + 0.05, abs=2e-3)
    fz = sum(c[8] for c, who in sw.contacts if who[2] == 1 or who[0] == 1)
    assert abs(fz) == pytest.approx(1.0 * G, abs=0.1)


def test_collada_meshes(N, oracle, tmp_path):
    """COLLADA: the instanced geometries under their node transforms (matrix,
    translate, rotate, scale; nested nodes), times <unit meter>; a geometry no
    node instantiates is ignored.  Exact-arithmetic case checked against a
    hand-computed box, rotated rock case C++ == oracle."""
    from mesh_models import write_dae
    cube = cube_vertices((2.0, 2.0, 2.0))
    far = cube + 100.0                                   # not instantiated
    perm = "<matrix>0 1 0 1 0 0 1 0 1 0 0 2 0 0 0 1</matrix>"   # x' = y + 1, y' = z, z' = x + 2
    path = str(tmp_path / "cube.dae")
    write_dae(path, {"cube": cube, "far": far}, [(perm, ["cube"], [])], unit=0.0625)
    rc, got = _collisions(N, mesh_body_urdf(path))
    assert rc == 0, got
    assert int(got[0, 1]) == 3 and int(got[0, 17]) == 8
    np.testing.assert_array_equal(got[0, 2:5], [0.125, 0.125, 0.125])
    np.testing.assert_array_equal(got[0, 14:17], [0.0625, 0.0, 0.125])   # box centre (mesh frame)
    _check_against_oracle(got, oracle.load_urdf(mesh_body_urdf(path)), tol=0.0)
    # the same box as STL gives the same shape
    stl = str(tmp_path / "cube.stl")
    write_stl_binary(stl, cube_vertices((0.125,) * 3) + [0.0625, 0.0, 0.125], CUBE_TRIS)
    rc, ref = _collisions(N, mesh_body_urdf(stl))
    np.testing.assert_array_equal(got[0, 2:17], ref[0, 2:17])
    # nested nodes with translate / rotate / scale, a rock instanced twice
    v, f = rock_vertices(3)
    nodes = [("<translate>0.5 0 0</translate><rotate>0 0 1 30</rotate>", ["rock"],
              [("<scale>1 2 1</scale><translate>0 0 0.25</translate>", ["rock"], [])])]
    path = str(tmp_path / "rock.dae")
    write_dae(path, {"rock": v}, nodes, unit=1.0)
    text = mesh_body_urdf(path, scale=(1.0, 0.5, 2.0))
    rc, got = _collisions(N, text)
    assert rc == 0, got
    _check_against_oracle(got, oracle.load_urdf(text), tol=1e-12)
    assert int(got[0, 17]) >= 8


def test_degenerate_meshes(N, oracle, tmp_path):
    """an empty file fails loudly; a flat mesh (a square) is a zero-thickness
    box whose support points are its 4 corners, alike in both compilers"""
    empty = tmp_path / "empty.obj"
    empty.write_text("# nothing\n")
    rc, msg = _collisions(N, mesh_body_urdf(str(empty)))
    assert rc == N.MW_EPARSE and "no vertices" in msg
    sq = np.array([[-0.1, -0.1, 0], [0.1, -0.1, 0], [0.1, 0.1, 0], [-0.1, 0.1, 0]], dtype=float)
    path = str(tmp_path / "square.obj")
    write_obj(path, sq, [(0, 1, 2), (0, 2, 3)])
    rc, got = _collisions(N, mesh_body_urdf(path, rpy=(0.3, 0, 0)))
    assert rc == 0, got
    np.testing.assert_allclose(got[0, 2:5], [0.1, 0.1, 0.0], atol=1e-12)
    assert int(got[0, 17]) == 4
    pts = got[0, 18:30].reshape(4, 3)
    np.testing.assert_allclose(sorted(map(tuple, pts)), sorted(map(tuple, sq)), atol=1e-12)
    _check_against_oracle(got, oracle.load_urdf(mesh_body_urdf(path, rpy=(0.3, 0, 0))))
