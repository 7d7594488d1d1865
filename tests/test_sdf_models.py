"""SDF models through the product's C++ compiler (host side, no GPU).

The reference inserts SDF models as well as URDF ones
(World::insertModelFromString, cpp/scenario/gazebo/src/World.cpp:416-429;
tests/test_scenario/test_world.py:129-134 inserts the SDF cube of
tests/common/utils.py:100-146).  The product's SDF front-end
(csrc/model.cpp: describe_sdf) is checked against the oracle's independent
reader, which rewrites the SDF as URDF text with numpy frame algebra
(oracle/pyoracle.py: sdf_to_urdf) and compiles that: random trees with link
poses, joint poses, axes in the joint or the model frame, fixed joints
(lumped), limits, and the three ways a model meets the world (floating, welded,
hinged to the world)."""

import ctypes

import numpy as np
import pytest

# tests/common/utils.py:100-146 (the reference's SDF cube)
REF_CUBE_SDF = """<?xml version="1.0" ?>
<sdf version="1.6">
    <model name='box'>
    <pose>0 0 0.5 0 -0 0</pose>
        <link name='box_link'>
            <inertial>
            <inertia>
                <ixx>1</ixx><ixy>0</ixy><ixz>0</ixz><iyy>1</iyy><iyz>0</iyz><izz>1</izz>
            </inertia>
            <mass>1</mass>
            </inertial>
            <collision name='box_collision'>
            <geometry><box><size>1 1 1</size></box></geometry>
            <surface><friction><ode/></friction><contact/></surface>
            </collision>
            <visual name='box_visual'>
            <geometry><box><size>1 1 1</size></box></geometry>
            <material><ambient>1 0 0 1</ambient></material>
            </visual>
        </link>
    </model>
</sdf>"""

IDENT = (0, 0, 0, 1, 0, 0, 0)


@pytest.fixture(scope="module")
def N():
    from mwstep import native
    native.lib()
    return native


def _compile(N, text, pose=IDENT):
    cfg = N.MwConfig(1e-3, 1.0, 1, 2, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array(pose, dtype=np.float64)
        rc = N.lib().mw_load_model(h, text.encode(), N.dptr(p), b"")
        if rc:
            return rc, N.last_error()
        n = ctypes.c_int32()
        N.check(N.lib().mw_dofs(h, ctypes.byref(n)))
        out = np.zeros(34 * n.value + 3)
        N.check(N.lib().mw_model_export(h, N.dptr(out), len(out)))
        base = np.zeros(23)
        N.check(N.lib().mw_model_export_base(h, N.dptr(base)))
        shapes = {}
        for b in range(-1, n.value):
            buf, c = np.zeros(16 * 16), ctypes.c_int32()
            N.check(N.lib().mw_model_export_shapes(h, b, N.dptr(buf), 16, ctypes.byref(c)))
            shapes[b] = buf[:16 * c.value].reshape(c.value, 16)
        names, links = [], []
        s = ctypes.create_string_buffer(128)
        for d in range(n.value):
            N.check(N.lib().mw_joint_name(h, d, s, 128))
            names.append(s.value.decode())
            N.check(N.lib().mw_link_name(h, d, s, 128))
            links.append(s.value.decode())
        N.lib().mw_base_frame(h, s, 128)
        return 0, dict(n=n.value, out=out, base=base, shapes=shapes, names=names, links=links,
                       base_frame=s.value.decode())
    finally:
        N.lib().mw_destroy(h)


def _quat_to_R(w, x, y, z):
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _compare(got, cm, tol=1e-10):
    """product compile (C++) == oracle compile (sdf_to_urdf + URDF reader)"""
    n, out = got["n"], got["out"]
    assert n == cm.n and got["names"] == cm.joint_names
    assert got["base_frame"] == cm.base_link
    M = cm.model
    big = lambda v: np.where(v > 1e299, np.inf, np.where(v < -1e299, -np.inf, v))
    for i in range(n):
        b = out[34 * i: 34 * (i + 1)]
        assert b[0] == M.jtype[i] and b[1] == M.limited[i], i
        np.testing.assert_allclose(b[2:11], list(M.E[i]), atol=tol)
        np.testing.assert_allclose(b[11:14], list(M.r[i]), atol=tol)
        np.testing.assert_allclose(b[14:17], list(M.axis[i]), atol=tol)
        assert b[17] == pytest.approx(M.mass[i], abs=tol)
        np.testing.assert_allclose(b[18:21], list(M.com[i]), atol=tol)
        np.testing.assert_allclose(b[21:27], list(M.Ic[i]), atol=tol)
        np.testing.assert_allclose(big(b[27:33]), [M.damping[i], M.friction[i], M.lower[i], M.upper[i],
                                                   M.effort[i], M.vel_limit[i]], atol=tol)
        assert b[33] == M.parent[i]
    np.testing.assert_allclose(out[34 * n:], list(M.gravity_base), atol=tol)
    base = got["base"]
    assert bool(base[0]) == cm.floating
    np.testing.assert_allclose(base[1:10].reshape(3, 3), cm.base_R, atol=tol)
    np.testing.assert_allclose(base[10:13], cm.base_p, atol=tol)
    if cm.floating:
        m, c, I = cm.base_inertial
        assert base[13] == pytest.approx(m)
        np.testing.assert_allclose(base[14:17], c, atol=tol)
        np.testing.assert_allclose(base[17:23], [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]], atol=tol)
        _compare_shapes(got["shapes"][-1], cm.base_shapes, tol)
    for i in range(n):
        _compare_shapes(got["shapes"][i], [s[1:] for s in cm.body_shapes if s[0] == i], tol)


def _compare_shapes(got, ref, tol):
    assert len(got) == len(ref)
    for g, (t, sz, SR, sp) in zip(got, ref):
        assert g[0] == t
        np.testing.assert_allclose(g[1:4], sz, atol=tol)
        np.testing.assert_allclose(g[4:13].reshape(3, 3), SR, atol=tol)
        np.testing.assert_allclose(g[13:16], sp, atol=tol)


def test_reference_sdf_cube(N, oracle):
    """utils.get_cube_sdf_string(): a floating unit cube, mass 1, unit inertia,
    its model <pose> kept under the identity insertion pose and replaced by any
    other (test_world.py:130-134 inserts it at [2, 0, 0], wxyz [0, 0, 0, 1])."""
    rc, got = _compile(N, REF_CUBE_SDF)
    assert rc == 0
    assert got["n"] == 0 and got["base"][0] == 1.0
    np.testing.assert_allclose(got["base"][10:13], [0, 0, 0.5])
    assert got["base"][13] == 1.0
    np.testing.assert_allclose(got["base"][17:23], [1, 1, 1, 0, 0, 0])
    sh = got["shapes"][-1]
    assert len(sh) == 1 and sh[0, 0] == 0 and list(sh[0, 1:4]) == [0.5, 0.5, 0.5]
    assert got["base_frame"] == "box_link"
    _compare(got, oracle.load_urdf(REF_CUBE_SDF))
    pose = (2, 0, 0, 0, 0, 0, 1)
    rc, got = _compile(N, REF_CUBE_SDF, pose)
    assert rc == 0
    np.testing.assert_allclose(got["base"][10:13], [2, 0, 0])
    np.testing.assert_allclose(got["base"][1:10].reshape(3, 3), _quat_to_R(0, 0, 0, 1), atol=1e-15)
    _compare(got, oracle.load_urdf(REF_CUBE_SDF, pose_xyz=pose[:3], pose_wxyz=pose[3:]))


def _pose(rng, scale=0.5, rot=True):
    p = rng.uniform(-scale, scale, 3)
    r = rng.uniform(-1.2, 1.2, 3) if rot else np.zeros(3)
    return " ".join(f"{v:.17g}" for v in (*p, *r))


def random_sdf_tree(seed, attach="floating", n_links=7):
    """A random SDF model: every link posed in the model frame, joints posed in
    their child frames, a mix of revolute (limited / unlimited), continuous,
    prismatic and fixed joints, axes in the joint or the model frame."""
    rng = np.random.default_rng(seed)
    L = []
    slots = 0  # contact slots (8 per box, 1 per sphere): the wave kernel holds 32
    for k in range(n_links):
        inert = ""
        if rng.random() < 0.85:
            A = rng.normal(size=(3, 3))
            I = A @ A.T * 0.05 + np.eye(3) * 0.02
            inert = (f"<inertial><pose>{_pose(rng, 0.1)}</pose><mass>{rng.uniform(0.2, 3):.17g}</mass><inertia>"
                     f"<ixx>{I[0,0]:.17g}</ixx><ixy>{I[0,1]:.17g}</ixy><ixz>{I[0,2]:.17g}</ixz>"
                     f"<iyy>{I[1,1]:.17g}</iyy><iyz>{I[1,2]:.17g}</iyz><izz>{I[2,2]:.17g}</izz></inertia></inertial>")
        col = ""
        for _ in range(rng.integers(0, 3)):
            if slots + 8 > 32:
                break
            u = rng.random()
            box, cyl = u < 0.3, 0.3 <= u < 0.55
            slots += 8 if (box or cyl) else 1
            if box:
                geo = f"<box><size>{' '.join(f'{v:.17g}' for v in rng.uniform(0.05, 0.4, 3))}</size></box>"
            elif cyl:
                geo = (f"<cylinder><radius>{rng.uniform(0.02, 0.2):.17g}</radius>"
                       f"<length>{rng.uniform(0.05, 0.5):.17g}</length></cylinder>")
            else:
                geo = f"<sphere><radius>{rng.uniform(0.02, 0.2):.17g}</radius></sphere>"
            col += f"<collision name='c{k}_{len(col)}'><pose>{_pose(rng, 0.2)}</pose><geometry>{geo}</geometry></collision>"
        L.append(f"<link name='l{k}'><pose>{_pose(rng, 1.0)}</pose>{inert}{col}</link>")
    J = []
    types = ["revolute", "revolute", "prismatic", "continuous", "fixed"]
    for k in range(1, n_links):
        parent = int(rng.integers(0, k))
        jt = types[int(rng.integers(0, len(types)))]
        body = f"<joint name='j{k}' type='{jt}'><parent>l{parent}</parent><child>l{k}</child><pose>{_pose(rng, 0.3)}</pose>"
        if jt != "fixed":
            ax = rng.normal(size=3)
            upm = "<use_parent_model_frame>true</use_parent_model_frame>" if rng.random() < 0.4 else ""
            lim = ""
            if jt in ("revolute", "prismatic") and rng.random() < 0.7:
                lo = rng.uniform(-2, -0.1)
                lim = (f"<limit><lower>{lo:.17g}</lower><upper>{rng.uniform(0.1, 2):.17g}</upper>"
                       f"<effort>{rng.uniform(5, 50):.17g}</effort><velocity>{rng.uniform(1, 5):.17g}</velocity></limit>")
            dyn = f"<dynamics><damping>{rng.uniform(0, 0.5):.17g}</damping><friction>{rng.uniform(0, 0.1):.17g}</friction></dynamics>"
            body += f"<axis><xyz>{' '.join(f'{v:.17g}' for v in ax)}</xyz>{upm}{lim}{dyn}</axis>"
        J.append(body + "</joint>")
    if attach == "welded":
        J.append("<joint name='weld' type='fixed'><parent>world</parent><child>l0</child><pose>0.1 0 0 0 0 0.3</pose></joint>")
    elif attach == "hinged":
        J.append("<joint name='hinge' type='revolute'><parent>world</parent><child>l0</child>"
                 "<axis><xyz>0 1 0</xyz><limit><lower>-1</lower><upper>1</upper></limit></axis></joint>")
    return (f"<?xml version='1.0'?><sdf version='1.6'><model name='rand{seed}'><pose>{_pose(rng, 2.0)}</pose>"
            + "".join(L) + "".join(J) + "</model></sdf>")


@pytest.mark.parametrize("attach", ["floating", "welded", "hinged"])
@pytest.mark.parametrize("seed", range(6))
def test_random_sdf_tree_matches_oracle_reader(N, oracle, attach, seed):
    text = random_sdf_tree(seed, attach)
    for pose in (IDENT, (0.3, -1, 2, 0.9238795, 0.3826834, 0, 0)):
        rc, got = _compile(N, text, pose)
        assert rc == 0, got
        cm = oracle.load_urdf(text, pose_xyz=pose[:3], pose_wxyz=pose[3:])
        _compare(got, cm)


def test_sdf_and_urdf_of_one_model_compile_alike(N, oracle, pendulum_file):
    """The pendulum written as SDF (hinged to the world through the model
    frame) compiles to the URDF pendulum's tree: same joint transform, axis,
    inertia, limits."""
    urdf = _compile(N, pendulum_file)[1]
    cm = oracle.load_urdf(pendulum_file)
    M = cm.model
    # re-express the URDF pendulum as SDF: the pivot joint frame = the pole link frame
    E = np.array(M.E[0]).reshape(3, 3)
    r = np.array(M.r[0])
    Rb, pb = cm.base_R, cm.base_p
    Rj, pj = Rb @ E, Rb @ r + pb
    rpy = oracle._mat_to_rpy(Rj)
    I = [M.Ic[0][k] for k in range(6)]
    sdf = f"""<sdf version='1.7'><model name='pendulum'>
      <link name='pole'><pose>{' '.join(f'{v:.17g}' for v in (*pj, *rpy))}</pose>
        <inertial><pose>{' '.join(f'{v:.17g}' for v in M.com[0])} 0 0 0</pose><mass>{M.mass[0]:.17g}</mass>
          <inertia><ixx>{I[0]:.17g}</ixx><iyy>{I[1]:.17g}</iyy><izz>{I[2]:.17g}</izz>
                   <ixy>{I[3]:.17g}</ixy><ixz>{I[4]:.17g}</ixz><iyz>{I[5]:.17g}</iyz></inertia></inertial></link>
      <joint name='{cm.joint_names[0]}' type='revolute'><parent>world</parent><child>pole</child>
        <axis><xyz>{' '.join(f'{v:.17g}' for v in M.axis[0])}</xyz></axis></joint>
    </model></sdf>"""
    rc, got = _compile(N, sdf)
    assert rc == 0, got
    o1, o2 = urdf["out"], got["out"]
    # world pose of the joint frame and every parameter agree
    R2 = got["base"][1:10].reshape(3, 3) @ o2[2:11].reshape(3, 3)
    np.testing.assert_allclose(R2, Rj, atol=1e-12)
    np.testing.assert_allclose(got["base"][1:10].reshape(3, 3) @ o2[11:14] + got["base"][10:13], pj, atol=1e-12)
    np.testing.assert_allclose(o2[14:27], o1[14:27], atol=1e-12)
    assert o2[0] == o1[0]
    _compare(got, oracle.load_urdf(sdf))


@pytest.mark.parametrize("text,needle", [
    ("<sdf version='1.6'><world name='w'/></sdf>", "world"),
    ("<sdf version='1.6'><model name='m'><model name='inner'/></model></sdf>", "nested"),
    ("<sdf version='1.7'><model name='m'><link name='a'><pose relative_to='b'>0 0 0 0 0 0</pose></link></model></sdf>",
     "relative_to"),
    ("<sdf version='1.6'><model name='m'><link name='a'/><link name='b'/>"
     "<joint name='j' type='universal'><parent>a</parent><child>b</child></joint></model></sdf>", "universal"),
    ("<sdf version='1.6'><model name='m'><link name='a'/>"
     "<joint name='j' type='revolute'><parent>a</parent><child>zz</child></joint></model></sdf>", "unknown link"),
])
def test_unsupported_sdf_fails_loudly(N, text, needle):
    rc, msg = _compile(N, text)
    assert rc != 0 and needle in msg, msg


STATIC_TABLE_SDF = """<sdf version='1.7'><model name='table'><static>true</static><pose>0.5 0 0 0 0 0.3</pose>
  <link name='top'><pose>0 0 0.45 0 0 0</pose>
    <collision name='c'><geometry><box><size>1 0.8 0.1</size></box></geometry></collision></link>
  <link name='leg'><pose>0.4 0.3 0.2 0 0 0</pose>
    <collision name='c'><geometry><cylinder><radius>0.03</radius><length>0.4</length></cylinder></geometry></collision>
  </link></model></sdf>"""


def test_static_sdf_model_is_a_welded_collider(N, oracle):
    """<static>true</static>: every root link welded to the world at the model
    frame, no moving joints, the links' shapes on the (fixed) base; the
    oracle's rewrite agrees.  A welded model without joints is a scene
    collider only: mw_sim refuses it."""
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array(IDENT, dtype=np.float64)
        assert N.lib().mw_load_model(h, STATIC_TABLE_SDF.encode(), N.dptr(p), b"") == N.MW_EPARSE
        assert "scene" in N.last_error()
    finally:
        N.lib().mw_destroy(h)
    cm = oracle.load_urdf(STATIC_TABLE_SDF)
    assert not cm.floating and cm.n == 0 and len(cm.base_shapes) == 2
    np.testing.assert_allclose(cm.base_p, [0.5, 0, 0], atol=1e-12)
    # the same shapes through the scene compiler (mw_scene_model_export has no
    # shape export: compare the oracle's lumped shapes with the C++ ones via a
    # fixed-base carrier model that mw_sim accepts)
    carrier = STATIC_TABLE_SDF.replace("<static>true</static>", "").replace(
        "</model>", "<link name='w'/><joint name='hinge' type='revolute'><parent>top</parent><child>w</child>"
        "<axis><xyz>0 0 1</xyz></axis></joint><joint name='weld' type='fixed'><parent>world</parent>"
        "<child>top</child></joint><joint name='weld2' type='fixed'><parent>top</parent><child>leg</child>"
        "</joint></model>")
    rc, got = _compile(N, carrier)
    assert rc == 0, got
    ref = oracle.load_urdf(carrier)
    assert got["base_frame"] == ref.base_link == "top"
    _compare_shapes(got["shapes"][-1], ref.base_shapes, 1e-10)
    # geometry of the welded shapes in the static model's base frame: the
    # table top 0.45 above the model frame, the leg cylinder offset
    tops = sorted(ref.base_shapes, key=lambda s: s[0])
    assert [s[0] for s in tops] == [0, 2]


def test_static_sdf_model_with_joints_fails_loudly(N):
    text = STATIC_TABLE_SDF.replace("</model>", "<joint name='j' type='revolute'><parent>top</parent>"
                                    "<child>leg</child></joint></model>")
    rc, msg = _compile(N, text)
    assert rc != 0 and "static" in msg


BALL_ARM_SDF = """<sdf version='1.7'><model name='arm'>
  <link name='base'><pose>0 0 1 0 0 0</pose></link>
  <joint name='fix' type='fixed'><parent>world</parent><child>base</child></joint>
  <link name='upper'><pose>0.1 0 0.9 0.3 -0.2 0.5</pose>
    <inertial><pose>0 0 -0.2 0 0 0</pose><mass>2</mass>
      <inertia><ixx>0.03</ixx><iyy>0.04</iyy><izz>0.01</izz><ixy>0.001</ixy><ixz>0</ixz><iyz>0</iyz></inertia>
    </inertial>
    <collision name='c'><pose>0 0 -0.2 0 0 0</pose><geometry><sphere><radius>0.05</radius></sphere></geometry></collision>
  </link>
  <joint name='shoulder' type='ball'><pose>0 0 0.05 0 0 0</pose><parent>base</parent><child>upper</child>
    <axis><dynamics><damping>0.2</damping></dynamics></axis></joint>
  <link name='lower'><pose>0.1 0 0.5 0 0.4 0</pose>
    <inertial><pose>0 0 -0.15 0 0 0</pose><mass>1</mass>
      <inertia><ixx>0.01</ixx><iyy>0.01</iyy><izz>0.002</izz><ixy>0</ixy><ixz>0</ixz><iyz>0</iyz></inertia>
    </inertial></link>
  <joint name='elbow' type='revolute'><parent>upper</parent><child>lower</child>
    <axis><xyz>0 1 0</xyz><limit><lower>-2</lower><upper>2</upper></limit></axis></joint>
</model></sdf>"""


def test_ball_joint_compiles_as_three_revolutes(N, oracle):
    """SDF ball joints (Joint.cpp:318-331: 3 dofs): the product lists a
    spherical pair as three bodies at one point (axes x, y, z of the joint
    frame, massless links between) whose coordinates are DART's BallJoint
    ones (jtype bits 4-5 = part 1..3: the rotation vector, the child-frame
    angular velocity; chain_dyn.hpp ball_part), the oracle's independent
    reader the same from three continuous URDF joints -- identical
    multibodies, and the C-ABI reports MW_JOINT_BALL for the three dofs."""
    rc, got = _compile(N, BALL_ARM_SDF)
    assert rc == 0, got
    assert got["names"] == ["shoulder#x", "shoulder#y", "shoulder#z", "elbow"]
    assert got["links"] == ["shoulder#x", "shoulder#y", "upper", "lower"]
    _compare(got, oracle.load_urdf(BALL_ARM_SDF))
    out = got["out"].reshape(-1)[:34 * 4].reshape(4, 34)
    assert out[0, 17] == out[1, 17] == 0.0 and out[2, 17] == 2.0  # masses: the child link on the z part
    np.testing.assert_allclose(out[:3, 14:17], np.eye(3))          # axes x, y, z
    np.testing.assert_allclose(out[1:3, 2:11], [np.eye(3).ravel()] * 2)  # no offset between the parts
    assert list(out[:4, 33]) == [-1, 0, 1, 2]
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array(IDENT, dtype=np.float64)
        N.check(N.lib().mw_load_model(h, BALL_ARM_SDF.encode(), N.dptr(p), b""))
        t = ctypes.c_int32()
        types = []
        for d in range(4):
            N.check(N.lib().mw_joint_type(h, d, ctypes.byref(t)))
            types.append(t.value)
        assert types == [4, 4, 4, 2]  # MW_JOINT_BALL x3, MW_JOINT_REVOLUTE
    finally:
        N.lib().mw_destroy(h)
