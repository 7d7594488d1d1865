"""The C-ABI library without a GPU: it loads, exports every symbol that
include/mwstep.h declares, compiles models (host side) exactly like the
oracle's independent URDF reader, and validates its inputs."""

import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mwstep.h")
SCENE_HEADER = os.path.join(ROOT, "include", "mwscene.h")
TEST_HEADER = os.path.join(ROOT, "include", "mwstep_testhooks.h")


def _declared_symbols(header=HEADER):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mw_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def N():
    from mwstep import native
    native.lib()
    return native


def test_every_declared_symbol_is_exported(N):
    L = ctypes.CDLL(N.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    bound = {name for name, _, _ in N.SIGNATURES}
    assert set(declared) == bound, set(declared) ^ bound


def test_every_scene_symbol_is_exported(N):
    """include/mwscene.h (multi-model worlds): every declared entry point is
    in the library and bound by the ctypes layer."""
    L = ctypes.CDLL(N.LIB_PATH)
    declared = _declared_symbols(SCENE_HEADER)
    assert len(declared) >= 35
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    bound = {name for name, _, _ in N.SCENE_SIGNATURES}
    assert set(declared) == bound, set(declared) ^ bound


def test_every_test_hook_is_exported(N):
    """include/mwstep_testhooks.h (test-only entry points, kept out of the
    ScenarI/O header): exported and bound by TEST_SIGNATURES."""
    L = ctypes.CDLL(N.LIB_PATH)
    declared = _declared_symbols(TEST_HEADER)
    assert declared == ["mw_debug_hull", "mw_debug_lcp_solve", "mw_debug_scene_big_ws"]
    assert all(hasattr(L, s) for s in declared)
    assert set(declared) == {name for name, _, _ in N.TEST_SIGNATURES}
    assert not set(declared) & set(_declared_symbols())


def test_scene_create_validates_arguments(N):
    h = ctypes.c_void_p()
    for step, rtf, spr, nw in [(0.0, 1.0, 1, 1), (1e-3, 0.0, 1, 1), (1e-3, 1.0, 0, 1), (1e-3, 1.0, 1, 0)]:
        cfg = N.MwConfig(step, rtf, spr, nw, 0, 0)
        assert N.lib().mw_scene_create(ctypes.byref(cfg), ctypes.byref(h)) == N.MW_EINVAL
        assert N.last_error()


def test_library_is_gfx950(N):
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _create(N, n_worlds=4, step=1e-3, rtf=1.0, steps=1):
    cfg = N.MwConfig(step, rtf, steps, n_worlds, 0, 0)
    h = ctypes.c_void_p()
    rc = N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h))
    return rc, h


@pytest.mark.parametrize("step,rtf,steps", [(0.0, 1.0, 1), (0.001, 0.0, 1), (0.001, -1.0, 1),
                                            (0.001, 1.0, 0)])
def test_create_validates_like_gazebo_simulator(N, step, rtf, steps):
    # tests/test_scenario/test_gazebo_simulator.py:17-51
    rc, h = _create(N, step=step, rtf=rtf, steps=steps)
    assert rc == N.MW_EINVAL and not h.value
    assert N.last_error()


def _export(N, path, pose=(0, 0, 0, 1, 0, 0, 0)):
    rc, h = _create(N)
    assert rc == 0
    try:
        p = np.array(pose, dtype=np.float64)
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(p), b""))
        n = ctypes.c_int32()
        N.check(N.lib().mw_dofs(h, ctypes.byref(n)))
        out = np.zeros(34 * n.value + 3)
        N.check(N.lib().mw_model_export(h, N.dptr(out), len(out)))
        names = []
        buf = ctypes.create_string_buffer(64)
        for d in range(n.value):
            N.check(N.lib().mw_joint_name(h, d, buf, 64))
            names.append(buf.value.decode())
        N.lib().mw_base_frame(h, buf, 64)
        return n.value, out, names, buf.value.decode()
    finally:
        N.lib().mw_destroy(h)


@pytest.mark.parametrize("model", ["cartpole", "pendulum", "panda"])
@pytest.mark.parametrize("pose", [(0, 0, 0, 1, 0, 0, 0), (0.3, -1, 2, 0.9238795, 0.3826834, 0, 0)])
def test_model_compiler_matches_oracle_reader(N, oracle, cartpole_file, pendulum_file, panda_file, model, pose):
    path = {"cartpole": cartpole_file, "pendulum": pendulum_file, "panda": panda_file}[model]
    n, out, names, base = _export(N, path, pose)
    cm = oracle.load_urdf(path, pose_xyz=pose[:3], pose_wxyz=pose[3:])
    assert names == cm.joint_names and n == cm.n
    assert base == cm.base_link
    M = cm.model
    big = lambda v: np.where(v > 1e299, np.inf, np.where(v < -1e299, -np.inf, v))
    for i in range(n):
        b = out[34 * i: 34 * (i + 1)]
        assert b[0] == M.jtype[i] and b[1] == M.limited[i]
        np.testing.assert_allclose(b[2:11], list(M.E[i]), atol=1e-12)
        np.testing.assert_allclose(b[11:14], list(M.r[i]), atol=1e-12)
        np.testing.assert_allclose(b[14:17], list(M.axis[i]), atol=1e-12)
        assert b[17] == pytest.approx(M.mass[i])
        np.testing.assert_allclose(b[18:21], list(M.com[i]), atol=1e-12)
        np.testing.assert_allclose(b[21:27], list(M.Ic[i]), atol=1e-12)
        np.testing.assert_allclose(big(b[27:33]), [M.damping[i], M.friction[i], M.lower[i], M.upper[i],
                                                   M.effort[i], M.vel_limit[i]])
        assert b[33] == M.parent[i]
    np.testing.assert_allclose(out[34 * n:], list(M.gravity_base), atol=1e-12)


def test_fixed_joint_lumping(N, oracle):
    urdf = """<robot name="r"><link name="world"/>
      <joint name="w" type="fixed"><parent link="world"/><child link="a"/></joint>
      <link name="a"><inertial><mass value="1"/><inertia ixx="1" iyy="1" izz="1"/></inertial></link>
      <joint name="j1" type="revolute"><parent link="a"/><child link="b"/><axis xyz="0 0 1"/>
        <origin xyz="0 0 1" rpy="0.1 0.2 0.3"/><limit lower="-1" upper="1" effort="10" velocity="3"/></joint>
      <link name="b"><inertial><origin xyz="0.1 0 0" rpy="0 0.5 0"/><mass value="2"/>
        <inertia ixx="0.1" iyy="0.2" izz="0.3" ixy="0.01"/></inertial></link>
      <joint name="fx" type="fixed"><parent link="b"/><child link="c"/><origin xyz="0 0.5 0" rpy="0.3 0 0"/></joint>
      <link name="c"><inertial><mass value="0.5"/><inertia ixx="0.01" iyy="0.01" izz="0.01"/></inertial></link>
      <joint name="j2" type="prismatic"><parent link="c"/><child link="d"/><axis xyz="1 1 0"/>
        <origin xyz="0.2 0 0"/><limit lower="-0.5" upper="0.5" effort="100" velocity="1"/>
        <dynamics damping="0.3" friction="0.05"/></joint>
      <link name="d"><inertial><mass value="0.3"/><inertia ixx="0.001" iyy="0.001" izz="0.001"/></inertial></link>
    </robot>"""
    n, out, names, base = _export(N, urdf)
    cm = oracle.load_urdf(urdf)
    assert names == ["j1", "j2"] == cm.joint_names and base == "a"
    np.testing.assert_allclose(out[34 + 2:34 + 11], list(cm.model.E[1]), atol=1e-12)
    np.testing.assert_allclose(out[34 + 11:34 + 14], list(cm.model.r[1]), atol=1e-12)
    np.testing.assert_allclose(out[21:27], list(cm.model.Ic[0]), atol=1e-12)
    np.testing.assert_allclose(out[18:21], list(cm.model.com[0]), atol=1e-12)
    assert out[17] == pytest.approx(2.5)


@pytest.mark.parametrize("bad, why", [
    # a floating chain of 13 joints: deeper than the wave kernel's stack
    ("<robot name='x'>" + "".join(
        f"<link name='l{i}'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        for i in range(14)) + "".join(
        f"<joint name='j{i}' type='revolute'><parent link='l{i}'/><child link='l{i + 1}'/></joint>"
        for i in range(13)) + "</robot>",
     "deeper than 12"),
    ("<robot name='x'><link name='a'/></robot>", "has no mass"),
    ("<robot name='x'><link name='world'/>", "XML"),
    ("<sdf><model name='m'/></sdf>", "no links"),
    ("<mjcf/>", "URDF"),
    # a welded chain of 13 joints: the fixed-base tree runs on the wave kernel, whose stack is 12 deep
    ("<robot name='x'><link name='world'/><joint name='w' type='fixed'><parent link='world'/><child link='l0'/>"
     "</joint>" + "".join(
        f"<link name='l{i}'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        for i in range(14)) + "".join(
        f"<joint name='j{i}' type='revolute'><parent link='l{i}'/><child link='l{i + 1}'/></joint>"
        for i in range(13)) + "</robot>",
     "deeper than 12"),
])
def test_unsupported_models_fail_loudly(N, bad, why):
    rc, h = _create(N)
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)
        rc = N.lib().mw_load_model(h, bad.encode(), N.dptr(p), b"")
        assert rc == N.MW_EPARSE
        assert why.lower() in N.last_error().lower()
    finally:
        N.lib().mw_destroy(h)


def test_generic_fixed_base_trees_take_the_wave_kernel(N):
    """A branched fixed-base tree outside the compiled chain topologies is
    accepted (no longer refused) and routed to the
    world-per-wavefront kernel with a welded base; so is a hinge to the world."""
    trees = [
        "<robot name='x'><link name='world'/><link name='a'/><joint name='w' type='fixed'>"
        "<parent link='world'/><child link='a'/></joint>"
        "<link name='b'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        "<link name='c'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        "<joint name='j1' type='revolute'><parent link='a'/><child link='b'/></joint>"
        "<joint name='j2' type='revolute'><parent link='a'/><child link='c'/></joint></robot>",
        "<robot name='y'><link name='world'/>"
        "<link name='b'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        "<link name='c'><inertial><mass value='1'/><inertia ixx='1' iyy='1' izz='1'/></inertial></link>"
        "<joint name='j1' type='revolute'><parent link='world'/><child link='b'/></joint>"
        "<joint name='j2' type='prismatic'><parent link='world'/><child link='c'/></joint></robot>",
    ]
    for text in trees:
        rc, h = _create(N)
        try:
            p = np.array([0, 0, 1, 1, 0, 0, 0], dtype=np.float64)
            N.check(N.lib().mw_load_model(h, text.encode(), N.dptr(p), b""))
            k, f = ctypes.c_int32(), ctypes.c_int32()
            N.check(N.lib().mw_float_kernel(h, ctypes.byref(k)))
            N.check(N.lib().mw_is_floating(h, ctypes.byref(f)))
            assert k.value == 2 and f.value == 0
        finally:
            N.lib().mw_destroy(h)


def test_initialize_without_model_or_gpu_reports_error(N, cartpole_file):
    rc, h = _create(N)
    try:
        assert N.lib().mw_initialize(h) == N.MW_ESTATE
        p = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)
        N.check(N.lib().mw_load_model(h, cartpole_file.encode(), N.dptr(p), b""))
        rc = N.lib().mw_run(h, 0)
        assert rc == N.MW_ESTATE  # not initialized: run refuses, like GazeboSimulator::run
    finally:
        N.lib().mw_destroy(h)


def test_joint_params_before_first_run(N, pendulum_file):
    rc, h = _create(N)
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)
        N.check(N.lib().mw_load_model(h, pendulum_file.encode(), N.dptr(p), b""))
        N.check(N.lib().mw_set_joint_param(h, 0, N.PARAM_COULOMB_FRICTION, 0.01))
        v = ctypes.c_double()
        N.check(N.lib().mw_joint_param(h, 0, N.PARAM_COULOMB_FRICTION, ctypes.byref(v)))
        assert v.value == 0.01
        assert N.lib().mw_set_joint_param(h, 3, N.PARAM_COULOMB_FRICTION, 0.01) == N.MW_EINVAL
    finally:
        N.lib().mw_destroy(h)


def test_pid_and_controller_period_semantics(N, panda_file):
    """Joint::setPID / pid (Joint.cpp:63, :479-525), Model::setControllerPeriod
    (Model.cpp:589-602) -- host logic, no GPU needed."""
    rc, h = _create(N)
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0], dtype=np.float64)
        N.check(N.lib().mw_load_model(h, panda_file.encode(), N.dptr(p), b""))
        g = np.zeros(8)
        N.check(N.lib().mw_joint_pid(h, 0, N.dptr(g)))
        np.testing.assert_array_equal(g, [1.0, 0.1, 0.01, 0.0, -1.0, 0.0, 0.0, -1.0])   # DefaultPID
        big = float(np.finfo(np.float64).max)
        # open output limits are less limiting than +-effort (87 Nm): replaced
        N.check(N.lib().mw_set_joint_pid(h, 0, N.dptr(np.array([50, 0, 20, -big, big, 0, -big, big.real]))))
        N.check(N.lib().mw_joint_pid(h, 0, N.dptr(g)))
        np.testing.assert_array_equal(g, [50, 0, 20, -87, 87, 0, -big, big])
        # tighter limits are kept
        N.check(N.lib().mw_set_joint_pid(h, 0, N.dptr(np.array([5, 1, 2, -10, 20, 0.5, -1, 1.0]))))
        N.check(N.lib().mw_joint_pid(h, 0, N.dptr(g)))
        np.testing.assert_array_equal(g, [5, 1, 2, -10, 20, 0.5, -1, 1])
        assert N.lib().mw_set_joint_pid(h, 9, N.dptr(g)) == N.MW_EINVAL
        t = ctypes.c_double()
        N.check(N.lib().mw_controller_period(h, ctypes.byref(t)))
        assert t.value == pytest.approx(9.223372036854776e9)        # max duration
        assert N.lib().mw_set_controller_period(h, 0.0) == N.MW_EINVAL
        assert "greater than zero" in N.last_error()
        N.check(N.lib().mw_set_controller_period(h, 1e-3))
        N.check(N.lib().mw_controller_period(h, ctypes.byref(t)))
        assert t.value == 1e-3
    finally:
        N.lib().mw_destroy(h)


CUBE = """<robot name="cube_robot"><link name="cube"><inertial><origin rpy="0 0 0" xyz="0 0 0"/>
  <mass value="5.0"/><inertia ixx="0.0333333" ixy="0" ixz="0" iyy="0.0333333" iyz="0" izz="0.0333333"/></inertial>
  <collision><geometry><box size="0.2 0.1 0.2"/></geometry><origin rpy="0 0 0" xyz="0 -0.05 0"/></collision>
  <collision><geometry><box size="0.2 0.1 0.2"/></geometry><origin rpy="0 0 0" xyz="0 0.05 0"/></collision>
</link></robot>"""


def test_floating_body_model(N, oracle):
    """A floating single body (the reference's double-collision test cube,
    tests/test_scenario/test_contacts.py:22-54) compiles with its two box
    shapes; base / contact calls need an initialised simulator."""
    rc, h = _create(N)
    try:
        p = np.array([0, 0, 0.15, 1, 0, 0, 0], dtype=np.float64)
        N.check(N.lib().mw_load_model(h, CUBE.encode(), N.dptr(p), b"cube"))
        f = ctypes.c_int32()
        N.check(N.lib().mw_is_floating(h, ctypes.byref(f)))
        assert f.value == 1
        n = ctypes.c_int32()
        N.check(N.lib().mw_dofs(h, ctypes.byref(n)))
        assert n.value == 0
        out = np.zeros(7)
        assert N.lib().mw_get_base_pose(h, 0, 1, N.dptr(out)) == N.MW_ESTATE
        N.check(N.lib().mw_set_ground_plane(h, 1, 1.0))
        assert N.lib().mw_set_ground_plane(h, 1, -1.0) == N.MW_EINVAL
        N.check(N.lib().mw_enable_contacts(h, 1))
        N.check(N.lib().mw_contacts_enabled(h, ctypes.byref(f)))
        assert f.value == 1
    finally:
        N.lib().mw_destroy(h)
    cm = oracle.load_urdf(CUBE, pose_xyz=(0, 0, 0.15))
    assert cm.floating and cm.n == 0 and cm.free.n_shapes == 2
    np.testing.assert_allclose(list(cm.free.shape_p[1]), [0, 0.05, 0])
    np.testing.assert_allclose(list(cm.free.shape_size[0]), [0.1, 0.05, 0.1])
