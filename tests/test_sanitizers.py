"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the host code
(SURVEY.md §5's sanitizer item; CPU only -- GPU sanitizers are not available
on the MI355X pool).  tests/sanitize/Makefile builds three drivers with
`-fsanitize=address,undefined -fno-sanitize-recover=all`:

  * oracle_san  -- the fp64 oracle (oracle/oracle.c): fixed-base steps with
    joint-limit rows (PGS and DART's two-stage LCP) and floating-base steps
    with ground contacts and warm starts (the exact LCP, the captured
    problem) on the Panda, the quadruped and the humanoid;
  * model_san   -- the C-ABI library's model compiler (csrc/model.cpp,
    csrc/mesh.cpp): every shipped URDF / SDF, the mesh test models (STL,
    OBJ, COLLADA) and malformed inputs that must be rejected;
  * hostdyn_san -- the device dynamics compiled for the host
    (tests/host_dyn/harness.cpp): chain / tree substeps with constraint rows
    and the floating-tree step with contacts.

Any sanitizer report aborts the driver (non-zero exit, the report on
stderr).  The sanitized results must also equal the unsanitized oracle's
(pyoracle, same inputs) -- bit for bit for the oracle, within the host_dyn
tests' fp32 tolerances for the device code -- so the builds check the code
that ships, not a variant of it."""

import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import MODELS, ROOT

SAN_DIR = os.path.join(ROOT, "tests", "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def san(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("san"))
    subprocess.run(["make", "-s", "-C", SAN_DIR, f"OUT={out}", "-j3"], check=True)
    return out


def _run(san, *args):
    r = subprocess.run([os.path.join(san, args[0]), *args[1:]], env=ENV, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, f"{args[0]} exit {r.returncode}:\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def _case_header(kind, steps, pgs, warm, dt):
    return np.array([kind, steps, pgs, warm], np.int32).tobytes() + np.array([dt], np.float64).tobytes()


def test_oracle_fixed_base_under_sanitizers(san, oracle, panda_file, tmp_path):
    """Panda with joints pushed beyond their limits (limit rows), PGS-30 and
    DART's two-stage LCP, 50 steps: bit-identical to the unsanitized oracle."""
    cm = oracle.load_urdf(panda_file)
    n = cm.n
    lo = np.array(cm.model.lower[:n])
    hi = np.array(cm.model.upper[:n])
    rng = np.random.default_rng(3)
    for pgs in (30, oracle.PGS_CONVERGED):
        q = np.where(rng.uniform(size=n) < 0.5, lo - 1e-3, hi + 1e-3)
        qd = rng.uniform(-0.5, 0.5, n)
        mode = np.full(n, oracle.FORCE, np.int32)
        cmd = rng.uniform(-20, 20, n)
        case = tmp_path / f"panda_{pgs}.bin"
        case.write_bytes(_case_header(0, 50, pgs, 0, 1e-3) + bytes(cm.model) + q.tobytes() + qd.tobytes() +
                         mode.tobytes() + cmd.tobytes())
        out = tmp_path / f"panda_{pgs}.out"
        _run(san, "oracle_san", str(case), str(out))
        got = np.frombuffer(out.read_bytes(), np.float64)
        rq, rqd = q.copy(), qd.copy()
        for _ in range(50):
            rq, rqd, *_ = oracle.step(cm, 1e-3, rq, rqd, mode, cmd, pgs)
        assert np.array_equal(got, np.concatenate([rq, rqd])), np.abs(got - np.concatenate([rq, rqd])).max()


@pytest.mark.parametrize("name", ["icub", "quadruped"])
def test_oracle_floating_contacts_under_sanitizers(san, oracle, tmp_path, name):
    """A floating model dropped tilted onto the ground with random joint
    torques, exact two-stage LCP with warm starts, 40 steps: the final state
    and contact forces equal the unsanitized oracle's bit for bit."""
    cm = oracle.load_urdf(os.path.join(MODELS, name + ".urdf"))
    n = cm.n
    rng = np.random.default_rng(5)
    ow = oracle.FloatWorld(cm, ground=True, mu=0.8, pgs_iters=oracle.PGS_CONVERGED, warm_start=True)
    ang = 0.2
    R = np.array([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]])
    z = 0.56 if name == "icub" else 0.40
    ow.set_pose(np.array([0.1, -0.2, z]), R)
    ow.set_twist(rng.uniform(-0.5, 0.5, 3), rng.uniform(-0.3, 0.3, 3))
    q0 = np.zeros(n)
    if name == "icub":
        from mwstep.models import icub_posture
        q0 = np.array(icub_posture(cm.joint_names))
    ow.set_joints(q0 + rng.uniform(-0.3, 0.3, n), rng.uniform(-1, 1, n))
    mode = np.full(n, oracle.FORCE, np.int32)
    cmd = rng.uniform(-10, 10, n)
    case = tmp_path / f"{name}.bin"
    case.write_bytes(_case_header(1, 40, oracle.PGS_CONVERGED, 1, 1e-3) + bytes(ow.m) + bytes(ow.s) +
                     mode.tobytes() + cmd.tobytes())
    out = tmp_path / f"{name}.out"
    _run(san, "oracle_san", str(case), str(out))
    raw = out.read_bytes()
    ssz = ctypes.sizeof(oracle.OrFloatState)
    st = oracle.OrFloatState.from_buffer_copy(raw[:ssz])
    nc = int(np.frombuffer(raw[ssz:ssz + 4], np.int32)[0])
    forces = np.frombuffer(raw[ssz + 4:], np.float64).reshape(-1, 3)
    for _ in range(40):
        ow.step(mode, cmd)
    assert nc == len(ow.contacts) and nc > 0
    assert np.array_equal(np.array(st.q[:n]), ow.q) and np.array_equal(np.array(st.qd[:n]), ow.qd)
    assert np.array_equal(np.array(st.p[:]), ow.p) and np.array_equal(np.array(st.V[:]), ow.V)
    assert np.array_equal(forces, np.array([f for _, f, _, _ in ow.contacts]))


def test_model_compiler_under_sanitizers(san, tmp_path):
    """Every shipped model, the mesh test models and malformed documents
    through the sanitized model compiler; the accepted ones compile to the
    same joints as the library does (mw_joint_name), the malformed ones are
    rejected with a message."""
    from mesh_models import rock_vertices, write_obj
    files = sorted(os.path.join(MODELS, f) for f in os.listdir(MODELS) if f.endswith((".urdf", ".sdf")))
    rock = str(tmp_path / "rock.obj")
    write_obj(rock, *rock_vertices(6))
    mesh_urdf = tmp_path / "mesh.urdf"
    mesh_urdf.write_text('<robot name="m"><link name="b"><inertial><mass value="1"/><inertia ixx="0.01" '
                         'iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial><collision><geometry>'
                         f'<mesh filename="{rock}" scale="1 2 1"/></geometry></collision></link></robot>')
    bad = {"truncated.urdf": '<robot name="x"><link name="a">',
           "two_roots.urdf": '<robot name="x"><link name="a"/><link name="b"/></robot>',
           "cycle.urdf": '<robot name="x"><link name="a"/><link name="b"/>'
                         '<joint name="j" type="revolute"><parent link="a"/><child link="b"/></joint>'
                         '<joint name="k" type="revolute"><parent link="b"/><child link="a"/></joint></robot>',
           "zero_axis.urdf": '<robot name="x"><link name="a"><inertial><mass value="1"/></inertial></link>'
                             '<link name="b"><inertial><mass value="1"/></inertial></link><joint name="j" '
                             'type="revolute"><parent link="a"/><child link="b"/><axis xyz="0 0 0"/>'
                             '</joint></robot>',
           "missing_mesh.urdf": '<robot name="x"><link name="a"><inertial><mass value="1"/></inertial>'
                                '<collision><geometry><mesh filename="/nonexistent/m.stl"/></geometry>'
                                '</collision></link></robot>'}
    for k, v in bad.items():
        (tmp_path / k).write_text(v)
    args = files + [str(mesh_urdf)] + [str(tmp_path / k) for k in bad]
    lines = _run(san, "model_san", *args).strip().split("\n")
    assert len(lines) == len(args)
    for path, line in zip(args, lines):
        if os.path.basename(path) in bad:
            assert line.startswith("error "), (path, line)
            continue
        if path.endswith("ground_plane.sdf"):
            continue  # a static model: the simulator places it, the compiler rejects an empty tree
        assert line.startswith("ok "), (path, line)
        assert line.split()[5:] == _library_joint_names(path), (path, line)


def _library_joint_names(path):
    """The joints libmwstep.so compiles the model to (host side, no GPU)."""
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(np.array([0, 0, 0, 1, 0, 0, 0.0])), b""))
        n = ctypes.c_int()
        N.check(N.lib().mw_dofs(h, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(256)
        names = []
        for d in range(n.value):
            N.check(N.lib().mw_joint_name(h, d, buf, 256))
            names.append(buf.value.decode())
        return names
    finally:
        N.lib().mw_destroy(h)


def _params(path):
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array([0, 0, 0, 1, 0, 0, 0.0])
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(p), b""))
        N.check(N.lib().mw_set_ground_plane(h, 1, 0.8))
        P = ctypes.create_string_buffer(1 << 16)
        N.check(N.lib().mw_device_params(h, P, len(P)))
        F = ctypes.create_string_buffer(1 << 16)
        floating = ctypes.c_int()
        N.check(N.lib().mw_is_floating(h, ctypes.byref(floating)))
        if floating.value:
            N.check(N.lib().mw_device_float_params(h, F, len(F)))
        return P, F
    finally:
        N.lib().mw_destroy(h)


def test_device_dynamics_on_host_under_sanitizers(san, oracle, panda_file, cartpole_file, tmp_path):
    """The device substep (chain_dyn.hpp) of the cartpole (limit row) and the
    Panda tree (limit rows, PGS-30) and the floating-tree step
    (float_tree.hpp) of the quadruped with foot contacts, under the
    sanitizers, against the fp64 oracle (the tolerances of
    tests/test_host_dyn.py)."""
    import ctypes as C
    from test_float_tree_oracle import STAND
    hd_sizes = {}
    # the exact parameter-block sizes come from the unsanitized harness build
    # the CPU suite uses (tests/test_host_dyn.py); the library copies at most
    # the caller's buffer, so ask it for the block of each model at that size
    lib = os.path.join(str(tmp_path), "libhd.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-DMW_FAST_MATH", "-I",
                    os.path.join(ROOT, "gym-ignition_amd", "csrc"), os.path.join(ROOT, "tests", "host_dyn",
                                                                                 "harness.cpp"), "-o", lib],
                   check=True)
    L = C.CDLL(lib)
    hd_sizes["chain"], hd_sizes["float"] = L.hd_sizeof_chain(), L.hd_sizeof_float()
    rng = np.random.default_rng(7)
    for path, n_steps in ((cartpole_file, 1), (panda_file, 1)):
        P, _ = _params(path)
        pfile = tmp_path / "P.bin"
        pfile.write_bytes(P.raw[:hd_sizes["chain"]])
        cm = oracle.load_urdf(path)
        n = cm.n
        lo = np.clip(np.array(cm.model.lower[:n]), -5, 5)
        hi = np.clip(np.array(cm.model.upper[:n]), -5, 5)
        worst = 0.0
        for k in range(10):
            q = rng.uniform(lo, hi)
            at = rng.uniform(size=n) < 0.5
            q[at] = np.where(rng.uniform(size=n) < 0.5, lo - 1e-3, hi + 1e-3)[at]
            q = q.astype(np.float32)
            qd = rng.uniform(-0.5, 0.5, n).astype(np.float32)
            tau = rng.uniform(-10, 10, n).astype(np.float32)
            case = tmp_path / "c.bin"
            case.write_bytes(np.array([n, 30, 1, 0], np.int32).tobytes() + np.float32(1e-3).tobytes() +
                             q.tobytes() + qd.tobytes() + tau.tobytes() + np.zeros(n, np.uint8).tobytes() +
                             np.zeros(n, np.float32).tobytes())
            out = tmp_path / "c.out"
            _run(san, "hostdyn_san", "chain", str(pfile), str(case), str(out))
            got = np.frombuffer(out.read_bytes(), np.float32).reshape(3, n).astype(float)
            ref = oracle.step(cm, 1e-3, q.astype(float), qd.astype(float), [oracle.FORCE] * n,
                              tau.astype(float), 30)
            worst = max(worst, float(np.abs(got[1] - ref[1]).max()))
        assert worst <= 2e-4, (path, worst)
    # floating tree with foot contacts
    qpath = os.path.join(MODELS, "quadruped.urdf")
    P, F = _params(qpath)
    pfile, ffile = tmp_path / "P.bin", tmp_path / "F.bin"
    pfile.write_bytes(P.raw[:hd_sizes["chain"]])
    ffile.write_bytes(F.raw[:hd_sizes["float"]])
    cm = oracle.load_urdf(qpath)
    n = cm.n
    n_contact, worst = 0, 0.0
    for k in range(10):
        q = (STAND + rng.uniform(-0.2, 0.2, n)).astype(np.float32)
        base = np.array([0.0, 0.0, 0.44 + rng.uniform(-0.01, 0.01), 1, 0, 0, 0, *rng.uniform(-0.2, 0.2, 6)],
                        np.float32)
        qd = rng.uniform(-0.3, 0.3, n).astype(np.float32)
        tau = rng.uniform(-5, 5, n).astype(np.float32)
        case = tmp_path / "f.bin"
        case.write_bytes(np.array([n, 50, 1], np.int32).tobytes() + np.float32(1e-3).tobytes() + base.tobytes() +
                         q.tobytes() + qd.tobytes() + tau.tobytes())
        out = tmp_path / "f.out"
        _run(san, "hostdyn_san", "float", str(pfile), str(ffile), str(case), str(out))
        raw = np.frombuffer(out.read_bytes()[:4 * (13 + 2 * n)], np.float32).astype(float)
        ow = oracle.FloatWorld(cm, ground=True, mu=0.8, pgs_iters=50)
        ow.set_pose(base[:3].astype(float), np.eye(3))
        ow.set_twist(base[7:10].astype(float), base[10:13].astype(float))
        ow.set_joints(q.astype(float), qd.astype(float))
        ow.step(np.full(n, oracle.FORCE, np.int32), tau.astype(float))
        n_contact += len(ow.contacts) > 0
        worst = max(worst, float(np.abs(raw[13 + n:] - ow.qd).max()))
    assert n_contact >= 5 and worst <= 1e-3, (n_contact, worst)
