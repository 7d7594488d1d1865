"""BASELINE config 5's model (CPU): the shipped iCub-class stand-in
(gym-ignition_amd/models/icub.urdf, make_icub.py) carries what the
reference's iCub wrapper pins (python/gym_ignition_environments/models/
icub.py): DOFS = NUM_JOINTS = 32 and NUM_LINKS = 39 (:15-17), the 32 joint
names of initial_positions (:19-40), a posture inside the joint limits, and
the insertion pose (0, 0, 0.572) wxyz (0, 0, 0, 1) (:86) puts the soles
just above the ground, from where the fp64 oracle (DART's two-stage LCP)
lands it on its feet and holds it standing under the JointController PID of
the posture."""

import ctypes
import re

import numpy as np
import pytest

G = 9.8


@pytest.fixture(scope="module")
def icub_file():
    from mwstep import get_model_file
    return get_model_file("icub")


def _library_joints(path):
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(np.array([0, 0, 0.572, 0, 0, 0, 1.0])), b""))
        n = ctypes.c_int()
        N.check(N.lib().mw_dofs(h, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(64)
        names = []
        for d in range(n.value):
            N.check(N.lib().mw_joint_name(h, d, buf, 64))
            names.append(buf.value.decode())
        fl = ctypes.c_int()
        N.check(N.lib().mw_is_floating(h, ctypes.byref(fl)))
        return names, bool(fl.value)
    finally:
        N.lib().mw_destroy(h)


def test_counts_and_names_match_the_reference_wrapper(icub_file):
    from gym_ignition_environments.models.icub import ICubGazebo
    text = open(icub_file).read()
    assert len(re.findall(r"<link ", text)) == ICubGazebo.NUM_LINKS == 39
    assert text.count('type="revolute"') == ICubGazebo.NUM_JOINTS == ICubGazebo.DOFS == 32
    # the six F/T-sensor frames: fixed joints that sdformat is told to keep
    fixed = re.findall(r'<joint name="([a-z_]+)" type="fixed">', text)
    kept = re.findall(r'<gazebo reference="([a-z_]+)">\s*<preserveFixedJoint>true', text)
    assert sorted(fixed) == sorted(kept) and len(fixed) == 6
    names, floating = _library_joints(icub_file)
    assert floating and len(names) == 32
    assert set(names) == set(ICubGazebo.initial_positions)


def test_posture_is_inside_the_limits(oracle, icub_file):
    from mwstep.models import icub_posture
    cm = oracle.load_urdf(icub_file)
    q0 = np.array(icub_posture(cm.joint_names))
    lo = np.array(cm.model.lower[:cm.n])
    hi = np.array(cm.model.upper[:cm.n])
    assert (q0 > lo).all() and (q0 < hi).all()


def test_wrapper_pose_lands_on_the_feet_and_stands(oracle, icub_file):
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    cm = oracle.load_urdf(icub_file, pose_xyz=ICUB_POSE[:3], pose_wxyz=ICUB_POSE[3:])
    n = cm.n
    q0 = np.array(icub_posture(cm.joint_names))
    ow = oracle.FloatWorld(cm, pgs_iters=oracle.PGS_CONVERGED)
    ow.set_joints(q0, np.zeros(n))
    # the wrapper's orientation: a half turn about z (the robot faces world +x)
    assert np.allclose(ow.R, np.diag([-1.0, -1.0, 1.0]))
    og = [oracle.pid_gains(p, 0.0, d, cmdmax=80.0, cmdmin=-80.0) for p, d in icub_pid_gains(cm.joint_names)]
    st = [oracle.OrPidState() for _ in range(n)]
    mode = np.full(n, oracle.FORCE, np.int32)
    first_contact = None
    for k in range(1000):
        tau = np.array([oracle.pid_update(og[d], st[d], ow.q[d] - q0[d], 1e-3) for d in range(n)])
        ow.step(mode, tau)
        if first_contact is None and ow.contacts:
            first_contact = k
    mass = cm.free.mass + sum(cm.model.mass[i] for i in range(n))
    fz = sum(f[2] for _, f, _, _ in ow.contacts)
    assert mass == pytest.approx(30.7)
    # free fall of 4.3 mm takes ~30 ms: the soles start just above the ground
    assert 15 <= first_contact <= 45
    assert len(ow.contacts) == 8 and fz == pytest.approx(mass * G, abs=3.0)
    assert ow.p[2] == pytest.approx(0.565, abs=0.005) and np.abs(ow.p[:2]).max() < 0.01
    assert np.abs(ow.q - q0).max() < 0.06
