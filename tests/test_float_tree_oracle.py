"""Pin the fp64 floating-tree oracle (or_float_step) before trusting it (CPU).

The dense restatement (CRBA mass matrix + RNEA bias with a free root, dense
contact / joint rows) is checked against the parts already pinned:

  * its joint block and joint bias equal the fixed-base CRBA / RNEA of the
    same tree (or_crba / or_rnea, pinned by the reference's pendulum and
    cartpole KATs), and its base block is the composite rigid-body inertia;
  * heavy-base reduction: a base of 1e9 kg in zero gravity reproduces the
    fixed-base engine step (or_step) of the same tree, limits and all;
  * free fall: with no contacts every body falls with g and the joints see
    no gravity (the relative motion is the zero-gravity fixed-base motion);
  * momentum conservation under internal joint torques (zero gravity, no
    contacts): the world spatial momentum drifts only at first order in dt
    (semi-implicit Euler), i.e. 10x less for a 10x smaller step;
  * the reference's contact KAT transposed to an articulated body
    (tests/test_scenario/test_contacts.py:57-122: the vertical contact forces
    sum to the weight within 0.1 N): the quadruped standing on its four feet
    under a joint PD hold carries its 16 kg on exactly its feet.
"""

import numpy as np
import pytest

G = 9.8


@pytest.fixture(scope="module")
def quad_file():
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "gym-ignition_amd", "models", "quadruped.urdf")


STAND = np.array([0.6, -1.2] * 4)


def chain_urdf(n=2, floating=True, cylinder_tip=False, mesh_tip=None):
    """A floating box base with an n-link revolute chain (links: 0.3 m rods,
    alternating y / x axes), a sphere (or a tilted cylinder, or the mesh file
    mesh_tip, tilted) at the tip."""
    links = ['<link name="base"><inertial><mass value="3.0"/>'
             '<inertia ixx="0.02" iyy="0.03" izz="0.04" ixy="0.001" ixz="0" iyz="0"/></inertial>'
             '<collision><geometry><box size="0.3 0.2 0.1"/></geometry></collision></link>']
    if not floating:
        links.insert(0, '<link name="world"/><joint name="fix" type="fixed"><parent link="world"/>'
                        '<child link="base"/></joint>')
    parent = "base"
    for i in range(n):
        axis = "0 1 0" if i % 2 == 0 else "1 0 0"
        z = "-0.05" if i == 0 else "-0.3"
        geo = ('<origin xyz="0 0 -0.3" rpy="0.4 1.1 0"/><geometry><cylinder radius="0.04" length="0.12"/>'
               '</geometry>' if cylinder_tip else
               f'<origin xyz="0 0 -0.3" rpy="0.3 -0.5 0.2"/><geometry><mesh filename="{mesh_tip}" scale="0.5 0.5 0.5"/>'
               '</geometry>' if mesh_tip else
               '<origin xyz="0 0 -0.3"/><geometry><sphere radius="0.04"/></geometry>')
        tip = f'<collision>{geo}</collision>' if i == n - 1 else ""
        links.append(f'<joint name="j{i}" type="revolute"><parent link="{parent}"/><child link="l{i}"/>'
                     f'<origin xyz="0.1 0 {z}" rpy="0 0 0"/><axis xyz="{axis}"/>'
                     f'<limit lower="-2.0" upper="2.0" effort="50" velocity="30"/></joint>'
                     f'<link name="l{i}"><inertial><origin xyz="0 0.01 -0.15"/><mass value="{0.8 - 0.2 * i}"/>'
                     f'<inertia ixx="0.006" iyy="0.007" izz="0.001" ixy="0.0002" ixz="0" iyz="0"/></inertial>'
                     f'{tip}</link>')
        parent = f"l{i}"
    return '<robot name="fchain">' + "".join(links) + "</robot>"


def momentum(fw):
    M, _ = fw.dynamics()
    nu = np.concatenate([fw.V, fw.qd])
    hb = M[:6] @ nu
    L = fw.R @ hb[3:]
    return np.concatenate([fw.R @ hb[:3] + np.cross(fw.p, L), L])


def test_dense_blocks_match_fixed_base(oracle, quad_file):
    cm = oracle.load_urdf(quad_file, pose_xyz=(0.1, -0.2, 0.5), pose_wxyz=(0.9, 0.1, -0.2, 0.3))
    fw = oracle.FloatWorld(cm, ground=False)
    rng = np.random.default_rng(1)
    q = rng.uniform(-1, 1, 8)
    fw.set_joints(q, np.zeros(8))
    M, h = fw.dynamics()
    assert np.abs(M - M.T).max() < 1e-12
    assert np.linalg.eigvalsh(M).min() > 0
    assert M[3, 3] == pytest.approx(16.0) and M[4, 4] == pytest.approx(16.0)
    # fixed-base routines with gravity expressed in the base frame
    cm.model.gravity_base[:] = list(fw.R.T @ np.array([0, 0, -G]))
    np.testing.assert_allclose(M[6:, 6:], oracle.crba(cm, q), atol=1e-12)
    np.testing.assert_allclose(h[6:], oracle.rnea(cm, q, np.zeros(8), np.zeros(8)), atol=1e-12)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_heavy_base_reduces_to_fixed_base_step(oracle, n):
    text = chain_urdf(n)
    cmf = oracle.load_urdf(text, gravity=(0, 0, 0))
    cmf.free.mass = 1e9
    for k in range(3):
        cmf.free.Ic[k] = 1e9
    fw = oracle.FloatWorld(cmf, ground=False, pgs_iters=50)
    cmx = oracle.load_urdf(chain_urdf(n, floating=False), gravity=(0, 0, 0))
    rng = np.random.default_rng(n)
    q = rng.uniform(-1.9, 1.9, n)
    q[0] = 2.05  # beyond the upper limit: a limit row is active
    qd = rng.uniform(-2, 2, n)
    tau = rng.uniform(-5, 5, n)
    fw.set_joints(q, qd)
    mode = np.full(n, oracle.FORCE, np.int32)
    for _ in range(50):
        fw.step(mode, tau)
    qx, qdx = q.copy(), qd.copy()
    for _ in range(50):
        qx, qdx, _, _, _ = oracle.step(cmx, 1e-3, qx, qdx, mode, tau, 50)
    np.testing.assert_allclose(fw.q, qx, atol=1e-7)
    np.testing.assert_allclose(fw.qd, qdx, atol=1e-6)
    assert np.abs(fw.V).max() < 1e-6


def test_free_fall_leaves_joints_weightless(oracle):
    text = chain_urdf(2)
    a = oracle.FloatWorld(oracle.load_urdf(text, pose_xyz=(0, 0, 5.0)), ground=False)
    b = oracle.FloatWorld(oracle.load_urdf(text, pose_xyz=(0, 0, 5.0), gravity=(0, 0, 0)), ground=False)
    for w in (a, b):
        w.set_joints([0.4, -0.3], [1.0, -0.5])
        w.set_twist([0.1, 0.2, -0.1], [0.0, 0.0, 0.0])
    for _ in range(300):
        a.step()
        b.step()
    np.testing.assert_allclose(a.q, b.q, atol=1e-10)
    np.testing.assert_allclose(a.qd, b.qd, atol=1e-10)
    # the base falls with g on top of the weightless motion (semi-implicit
    # Euler), up to the O(dt^2 |w| |v|) rotation-translation coupling of the
    # SE(3) exponential (the base spins)
    t_steps = 300
    dz = -G * 1e-3 * 1e-3 * t_steps * (t_steps + 1) / 2
    assert a.p[2] - b.p[2] == pytest.approx(dz, abs=1e-5)


def test_momentum_drift_is_first_order(oracle, quad_file):
    drifts = []
    for dt in (1e-3, 1e-4):
        cm = oracle.load_urdf(quad_file, pose_xyz=(0, 0, 1.0), gravity=(0, 0, 0))
        fw = oracle.FloatWorld(cm, dt=dt, ground=False)
        rng = np.random.default_rng(0)
        fw.set_joints(np.array([0.3, -0.8] * 4), rng.uniform(-1, 1, 8))
        fw.set_twist(rng.uniform(-.5, .5, 3), rng.uniform(-.5, .5, 3))
        h0 = momentum(fw)
        steps = int(round(0.1 / dt))
        mode = np.full(8, oracle.FORCE, np.int32)
        for k in range(steps):
            fw.step(mode, 2 * np.sin(10 * k * dt + np.arange(8)))
        drifts.append(np.abs(momentum(fw) - h0).max())
    assert drifts[0] < 0.05
    assert 7.0 < drifts[0] / drifts[1] < 13.0


def test_standing_quadruped_carries_its_weight(oracle, quad_file):
    cm = oracle.load_urdf(quad_file, pose_xyz=(0, 0, 0.45))
    fw = oracle.FloatWorld(cm, pgs_iters=50)
    fw.set_joints(STAND, np.zeros(8))
    mode = np.full(8, oracle.FORCE, np.int32)
    heights = []
    for k in range(2000):
        fw.step(mode, -400 * (fw.q - STAND) - 10 * fw.qd)
        heights.append(fw.p[2])
    assert len(fw.contacts) == 4
    assert sorted(c[3] for c in fw.contacts) == [1, 3, 5, 7]     # the shanks (feet)
    fz = sum(c[1][2] for c in fw.contacts)
    assert fz == pytest.approx(16.0 * G, abs=0.1)
    for c in fw.contacts:
        assert c[1][2] > 0 and c[2] > 0                           # pushing up, penetrating
    assert np.ptp(heights[-500:]) < 1e-4                           # at rest
    assert abs(heights[-1] - 0.4408) < 2e-3                        # feet 3 cm spheres, small sag


def test_warm_started_pgs_mode(oracle):
    """or_float_step_warm (the wave kernel's mw_set_pgs_options twin): without
    options it is or_float_step bit for bit; the warm record holds the step's
    impulses by contact slot (3 slot + d) and joint row; on the standing
    humanoid the normal impulses of the record carry the weight (m g dt), and
    the velocity-tolerance exit runs fewer sweeps than the budget while staying
    within 1e-4 of the fixed-count step."""
    import ctypes
    from mwstep import get_model_file
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    cm = oracle.load_urdf(get_model_file("icub"), pose_xyz=ICUB_POSE[:3], pose_wxyz=ICUB_POSE[3:])
    n = cm.n
    q0 = np.array(icub_posture(cm.joint_names))
    kp, kd = np.array(icub_pid_gains(cm.joint_names)).T
    hold = lambda w: np.clip(-kp * (w.q - q0) - kd * w.qd, -80, 80)
    mode = np.full(n, oracle.FORCE, np.int32)
    a = oracle.FloatWorld(cm, pgs_iters=50)
    b = oracle.FloatWorld(cm, pgs_iters=50, warm_start=True)
    for w in (a, b):
        w.set_joints(q0, np.zeros(n))
    for _ in range(600):           # lands (4 mm) and settles on its feet
        a.step(mode, hold(a))
        b.warm[:] = 0.0            # cold every step: identical arithmetic
        b.step(mode, hold(b))
    assert np.array_equal(a.q, b.q) and np.array_equal(a.V, b.V)
    # the record: normal impulses at 3 slot, their sum m g dt
    normals = b.warm[0:3 * oracle.OR_MAXFC:3]
    mass = cm.free.mass + sum(cm.model.mass[i] for i in range(n))
    assert np.count_nonzero(normals) == len(b.contacts)
    assert normals.sum() == pytest.approx(mass * 9.8 * 1e-3, rel=0.02)
    # tolerance exit
    c = oracle.FloatWorld(cm, pgs_iters=50, pgs_tol=1e-6, warm_start=True)
    c.s = oracle.OrFloatState()
    ctypes.pointer(c.s)[0] = b.s
    c.warm[:] = b.warm
    sweeps = []
    for _ in range(50):
        tau = hold(b)
        c.step(mode, tau)
        s = ctypes.c_int()
        oracle.lib().or_pgs_stats(ctypes.byref(s), None)
        sweeps.append(s.value)
        b.step(mode, tau)
    assert np.mean(sweeps) < 50
    assert np.abs(c.q - b.q).max() <= 1e-4 and np.abs(c.p - b.p).max() <= 1e-5
