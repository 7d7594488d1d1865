"""GPU tests of floating bodies with ground contacts (SURVEY.md §8f row 1,
first slice: single floating bodies).

  * the reference's contact KAT through the ScenarI/O mirror
    (tests/test_scenario/test_contacts.py:57-122; single and double-collision
    cube): no contact before falling, one contact (cube::cube vs
    ground_plane::link) after 150 ms, normals +z, the vertical forces sum to
    the weight within 0.1 N, Link::contactWrench = [0, 0, sum Fz, 0, 0, 0];
  * teacher-forced one-step parity against the fp64 oracle (or_free_step) on
    random poses / twists near the ground: pose and twist within 1e-5 (fp32 vs
    fp64), contact forces within 1e-3 relative -- on the world-per-wavefront
    kernel with DART's exact boxed LCP (the default for mw_sim floating
    models; oracle PGS_CONVERGED) and on the PGS-only free-body kernel
    (MW_LCP_PGS chosen before the model is loaded; oracle PGS 50);
  * free fall and torque-free spin over 1000 steps against the oracle;
  * base reset semantics (visible after the next run).
"""

import numpy as np
import pytest

from test_cylinder_oracle import cylinder_urdf
from test_free_body_oracle import cube_urdf, sphere_urdf

pytestmark = pytest.mark.gpu
G = 9.8


@pytest.mark.parametrize("double", [False, True])
def test_cube_contact_kat(require_gpu, double):
    from mwstep import get_model_file
    from scenario import core
    from scenario import gazebo as scenario
    gazebo = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gazebo.initialize()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    assert len(world.model_names()) == 1
    assert world.insert_model_from_string(cube_urdf(double), core.Pose([0, 0, 0.15], [1., 0, 0, 0]), "cube")
    assert len(world.model_names()) == 2
    cube = world.get_model("cube")
    assert not cube.contacts_enabled()
    assert cube.enable_contacts(enable=True)
    assert cube.contacts_enabled()
    gazebo.run(paused=True)
    assert not cube.get_link("cube").in_contact()
    assert len(cube.contacts()) == 0
    for _ in range(150):
        gazebo.run()
    assert cube.get_link("cube").in_contact()
    assert len(cube.contacts()) == 1
    c = cube.contacts()[0]
    assert c.body_a == "cube::cube" and c.body_b == "ground_plane::link"
    for point in c.points:
        assert point.normal == pytest.approx([0, 0, 1])
    z_forces = [point.force[2] for point in c.points]
    assert np.sum(z_forces) == pytest.approx(-5 * world.gravity()[2], abs=0.1)
    assert cube.get_link("cube").contact_wrench() == pytest.approx([0, 0, np.sum(z_forces), 0, 0, 0], abs=1e-4)
    gazebo.close()


def _quat_to_R(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _rock_body_urdf():
    """a free body whose collision is the 12-vertex rock mesh (two shape
    entries of 8 + 4 support points on the free-body kernel)"""
    import os
    import tempfile
    from mesh_models import mesh_body_urdf, rock_vertices, write_stl_binary
    path = os.path.join(tempfile.mkdtemp(), "rock.stl")
    write_stl_binary(path, *rock_vertices(7))
    return mesh_body_urdf(path, mass=3.0, half=(0.12, 0.08, 0.06), rpy=(0.2, 0.1, -0.3))


@pytest.mark.parametrize("kernel", ["wave", "free"])
@pytest.mark.parametrize("urdf", ["cube", "double", "sphere", "cylinder", "rock"])
def test_one_step_parity_with_contacts(require_gpu, oracle, urdf, kernel):
    from mwstep.sim import Simulator
    text = {"cube": cube_urdf, "double": lambda: cube_urdf(True), "sphere": sphere_urdf,
            "cylinder": lambda: cylinder_urdf(rpy="0.2 0 0"), "rock": _rock_body_urdf}[urdf]()
    W, pgs = 256, 50
    rng = np.random.default_rng(5)
    sim = Simulator(text, n_worlds=W, pgs_iters=pgs, lcp_exact=(kernel == "wave"))
    assert sim.float_kernel() == (2 if kernel == "wave" else 0)
    assert sim.lcp_solver()[0] is (kernel == "wave")
    opgs = oracle.PGS_CONVERGED if kernel == "wave" else pgs
    sim.set_ground_plane(True, 0.8)
    sim.enable_contacts(True)
    q = rng.normal(size=(W, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    zr = (0.0, 0.09) if urdf == "rock" else (0.05, 0.2)   # the rock is a few cm across
    pos = np.column_stack([rng.uniform(-1, 1, W), rng.uniform(-1, 1, W), rng.uniform(*zr, W)])
    lin = rng.uniform(-0.5, 0.5, (W, 3))
    ang = rng.uniform(-2, 2, (W, 3))
    sim.reset_base_pose(np.column_stack([pos, q]).astype(np.float32).astype(np.float64))
    sim.reset_base_velocity(np.column_stack([lin, ang]).astype(np.float32).astype(np.float64))
    sim.run(paused=True)
    p0, v0 = sim.base_pose(), sim.base_velocity()
    sim.run()
    p1, v1 = sim.base_pose(), sim.base_velocity()
    cm = oracle.load_urdf(text)
    worst_p = worst_v = worst_f = 0.0
    n_contact, ill = 0, []

    def oracle_step(w, eps=0.0, seed=0):
        # eps > 0: the conditioning probe -- every exact LCP solve of the step
        # sees its Delassus matrix perturbed by eps relative (pyoracle
        # set_lcp_perturbation)
        oracle.set_lcp_perturbation(eps, seed)
        try:
            R0 = _quat_to_R(p0[w, 3:])
            ow = oracle.FreeWorld(cm, ground=True, mu=0.8, pgs_iters=opgs)
            ow.set_pose(p0[w, :3], R0)
            ow.set_twist(R0.T @ v0[w, 3:], R0.T @ v0[w, :3])
            ow.step()
        finally:
            oracle.set_lcp_perturbation(0.0)
        return ow, np.concatenate([ow.R @ ow.twist[1], ow.R @ ow.twist[0]])

    for w in range(W):
        ow, wv = oracle_step(w)
        e_p = max(float(np.abs(p1[w, :3] - ow.p).max()), float(np.abs(_quat_to_R(p1[w, 3:]) - ow.R).max()))
        e_v = float(np.abs(v1[w] - wv).max())
        if kernel == "wave" and (e_v > 1e-4 or e_p > 1e-5):
            # DART's two-stage LCP boxes the friction by the FRICTIONLESS
            # normals; over redundant contacts (a rock's or a double box's
            # coincident points, cond(A) ~1e7 from the CFM) their split is
            # set by the CFM alone, and with it the saturated friction boxes:
            # accept the world only if the fp64 oracle moves as much when its
            # Delassus matrix carries a fp32-size error (1e-6 relative, ~16
            # ulps: the order of the kernel's fp32 A)
            sens = max(float(np.abs(oracle_step(w, 1e-6, k + 1)[1] - wv).max()) for k in range(4))
            ill.append((w, f"{e_v:.1e}", f"{sens:.1e}"))
            assert sens >= 0.1 * e_v, f"world {w}: GPU-oracle |dv| {e_v:.2e}, oracle sensitivity {sens:.2e}"
            assert e_p <= 2e-3 * e_v + 1e-5
            e_p = e_v = 0.0
        worst_p = max(worst_p, e_p)
        worst_v = max(worst_v, e_v)
        gc = sim.contacts(w)
        assert len(gc) == len(ow.contacts)
        n_contact += len(gc) > 0
        for row, (p, n, f, d) in zip(gc, ow.contacts):
            assert np.abs(row[0:3] - p).max() <= 1e-5
        if len(gc) and not (ill and ill[-1][0] == w):
            # the resultant: a body resting on redundant points (a cube's four
            # corners) has A of condition ~1e7 (DART's CFM), so the split of
            # the load among the corners is round-off sensitive in fp32 while
            # the force on the body -- what moves it -- is not
            fg = np.sum([row[6:9] for row in gc], axis=0)
            fo = np.sum([f for (_, _, f, _) in ow.contacts], axis=0)
            worst_f = max(worst_f, float(np.abs(fg - fo).max()) / (1.0 + float(np.abs(fo).max())))
    print(f"free body {urdf}, {kernel} kernel: one-step max|pose err| {worst_p:.2e}, max|vel err| {worst_v:.2e}, "
          f"force rel err {worst_f:.2e}, {n_contact}/{W} worlds in contact, "
          f"ill-conditioned (world, |dv|, oracle sensitivity): {ill}")
    assert n_contact > W // 4
    # excused worlds (W/64): the boxes, spheres and
    # cylinders stay within it; the rock mesh's support points are redundant
    # by construction (coplanar hull vertices: its frictionless stage splits
    # the load by the CFM alone, the oracle itself moves by 1e-2..1e-1 under a
    # 1e-6 relative error in A), measured 18 of 256 (profiles/r05a)
    assert len(ill) <= (W // 10 if urdf == "rock" else W // 64)
    assert worst_p <= 1e-5 and worst_v <= 1e-4 and worst_f <= 1e-3
    sim.close()


@pytest.mark.parametrize("exact", [True, False])
def test_free_fall_and_spin_parity(require_gpu, oracle, exact):
    from mwstep.sim import Simulator
    text = cube_urdf()
    sim = Simulator(text, n_worlds=2, pose=(0, 0, 10.0, 1, 0, 0, 0), gravity=(0, 0, -G), lcp_exact=exact)
    sim.reset_base_velocity([[0.3, -0.2, 1.0, 0.5, -1.0, 2.0], [0, 0, 0, 0, 0, 0]])
    sim.run(paused=True)
    cm = oracle.load_urdf(text, pose_xyz=(0, 0, 10.0))
    ow = oracle.FreeWorld(cm, ground=False)
    ow.set_twist([0.5, -1.0, 2.0], [0.3, -0.2, 1.0])
    for _ in range(1000):
        sim.run()
        ow.step()
    p = sim.base_pose()[0]
    assert np.abs(p[:3] - ow.p).max() <= 1e-4
    assert np.abs(_quat_to_R(p[3:]) - ow.R).max() <= 1e-4
    sim.close()


def test_base_reset_semantics(require_gpu):
    from mwstep import get_model_file
    from scenario import core
    from scenario import gazebo as scenario
    gazebo = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gazebo.initialize()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model_from_string(cube_urdf(), core.Pose([0, 0, 1.0], [1., 0, 0, 0]), "cube")
    cube = world.get_model("cube")
    assert cube.base_position() == pytest.approx([0, 0, 1.0])
    assert cube.reset_base_pose([1, 2, 3], [0, 0, 0, 1])
    assert cube.base_position() == pytest.approx([0, 0, 1.0])      # applied by the next run
    assert cube.reset_base_world_linear_velocity([0.1, 0, 0])
    assert cube.reset_base_world_angular_velocity([0, 0, 0.5])     # keeps the linear part
    gazebo.run(paused=True)
    assert cube.base_position() == pytest.approx([1, 2, 3])
    assert cube.base_orientation() == pytest.approx([0, 0, 0, 1])
    assert cube.base_world_linear_velocity() == pytest.approx([0.1, 0, 0], abs=1e-6)
    assert cube.base_world_angular_velocity() == pytest.approx([0, 0, 0.5], abs=1e-6)
    # the world-frame velocity of a body rotated by pi about z, seen in its frame
    assert cube.base_body_linear_velocity() == pytest.approx([-0.1, 0, 0], abs=1e-6)
    gazebo.close()


@pytest.mark.parametrize("exact", [True, False])
def test_run_device_equals_run(require_gpu, exact):
    """mw_run_device (no readback, graph-capturable) == repeated mw_run."""
    from mwstep import get_model_file
    from mwstep.sim import Simulator
    sims = [Simulator(get_model_file("cube"), n_worlds=64, pose=(0, 0, 0.3, 0.9, 0.3, 0.2, 0.1), lcp_exact=exact)
            for _ in range(2)]
    for s in sims:
        s.set_ground_plane(True, 0.7)
        s.enable_contacts(True)
        s.reset_base_velocity([0.2, 0.1, -0.5, 1.0, -2.0, 0.5])
        s.run(paused=True)
    for _ in range(300):
        sims[0].run()
    sims[1].run_device(300)
    assert np.array_equal(sims[0].base_pose(), sims[1].base_pose())
    assert np.array_equal(sims[0].base_velocity(), sims[1].base_velocity())
    assert np.array_equal(sims[0].contacts(5), sims[1].contacts(5))
    assert len(sims[0].contacts(5)) > 0
    for s in sims:
        s.close()


@pytest.mark.parametrize("exact", [True, False])
def test_cylinder_kats_on_mw_sim(require_gpu, oracle, exact):
    """The oracle's cylinder KATs (tests/test_cylinder_oracle.py) on mw_sim --
    the world-per-wavefront kernel with DART's exact LCP (default) and the
    PGS-only free-body kernel: a standing cylinder rests at half its length
    carrying its weight on 4 rim points; a lying one spun about its axis rolls
    without slipping at omega0 r / 3; both follow the fp64 oracle step by step."""
    import math
    from mwstep.sim import Simulator
    from test_cylinder_oracle import cylinder_urdf
    sim = Simulator(cylinder_urdf(), n_worlds=2, pose=(0, 0, 0.25, 1, 0, 0, 0), pgs_iters=100, lcp_exact=exact)
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    for _ in range(600):
        sim.run()
    p = sim.base_pose()
    assert p[:, 2] == pytest.approx(0.2, abs=2e-3)
    c = sim.contacts(0)
    assert len(c) == 4 and float(np.sum(c[:, 8])) == pytest.approx(2.0 * G, abs=0.05)
    sim.close()
    r, m = 0.1, 2.0
    ixx = m * (3 * r * r + 0.16) / 12.0
    text = (f'<robot name="roll"><link name="roll"><inertial><mass value="{m}"/>'
            f'<inertia ixx="{0.5 * m * r * r}" iyy="{ixx}" izz="{ixx}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><origin rpy="0 {math.pi / 2} 0" xyz="0 0 0"/><geometry>'
            f'<cylinder radius="{r}" length="0.4"/></geometry></collision></link></robot>')
    sim = Simulator(text, n_worlds=2, pose=(0, 0, r, 1, 0, 0, 0), pgs_iters=100, lcp_exact=exact)
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    ow = oracle.FreeWorld(oracle.load_urdf(text, pose_xyz=(0, 0, r)), mu=1.0,
                          pgs_iters=oracle.PGS_CONVERGED if exact else 100)
    for _ in range(100):
        sim.run()
        ow.step()
    sim.reset_base_velocity([[0, 0, 0, -10.0, 0, 0]] * 2)
    ow.set_twist(ow.R.T @ np.array([-10.0, 0, 0]), [0, 0, 0])
    worst = 0.0
    for k in range(1500):
        sim.run()
        ow.step()
        worst = max(worst, float(np.abs(sim.base_pose()[0, :3] - ow.p).max()))
    v = sim.base_velocity()[0]
    assert v[1] == pytest.approx(10.0 * r / 3.0, rel=0.03) and v[1] == pytest.approx(-v[3] * r, rel=0.02)
    print(f"rolling cylinder: v {v[1]:.4f} (omega0 r / 3 = {10 * r / 3:.4f}), max |dp| vs oracle {worst:.2e}")
    assert worst <= 2e-4
    sim.close()


def test_cube_kat_exact_on_mw_sim(require_gpu):
    """the reference's contact KAT
    (tests/test_scenario/test_contacts.py:58-122) on mw_sim with DART's exact
    LCP -- a cube dropped onto the plane rests on its 4 bottom corners, the
    normal forces carry its weight within 0.1 N, and the contact answer does
    not depend on the world count."""
    from mwstep.sim import Simulator
    for W in (1, 4096):
        sim = Simulator(cube_urdf(), n_worlds=W, pose=(0, 0, 0.15, 1, 0, 0, 0))
        assert sim.float_kernel() == 2 and sim.lcp_solver() == (True, 48)
        sim.set_ground_plane(True, 1.0)
        sim.enable_contacts(True)
        for _ in range(150):
            sim.run()
        c = sim.contacts(0)
        assert len(c) == 4 and np.allclose(c[:, 3:6], [0, 0, 1])
        assert float(np.sum(c[:, 8])) == pytest.approx(5.0 * G, abs=0.1)
        if W == 1:
            ref = (sim.base_pose()[0].copy(), c.copy())
        else:
            assert np.array_equal(sim.base_pose()[0], ref[0]) and np.array_equal(c, ref[1])
        assert sim.lcp_unconverged() == 0
        sim.close()
