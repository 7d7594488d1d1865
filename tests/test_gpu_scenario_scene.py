"""GPU tests of the ScenarI/O mirror on its scene backend (several models
per world, batched worlds, world wrenches), as the reference's own scenario
tests state them:

  * tests/test_scenario/test_contacts.py:58-122 (cube on the ground) and
    :125-236 (three cubes, the third inserted after 50 steps onto the gap of
    the other two), both collision variants, through World / Model / Link;
  * Link.apply_world_force / torque / wrench / wrench_to_com (Link.cpp:484-560)
    with durations, and the free-fall result v = F t / m;
  * multi-world (GazeboSimulator.cpp:435-488): N worlds inserted from one SDF
    are the N worlds of ONE scene stepped by one launch; the same model
    inserted into each world shares one slot; worlds stay independent.
"""

import numpy as np
import pytest

from scene_models import cube_urdf

pytestmark = pytest.mark.gpu
G = 9.8


def _gazebo(worlds=None):
    from mwstep import get_model_file
    from scenario import gazebo as scenario
    gz = scenario.GazeboSimulator(0.001, 1.0, 1)
    if worlds:
        assert gz.insert_worlds_from_sdf(
            '<sdf version="1.6">' + "".join(f'<world name="{w}"></world>' for w in worlds) + "</sdf>")
    assert gz.initialize()
    return gz, get_model_file


@pytest.mark.parametrize("double", [False, True])
def test_cube_contact(require_gpu, double):
    from scenario import core
    from scenario import gazebo as scenario
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    assert world.insert_model_from_string(cube_urdf(double), core.Pose([0, 0, 0.15], [1., 0, 0, 0]), "cube")
    cube = world.get_model("cube")
    assert not cube.contacts_enabled()
    assert cube.enable_contacts(enable=True)
    gazebo.run(paused=True)
    assert not cube.get_link("cube").in_contact()
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
    # the reference compares with the default approx (exact zeros): float32
    # impulses leave 4e-6 N of tangential residual on the 49 N contact
    assert cube.get_link("cube").contact_wrench() == pytest.approx([0, 0, np.sum(z_forces), 0, 0, 0], abs=2e-5)
    gazebo.close()


@pytest.mark.parametrize("double", [False, True])
def test_cube_multiple_contacts(require_gpu, double):
    """tests/test_scenario/test_contacts.py:125-236, line by line."""
    from scenario import core
    from scenario import gazebo as scenario
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    cube_urdf_s = cube_urdf(double)
    assert world.insert_model_from_string(cube_urdf_s, core.Pose([0, -0.15, 0.101], [1., 0, 0, 0]), "cube1")
    assert world.insert_model_from_string(cube_urdf_s, core.Pose([0, 0.15, 0.101], [1., 0, 0, 0]), "cube2")
    assert len(world.model_names()) == 3
    cube1, cube2 = world.get_model("cube1"), world.get_model("cube2")
    assert cube1.enable_contacts(enable=True) and cube2.enable_contacts(enable=True)
    gazebo.run(paused=True)
    assert not cube1.get_link("cube").in_contact() and not cube2.get_link("cube").in_contact()
    for _ in range(50):
        gazebo.run()
    assert cube1.get_link("cube").in_contact() and cube2.get_link("cube").in_contact()
    assert len(cube1.contacts()) == 1 and len(cube2.contacts()) == 1
    assert world.insert_model_from_string(cube_urdf_s, core.Pose([0, 0, 0.301], [1., 0, 0, 0]), "cube3")
    assert len(world.model_names()) == 4
    cube3 = world.get_model("cube3")
    assert not cube3.contacts_enabled()
    assert cube3.enable_contacts(enable=True)
    gazebo.run(paused=True)
    assert not cube3.get_link("cube").in_contact()
    assert len(cube3.contacts()) == 0
    for _ in range(50):
        gazebo.run()
    assert cube3.get_link("cube").in_contact()
    assert len(cube3.contacts()) == 2
    contact1, contact2 = cube3.contacts()
    assert contact1.body_a == "cube3::cube" and contact2.body_a == "cube3::cube"
    assert contact1.body_b == "cube1::cube" and contact2.body_b == "cube2::cube"
    assert cube3.get_link("cube").contact_wrench() == pytest.approx([0, 0, 50, 0, 0, 0], abs=1.1)
    assert cube1.get_link("cube").contact_wrench()[2] == pytest.approx(50, abs=1.1)
    assert cube2.get_link("cube").contact_wrench()[2] == pytest.approx(50, abs=1.1)
    for contact in cube2.contacts():
        if contact.body_b == "cube3::cube":
            for point in contact.points:
                assert point.force[2] < 0
                assert point.normal == pytest.approx([0, 0, -1], abs=0.001)
        if contact.body_b == "ground_plane::link":
            for point in contact.points:
                assert point.force[2] > 0
                assert point.normal == pytest.approx([0, 0, 1], abs=0.001)
    gazebo.close()


def test_link_world_wrenches(require_gpu):
    """Link.apply_world_force for 0.1 s at 1 kHz (100 steps) on a floating
    cube in the air: v_x = F t / m; apply_world_wrench_to_com on a second
    cube's COM for 0.05 s: v_y = F t / m; apply_world_torque on a third spins
    it about z at tau t / I."""
    from scenario import core
    from scenario import gazebo as scenario
    gazebo, _ = _gazebo()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    for k, name in enumerate(("a", "b", "c")):
        assert world.insert_model_from_string(cube_urdf(), core.Pose([2.0 * k, 0, 10.0], [1., 0, 0, 0]), name)
    gazebo.run(paused=True)
    a, b, c = (world.get_model(n) for n in ("a", "b", "c"))
    assert a.get_link("cube").apply_world_force([25.0, 0.0, 0.0], 0.1)
    assert b.get_link("cube").apply_world_wrench_to_com([0.0, 10.0, 0.0], [0.0, 0.0, 0.0], 0.05)
    assert c.get_link("cube").apply_world_torque([0.0, 0.0, 0.05], 0.1)
    for _ in range(150):
        assert gazebo.run()
    I = 1 / 12 * 5.0 * (0.04 + 0.04)
    assert a.base_world_linear_velocity()[0] == pytest.approx(25.0 / 5.0 * 0.1, rel=1e-5)
    assert a.base_world_linear_velocity()[2] == pytest.approx(-G * 0.15, rel=1e-5)
    assert b.base_world_linear_velocity()[1] == pytest.approx(10.0 / 5.0 * 0.05, rel=1e-5)
    assert c.base_world_angular_velocity()[2] == pytest.approx(0.05 / I * 0.1, rel=1e-5)
    assert c.base_world_linear_velocity()[0] == pytest.approx(0.0, abs=1e-9)
    gazebo.close()


def test_multi_world_is_one_batched_scene(require_gpu):
    from scenario import gazebo as scenario
    names = [f"w{k}" for k in range(6)]
    gazebo, get_model_file = _gazebo(names)
    assert gazebo.world_names() == names
    assert gazebo._scene.n_worlds == 6
    q0 = np.linspace(-1.0, 1.0, 6)
    for name, q in zip(names, q0):
        w = gazebo.get_world(name)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(get_model_file("pendulum"))
        assert w.get_model("pendulum").reset_joint_positions([q])
    assert len(gazebo._slots) == 1            # one model slot, present in all six worlds
    for _ in range(200):
        assert gazebo.run()
    qs = [gazebo.get_world(n).get_model("pendulum").joint_positions()[0] for n in names]
    # independent worlds: a world started at -q mirrors the one started at q
    assert qs[0] == pytest.approx(-qs[5], abs=1e-5) and qs[1] == pytest.approx(-qs[4], abs=1e-5)
    assert len(set(np.round(qs, 6))) == 6
    # removing the model from one world leaves the others stepping
    assert gazebo.get_world("w2").remove_model("pendulum")
    q3 = gazebo.get_world("w3").get_model("pendulum").joint_positions()[0]
    assert gazebo.run()
    assert gazebo.get_world("w3").get_model("pendulum").joint_positions()[0] != q3
    gazebo.close()


def test_model_total_mass(require_gpu):
    """Model::totalMass (Model.cpp:413-425): the sum of Link::mass over the
    links -- the CartPole's rail (welded to the world), cart and pole; the
    iCub-class model's 30.7 kg; a subset of links."""
    from scenario import core
    from scenario import gazebo as scenario
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("cartpole"))
    assert world.insert_model(get_model_file("icub"), core.Pose([2.0, 0, 0.6], [0., 0, 0, 1]), "h")
    cp, h = world.get_model("cartpole"), world.get_model("h")
    assert cp.total_mass() == pytest.approx(5.0 + 1.0 + 0.1, abs=1e-6)
    assert cp.total_mass(["cart", "pole"]) == pytest.approx(1.1, abs=1e-6)
    assert h.total_mass() == pytest.approx(30.7, abs=1e-3)
    gazebo.close()


def _ground_plane_sdf(mu):
    return ('<sdf version="1.6"><model name="ground_plane"><static>true</static><link name="link">'
            '<collision name="collision"><geometry><plane><normal>0 0 1</normal><size>100 100</size></plane>'
            f'</geometry><surface><friction><ode><mu>{mu}</mu></ode></friction></surface></collision>'
            '</link></model></sdf>')


def test_floating_model_at_random_poses_shares_one_slot(require_gpu):
    """N worlds inserting one floating model at N different poses (an env's
    randomised spawn) take one scene slot, not N (the slot capacity is 8):
    each world's base starts at its own insert pose and falls freely from it."""
    from scenario import core
    from scenario import gazebo as scenario
    names = [f"w{k}" for k in range(12)]
    gazebo, get_model_file = _gazebo(names)
    rng = np.random.default_rng(3)
    xyz = np.c_[rng.uniform(-2, 2, (12, 2)), rng.uniform(1.0, 3.0, 12)]
    for n, p in zip(names, xyz):
        w = gazebo.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(get_model_file("cube"), core.Pose(list(p), [1., 0, 0, 0]), "c")
    assert len(gazebo._slots) == 1
    assert gazebo.run(paused=True)  # inserted models appear at the next (paused) run, as in the reference
    for n, p in zip(names, xyz):
        assert gazebo.get_world(n).get_model("c").base_position() == pytest.approx(list(p), abs=1e-6), n
    T = 100
    for _ in range(T):
        assert gazebo.run()
    dt = 1e-3
    for n, p in zip(names, xyz):
        pos = gazebo.get_world(n).get_model("c").base_position()
        assert pos[:2] == pytest.approx(list(p[:2]), abs=1e-6), n
        assert pos[2] == pytest.approx(p[2] - 9.8 * dt * dt * T * (T + 1) / 2, abs=1e-4), n
    gazebo.close()


def test_per_world_gravity_and_ground_friction(require_gpu):
    """World::setGravity and the ground plane's friction act on their own world
    only (World.cpp:301-319: each world of a server keeps its own Gravity
    component), although all worlds of the simulator are one batched scene:
    free-falling cubes fall with their world's gravity (z = z0 - g t^2 / 2
    under semi-implicit Euler), a cube pushed sideways on the ground slides
    to rest sooner on the rougher plane."""
    from scenario import core
    from scenario import gazebo as scenario
    names = ["low", "earth", "rough"]
    gazebo, get_model_file = _gazebo(names)
    grav = {"low": -1.62, "earth": -9.8, "rough": -9.8}
    for n in names:
        w = gazebo.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.set_gravity([0.0, 0.0, grav[n]])
    for n in names:
        assert gazebo.get_world(n).gravity() == pytest.approx([0.0, 0.0, grav[n]])
    for n in ("low", "earth"):
        assert gazebo.get_world(n).insert_model(get_model_file("cube"), core.Pose([0, 0, 5.0], [1., 0, 0, 0]), "c")
    T = 200
    for _ in range(T):
        assert gazebo.run()
    dt = 1e-3
    for n in ("low", "earth"):
        z = gazebo.get_world(n).get_model("c").base_position()[2]
        # semi-implicit Euler from rest: z_T = z0 + g dt^2 T (T + 1) / 2
        assert z == pytest.approx(5.0 + grav[n] * dt * dt * T * (T + 1) / 2, abs=1e-4), n
    gazebo.close()
    # friction per world: the same push on two planes of different mu
    gazebo, get_model_file = _gazebo(["smooth", "rough"])
    for n, mu in (("smooth", 0.1), ("rough", 0.8)):
        w = gazebo.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(_ground_plane_sdf(mu))
        assert w.insert_model(get_model_file("cube"), core.Pose([0, 0, 0.1], [1., 0, 0, 0]), "c")
        assert w.get_model("c").to_gazebo().reset_base_world_velocity([1.0, 0, 0], [0, 0, 0])
    for _ in range(300):
        assert gazebo.run()
    v = {n: gazebo.get_world(n).get_model("c").base_world_linear_velocity()[0] for n in ("smooth", "rough")}
    x = {n: gazebo.get_world(n).get_model("c").base_position()[0] for n in ("smooth", "rough")}
    # Coulomb deceleration mu g: after 0.3 s the smooth cube still slides at ~1 - 0.1 * 9.8 * 0.3
    assert v["smooth"] == pytest.approx(1.0 - 0.1 * 9.8 * 0.3, abs=0.05)
    assert abs(v["rough"]) < 1e-3 and x["rough"] < x["smooth"]
    gazebo.close()


def test_world_api_with_sdf_model(require_gpu):
    """tests/test_scenario/test_world.py:73-146 (test_world_api): gravity,
    model names, default / custom names and poses, URDF file and string, the
    SDF cube of tests/common/utils.py:100-146 inserted from a string, removal
    taking effect at the next run, no time without the Physics system."""
    from scenario import core
    from scenario import gazebo as scenario
    from test_sdf_models import REF_CUBE_SDF
    import tempfile
    gazebo, _ = _gazebo()
    world = gazebo.get_world()
    gravity = [0, 0, 10.0]
    assert world.set_gravity(gravity)
    assert world.gravity() == pytest.approx(gravity)
    assert len(world.model_names()) == 0
    assert not world.insert_model("")
    with tempfile.NamedTemporaryFile("w", suffix=".urdf", delete=False) as f:
        f.write(cube_urdf())
        cube_file = f.name
    assert world.insert_model(cube_file)
    assert len(world.model_names()) == 1
    default_model_name = scenario.get_model_name_from_sdf(cube_file, 0)
    assert default_model_name in world.model_names()
    cube1 = world.get_model(default_model_name)
    assert cube1.name() == default_model_name
    assert cube1.base_position() == pytest.approx([0, 0, 0])
    assert cube1.base_orientation() == pytest.approx([1, 0, 0, 0])
    assert not world.insert_model(cube_file)
    assert len(world.model_names()) == 1
    custom_model_name = "other_cube"
    custom_model_pose = core.Pose([1, 1, 0], [0, 0, 0, 1])
    assert world.insert_model(cube_file, custom_model_pose, custom_model_name)
    assert custom_model_name in world.model_names() and len(world.model_names()) == 2
    cube2 = world.get_model(custom_model_name)
    assert cube1 != cube2
    assert cube2.name() == custom_model_name
    assert cube2.base_position() == pytest.approx(custom_model_pose.position)
    assert cube2.base_orientation() == pytest.approx(custom_model_pose.orientation)
    assert world.insert_model_from_string(cube_urdf(), core.Pose([1, 0, 0], [0, 0, 0, 1]), "cube3")
    assert "cube3" in world.model_names()
    cube_4_pose = core.Pose([2, 0, 0], [0, 0, 0, 1])
    assert world.insert_model_from_string(REF_CUBE_SDF, cube_4_pose, "cube4")
    assert "cube4" in world.model_names()
    cube4 = world.get_model("cube4")
    assert cube4.base_position() == pytest.approx([2, 0, 0])
    assert cube4.base_orientation() == pytest.approx([0, 0, 0, 1])
    assert cube4.link_names() == ["box_link"]
    assert world.remove_model(default_model_name)
    assert len(world.model_names()) == 4
    gazebo.run(paused=True)
    assert len(world.model_names()) == 3
    gazebo.run()
    gazebo.run()
    gazebo.run()
    assert world.time() == 0.0
    gazebo.close()


def test_sdf_cube_falls_and_lands(require_gpu):
    """The reference's SDF cube (1 m edge, 1 kg, unit inertia, model pose
    0 0 0.5 kept under the identity insertion pose) lifted to z = 2: free fall
    z = 2 - g t^2 / 2 (semi-implicit Euler: g dt^2 k (k + 1) / 2 after k
    steps) until it touches the plane, then rests on it (z = 0.5, weight
    carried by the contact)."""
    from scenario import core
    from scenario import gazebo as scenario
    from test_sdf_models import REF_CUBE_SDF
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    assert world.insert_model_from_string(REF_CUBE_SDF)
    box = world.get_model("box")
    assert box.base_position() == pytest.approx([0, 0, 0.5])
    assert box.reset_base_pose([0, 0, 2.0], [1, 0, 0, 0])
    assert box.enable_contacts(True)
    gazebo.run(paused=True)
    assert box.base_position()[2] == pytest.approx(2.0)
    dt = 1e-3
    for k in range(1, 301):
        assert gazebo.run()
        z = box.base_position()[2]
        assert z == pytest.approx(2.0 - G * dt * dt * k * (k + 1) / 2, abs=2e-5), k
    for _ in range(1200):
        assert gazebo.run()
    assert box.base_position()[2] == pytest.approx(0.5, abs=2e-3)
    assert box.get_link("box_link").in_contact()
    fz = box.get_link("box_link").contact_wrench()[2]
    assert fz == pytest.approx(G * 1.0, abs=0.05)
    gazebo.close()


def test_sdf_and_urdf_pendulum_trajectories_agree(require_gpu, oracle):
    """The pendulum written as SDF (a revolute joint to the world, link and
    inertial poses in the model frame) and the shipped URDF pendulum, inserted
    into two worlds of one simulator: their joint trajectories agree over 500
    steps from the same reset, and both follow the fp64 oracle."""
    from scenario import gazebo as scenario
    from mwstep import get_model_file
    cm = oracle.load_urdf(get_model_file("pendulum"))
    M = cm.model
    E = np.array(M.E[0]).reshape(3, 3)
    Rj, pj = cm.base_R @ E, cm.base_R @ np.array(M.r[0]) + cm.base_p
    rpy = oracle._mat_to_rpy(Rj)
    I = [M.Ic[0][k] for k in range(6)]
    f = lambda v: " ".join(f"{x:.17g}" for x in v)
    sdf = f"""<sdf version='1.7'><model name='pendulum'>
      <link name='pole'><pose>{f((*pj, *rpy))}</pose>
        <inertial><pose>{f(M.com[0])} 0 0 0</pose><mass>{M.mass[0]:.17g}</mass>
          <inertia><ixx>{I[0]:.17g}</ixx><iyy>{I[1]:.17g}</iyy><izz>{I[2]:.17g}</izz>
                   <ixy>{I[3]:.17g}</ixy><ixz>{I[4]:.17g}</ixz><iyz>{I[5]:.17g}</iyz></inertia></inertial></link>
      <joint name='{cm.joint_names[0]}' type='revolute'><parent>world</parent><child>pole</child>
        <axis><xyz>{f(M.axis[0])}</xyz></axis></joint></model></sdf>"""
    gazebo, _ = _gazebo(["w_urdf", "w_sdf"])
    models = []
    for wn, text in (("w_urdf", open(get_model_file("pendulum")).read()), ("w_sdf", sdf)):
        world = gazebo.get_world(wn)
        assert world.set_physics_engine(scenario.PhysicsEngine_dart)
        assert world.insert_model_from_string(text)
        m = world.get_model("pendulum")
        assert m.reset_joint_positions([0.7]) and m.reset_joint_velocities([0.0])
        models.append(m)
    gazebo.run(paused=True)
    q_u, q_s = [], []
    for _ in range(500):
        assert gazebo.run()
        q_u.append(models[0].joint_positions()[0])
        q_s.append(models[1].joint_positions()[0])
    q_u, q_s = np.array(q_u), np.array(q_s)
    err = float(np.abs(q_u - q_s).max())
    print(f"SDF vs URDF pendulum over 500 steps: max |dq| {err:.2e}")
    assert err <= 1e-5
    # the fp64 oracle from the same start
    q, qd = np.array([0.7]), np.array([0.0])
    worst = 0.0
    for k in range(500):
        q, qd, *_ = oracle.step(cm, 1e-3, q, qd, np.full(1, oracle.FORCE, np.int32), np.zeros(1), 20)
        worst = max(worst, abs(float(q[0]) - q_s[k]))
    assert worst <= 1e-4, worst
    gazebo.close()


def test_static_sdf_collider(require_gpu, oracle):
    """A static SDF model with box / cylinder collisions (a table: top and a
    leg, yawed model frame) is a welded collider (Physics.cpp:687-1219 creates
    static models in the engine): a ball dropped on the table top comes to rest
    on it at top + r, carried by its contact with the table (weight within
    0.05 N), the table does not move, and the ball follows the fp64 scene
    oracle (position within 1e-4 m over 800 steps)."""
    from scenario import core
    from scenario import gazebo as scenario
    from scene_models import sphere_urdf
    from test_sdf_models import STATIC_TABLE_SDF
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    assert world.insert_model_from_string(STATIC_TABLE_SDF)
    table = world.get_model("table")
    assert table.base_position() == pytest.approx([0.5, 0, 0]) and table.dofs() == 0
    ball_text = sphere_urdf(1.0, 0.05)
    assert world.insert_model_from_string(ball_text, core.Pose([0.5, 0, 0.8], [1.0, 0, 0, 0]), "ball")
    ball = world.get_model("ball")
    assert ball.enable_contacts(True)
    cms = [oracle.load_urdf(STATIC_TABLE_SDF), oracle.load_urdf(ball_text, pose_xyz=(0.5, 0, 0.8))]
    ow = oracle.SceneWorld(cms, mu=1.0, pgs_iters=oracle.PGS_CONVERGED)  # the ScenarI/O scene solves exactly
    worst = 0.0
    for k in range(800):
        assert gazebo.run()
        ow.step()
        if k % 50 == 49:
            worst = max(worst, float(np.abs(np.array(ball.base_position()) - ow.p(1)).max()))
    z = ball.base_position()[2]
    print(f"ball on a static SDF table: z {z:.5f} (top 0.5 + r 0.05), max |dp| vs oracle {worst:.2e}")
    assert z == pytest.approx(0.55, abs=2e-3)
    assert worst <= 1e-4
    assert table.base_position() == pytest.approx([0.5, 0, 0])
    cs = ball.contacts()
    assert len(cs) == 1 and cs[0].body_b.startswith("table::")
    fz = sum(p.force[2] for p in cs[0].points)
    assert fz == pytest.approx(G * 1.0, abs=0.05)
    gazebo.close()


def test_model_api_completion(require_gpu):
    """ScenarI/O accessors without physics effect (core/Model.h, Joint.h,
    Link.h): nrOfJoints / nrOfLinks, jointLimits (Model.cpp:797-815),
    linksInContact (:725-736), joint acceleration targets (stored, a missing
    one raises like getExistingComponentData), the Base*Target components
    (:1077-1246; setBasePositionTarget keeps the orientation, default
    identity), the vectorised Joint forms and Link::mass."""
    import math
    from scenario import core
    from scenario import gazebo as scenario
    gazebo, get_model_file = _gazebo()
    world = gazebo.get_world()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    assert world.insert_model(get_model_file("cartpole"))
    assert world.insert_model_from_string(cube_urdf(), core.Pose([2, 0, 0.1], [1.0, 0, 0, 0]), "cube")
    cart = world.get_model("cartpole")
    cube = world.get_model("cube")
    assert cart.nr_of_joints() == 2 and cart.nr_of_links() == len(cart.link_names()) == 3
    lim = cart.joint_limits()
    assert len(lim.min) == 2 and lim.max[1] == math.inf
    assert lim.min[0] == cart.get_joint(cart.joint_names()[0]).position_limit().min
    with pytest.raises(RuntimeError):
        cart.joint_acceleration_targets()
    assert cart.set_joint_acceleration_targets([1.0, -2.0])
    assert cart.joint_acceleration_targets() == [1.0, -2.0]
    j = cart.get_joint(cart.joint_names()[1])
    assert j.acceleration_target() == -2.0 and j.joint_acceleration_target() == [-2.0]
    assert j.set_joint_acceleration_target([0.5]) and j.acceleration_target() == 0.5
    assert not cart.set_joint_acceleration_targets([1.0])
    assert j.joint_max_generalized_force() == [j.max_generalized_force()]
    with pytest.raises(RuntimeError):
        cube.base_position_target()
    assert cube.set_base_position_target([1, 2, 3])
    assert cube.base_position_target() == [1, 2, 3] and cube.base_orientation_target() == [1, 0, 0, 0]
    assert cube.set_base_orientation_target([0, 0, 0, 1]) and cube.base_position_target() == [1, 2, 3]
    assert cube.set_base_world_velocity_target([0.1, 0, 0], [0, 0, 0.2])
    assert cube.base_world_linear_velocity_target() == [0.1, 0, 0]
    assert cube.base_world_angular_velocity_target() == [0, 0, 0.2]
    assert cube.set_base_world_linear_acceleration_target([0, 0, -1])
    assert cube.base_world_linear_acceleration_target() == [0, 0, -1]
    with pytest.raises(RuntimeError):
        cube.base_world_angular_acceleration_target()
    assert cube.get_link("cube").mass() == pytest.approx(5.0)
    pole = cart.get_link(cart.link_names()[-1])
    assert pole.mass() > 0.0
    assert cube.enable_contacts(True)
    for _ in range(100):
        assert gazebo.run()
    assert cube.links_in_contact() == ["cube"]
    gazebo.close()


def test_per_world_pid_and_joint_parameters(require_gpu):
    """Joint::setPID / setViscousFriction / Model::setControllerPeriod act on
    their own world (the reference keeps these components per world).  The
    same model inserted into several worlds shares one scene slot until one
    world changes a slot-wide parameter; that world's model then moves to a
    slot of its own, carrying its state: the worlds whose gains did not
    change keep tracking exactly as a never-touched world does."""
    from scenario import core
    from scenario import gazebo as scenario
    names = ["a", "b", "c"]
    gazebo, get_model_file = _gazebo(names)
    for n in names:
        w = gazebo.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(get_model_file("pendulum"))
        m = w.get_model("pendulum")
        assert m.set_joint_control_mode(core.JointControlMode_position)
        assert m.set_joint_position_targets([0.5])
    assert len(gazebo._slots) == 1
    for _ in range(50):
        assert gazebo.run()
    q50 = [gazebo.get_world(n).get_model("pendulum").joint_positions()[0] for n in names]
    assert q50[0] == q50[1] == q50[2]
    # world "a": stiffer gains, mid-run
    ja = gazebo.get_world("a").get_model("pendulum").get_joint(gazebo.get_world("a").get_model("pendulum").joint_names()[0])
    pid_b = gazebo.get_world("b").get_model("pendulum").joints()[0].pid()
    # (a new PID starts from a fresh state, as ign-math's does in the
    # reference: its first derivative term kicks)
    assert ja.set_pid(core.PID(50.0, 0.0, 0.0))
    assert ja.pid().p == pytest.approx(50.0)
    jb = gazebo.get_world("b").get_model("pendulum").joints()[0]
    assert jb.pid().p == pytest.approx(pid_b.p)         # "b" kept its gains
    assert gazebo.run()
    assert len(gazebo._slots) == 2                      # "a" left the shared slot at the run
    assert ja.pid().p == pytest.approx(50.0) and jb.pid().p == pytest.approx(pid_b.p)
    for _ in range(99):
        assert gazebo.run()
    qa, qb, qc = (gazebo.get_world(n).get_model("pendulum").joint_positions()[0] for n in names)
    assert qb == qc                                     # untouched worlds stay identical
    assert abs(qa - qb) > 1e-4 and abs(qa) < 10.0       # the retuned world moved differently
    # the other slot-wide components follow the same rule
    mb = gazebo.get_world("b").get_model("pendulum")
    assert mb.set_controller_period(0.01)
    assert gazebo.run() and len(gazebo._slots) == 3
    assert mb.controller_period() == pytest.approx(0.01)
    assert gazebo.get_world("c").get_model("pendulum").controller_period() != pytest.approx(0.01)
    gazebo.close()


def test_many_worlds_set_same_pid_share_one_slot(require_gpu):
    """the reference Panda wrapper calls set_pid on every joint and
    set_controller_period on its model (models/panda.py:48-71).  Eight worlds
    that each insert a Panda and make the same calls keep sharing one scene
    slot (the changes are applied to it once, at the next run); worlds that
    make different calls move as groups, one slot per distinct set of
    changes, and each world steps with its own gains."""
    from scenario import core
    from scenario import gazebo as scenario
    names = [f"w{i}" for i in range(8)]
    gazebo, get_model_file = _gazebo(names)
    gains = [core.PID(600.0 - 10 * i, 0.0, 5.0) for i in range(9)]
    for n in names:
        w = gazebo.get_world(n)
        assert w.set_physics_engine(scenario.PhysicsEngine_dart)
        assert w.insert_model(get_model_file("panda"))
        m = w.get_model("panda")
        assert m.set_controller_period(0.001)
        for jn, g in zip(m.joint_names(), gains):
            assert m.get_joint(jn).set_pid(g)
        assert m.set_joint_control_mode(core.JointControlMode_position)
        assert m.set_joint_position_targets([0.1] * m.dofs())
    assert gazebo.run()
    assert len(gazebo._slots) == 1
    models = [gazebo.get_world(n).get_model("panda") for n in names]
    for m in models:
        assert m.controller_period() == pytest.approx(0.001)
        assert [m.get_joint(j).pid().p for j in m.joint_names()] == pytest.approx([g.p for g in gains])
    for _ in range(20):
        assert gazebo.run()
    q = [m.joint_positions() for m in models]
    assert all(qq == q[0] for qq in q)
    # worlds 0-2 retune joint 0 the same way, world 3 another way: two groups move
    for i in range(4):
        j0 = models[i].get_joint(models[i].joint_names()[0])
        assert j0.set_pid(core.PID(100.0 if i < 3 else 50.0, 0.0, 1.0))
    # a change back to the slot's value is no change at all
    j0 = models[4].get_joint(models[4].joint_names()[0])
    assert j0.set_pid(core.PID(10.0, 0.0, 0.0)) and j0.set_pid(gains[0])
    assert gazebo.run()
    assert len(gazebo._slots) == 3
    assert len({m._sim.m for m in models[:3]}) == 1 and models[3]._sim.m != models[0]._sim.m
    assert len({m._sim.m for m in models[4:]}) == 1 and models[4]._sim.m not in (models[0]._sim.m, models[3]._sim.m)
    assert models[0].get_joint(models[0].joint_names()[0]).pid().p == pytest.approx(100.0)
    assert models[3].get_joint(models[3].joint_names()[0]).pid().p == pytest.approx(50.0)
    assert models[7].get_joint(models[7].joint_names()[0]).pid().p == pytest.approx(gains[0].p)
    for _ in range(50):
        assert gazebo.run()
    q = [m.joint_positions() for m in models]
    assert q[0] == q[1] == q[2] and q[4] == q[5] == q[6] == q[7]
    assert q[0] != q[4] and q[3] != q[0] and q[3] != q[4]
    gazebo.close()
