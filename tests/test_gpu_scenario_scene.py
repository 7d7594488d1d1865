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
