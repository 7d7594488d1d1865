"""The reference's iCub wrapper through the ScenarI/O mirror on the GPU
backend: ICubGazebo (python/gym_ignition_environments/
models/icub.py:80-99) inserts the iCub-class model at (0, 0, 0.572), wxyz
(0, 0, 0, 1) and calls reset_joint_positions(q0, joint_names) with the
wrapper's 32 names -- it must succeed, and the model reports the wrapper's
DOFS / NUM_JOINTS / NUM_LINKS.  Then the reference's JointController drives
a PID hold of that posture (Joint::setPID, Position mode, period = step
size) for 1 s: the robot lands on its feet and stands, its soles (the kept
l_foot / r_foot F/T-sensor links) carry the weight."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = 9.8


def test_icub_wrapper_through_scenario(require_gpu):
    from mwstep import get_model_file
    from mwstep.models import icub_pid_gains
    from scenario import core
    from scenario import gazebo as scenario

    from gym_ignition_environments.models.icub import ICubGazebo
    gazebo = scenario.GazeboSimulator(0.001, 1.0, 1)
    assert gazebo.initialize()
    world = gazebo.get_world().to_gazebo()
    assert world.set_physics_engine(scenario.PhysicsEngine_dart)
    assert world.insert_model(get_model_file("ground_plane"))
    icub = ICubGazebo(world=world)
    assert icub.name() == "icub"
    assert icub.dofs() == ICubGazebo.DOFS == 32
    assert icub.nr_of_joints() == ICubGazebo.NUM_JOINTS == 32
    assert icub.nr_of_links() == ICubGazebo.NUM_LINKS == 39
    assert {"l_foot", "r_foot", "l_hip_3", "r_upper_arm"} <= set(icub.link_names())
    assert icub.total_mass() == pytest.approx(30.7, abs=1e-4)
    names = list(ICubGazebo.initial_positions)
    q0 = np.array(list(ICubGazebo.initial_positions.values()))
    assert gazebo.run(paused=True)
    assert np.abs(np.array(icub.joint_positions(names)) - q0).max() <= 1e-6
    assert icub.base_position() == pytest.approx([0.0, 0.0, 0.572], abs=1e-6)
    assert icub.base_orientation() == pytest.approx([0.0, 0.0, 0.0, 1.0], abs=1e-6)
    # a kept link sits at its fixed offset from its body: the sole frame
    # 5 cm below the ankle's
    ankle, foot = icub.get_link("l_ankle_2"), icub.get_link("l_foot")
    d = np.array(foot.position()) - np.array(ankle.position())
    assert np.linalg.norm(d) == pytest.approx(0.05, abs=1e-6)
    assert foot.orientation() == pytest.approx(ankle.orientation(), abs=1e-6)
    # the posture hold
    assert icub.enable_contacts(True)
    assert icub.set_controller_period(0.001)
    for name, (p, d_) in zip(icub.joint_names(), icub_pid_gains(icub.joint_names())):
        j = icub.get_joint(name)
        assert j.set_pid(core.PID(p, 0.0, d_))
        assert j.set_control_mode(core.JointControlMode_position)
    assert icub.set_joint_position_targets(list(q0), names)
    for _ in range(1000):
        assert gazebo.run()
    assert icub.base_position()[2] == pytest.approx(0.565, abs=0.005)
    assert sorted(icub.links_in_contact()) == ["l_foot", "r_foot"]
    contacts = icub.contacts()
    assert sorted(c.body_a for c in contacts) == ["icub::l_foot", "icub::r_foot"]
    fz = sum(p.force[2] for c in contacts for p in c.points)
    assert sum(len(c.points) for c in contacts) == 8
    assert fz == pytest.approx(30.7 * G, abs=3.0)
    assert np.abs(np.array(icub.joint_positions(names)) - q0).max() < 0.06
    gazebo.close()
