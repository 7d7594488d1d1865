from mwstep import get_model_file
from scenario import core as scenario_core

from gym_ignition.scenario import model_with_file, model_wrapper

from ._insert import insert


class Panda(model_wrapper.ModelWrapper, model_with_file.ModelWithFile):
    """The shipped Franka Panda (reference: models/panda.py:11-77): the arm's
    home configuration, the Franka Gazebo PID gains of every joint and the
    reference's controller-period call."""

    HOME = [0, -0.785, 0, -2.356, 0, 1.571, 0.785]
    PID_GAINS_1000HZ = {  # models/panda.py:48-58
        "panda_joint1": (50, 0, 20), "panda_joint2": (10000, 0, 500),
        "panda_joint3": (100, 0, 10), "panda_joint4": (1000, 0, 50),
        "panda_joint5": (100, 0, 10), "panda_joint6": (100, 0, 10),
        "panda_joint7": (10, 0.5, 0.1), "panda_finger_joint1": (100, 0, 50),
        "panda_finger_joint2": (100, 0, 50),
    }

    def __init__(self, world, position=(0.0, 0.0, 0.0), orientation=(1.0, 0, 0, 0),
                 model_file: str = None):
        model = insert(world, "panda", model_file or self.get_model_file(), position, orientation)
        model.to_gazebo().reset_joint_positions(
            self.HOME, [name for name in model.joint_names() if "panda_joint" in name])
        if set(model.joint_names()) != set(self.PID_GAINS_1000HZ):
            raise ValueError("The number of PIDs does not match the number of joints")
        for joint_name, gains in self.PID_GAINS_1000HZ.items():
            if not model.get_joint(joint_name).set_pid(pid=scenario_core.PID(*gains)):
                raise RuntimeError(f"Failed to set the PID of joint '{joint_name}'")
        # the reference passes 1000.0 here (a period in seconds): the PID then
        # computes on the first step and holds its command; callers that track
        # targets set the period to the step size (test_pid_controllers.py:69)
        assert model.set_controller_period(1000.0)
        super().__init__(model=model)

    @classmethod
    def get_model_file(cls) -> str:
        return get_model_file("panda")
