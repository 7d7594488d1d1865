"""Scene preparation for the Pendulum task without randomization."""

from gym_ignition.randomizers import gazebo_env_randomizer

from ..models import pendulum
from .cartpole_no_rand import _replace_model


class PendulumEnvNoRandomizations(gazebo_env_randomizer.GazeboEnvRandomizer):
    def __init__(self, env):
        super().__init__(env=env)

    def randomize_task(self, task, **kwargs) -> None:
        if "gazebo" not in kwargs:
            raise ValueError("gazebo kwarg not passed to the task randomizer")
        _replace_model(task, kwargs["gazebo"], pendulum.Pendulum)
