"""Scene preparation for the CartPole tasks without randomization (reference:
python/gym_ignition_environments/randomizers/cartpole_no_rand.py:17-60):
every reset replaces the cartpole with a fresh one, then the task resets it."""

from gym_ignition.randomizers import gazebo_env_randomizer

from ..models import cartpole


def _replace_model(task, gazebo, factory) -> None:
    world = task.world
    if task.model_name is not None and task.model_name in world.model_names():
        if not world.to_gazebo().remove_model(task.model_name):
            raise RuntimeError("Failed to remove the model from the world")
    if not gazebo.run(paused=True):
        raise RuntimeError("Failed to execute a paused Gazebo run")
    task.model_name = factory(world=world).name()
    if not gazebo.run(paused=True):
        raise RuntimeError("Failed to execute a paused Gazebo run")


class CartpoleEnvNoRandomizations(gazebo_env_randomizer.GazeboEnvRandomizer):
    def __init__(self, env):
        super().__init__(env=env)

    def randomize_task(self, task, **kwargs) -> None:
        if "gazebo" not in kwargs:
            raise ValueError("gazebo kwarg not passed to the task randomizer")
        _replace_model(task, kwargs["gazebo"], cartpole.CartPole)
