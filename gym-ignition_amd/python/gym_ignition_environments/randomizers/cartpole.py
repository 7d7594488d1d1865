"""Randomized CartPole environments on the ScenarI/O path (reference:
python/gym_ignition_environments/randomizers/cartpole.py:20-174).

Every reset removes the cartpole, inserts a new one whose link masses are the
nominal ones + max(U(-0.2, 0.2), 0) (SDFRandomizer, Additive, force_positive,
sampled from the task RNG), and lets the task reset it.  `randomize_physics`
draws gravity z ~ N(-9.8, 0.2) from the task RNG; as in the reference, the
environment randomizer itself only re-creates the simulator every
`num_physics_rollouts` rollouts and does not call it.  The batched
counterpart (per-world masses and gravity on the device) is
`mwstep.vecenv.VecEnv(..., randomize=True)`.
"""

import abc
from typing import Optional

from scenario import gazebo as scenario

from gym_ignition import randomizers
from gym_ignition.randomizers import gazebo_env_randomizer
from gym_ignition.randomizers.model.sdf import Distribution, Method, SDFRandomizer, UniformParams
from gym_ignition.utils import misc

from ..models import cartpole


class CartpoleRandomizersMixin(randomizers.abc.TaskRandomizer,
                               randomizers.abc.PhysicsRandomizer,
                               randomizers.abc.ModelDescriptionRandomizer,
                               abc.ABC):
    """Task, model-description and physics randomizations of the CartPole tasks."""

    def __init__(self, randomize_physics_after_rollouts: int = 0):
        randomizers.abc.PhysicsRandomizer.__init__(
            self, randomize_after_rollouts_num=randomize_physics_after_rollouts)
        self._sdf_randomizer: Optional[SDFRandomizer] = None

    # PhysicsRandomizer
    def get_engine(self):
        return scenario.PhysicsEngine_dart

    def randomize_physics(self, task, **kwargs) -> None:
        gravity_z = task.np_random.normal(loc=-9.8, scale=0.2)
        if not task.world.to_gazebo().set_gravity((0, 0, gravity_z)):
            raise RuntimeError("Failed to set the gravity")

    # TaskRandomizer
    def randomize_task(self, task, **kwargs) -> None:
        if "gazebo" not in kwargs:
            raise ValueError("gazebo kwarg not passed to the task randomizer")
        gazebo = kwargs["gazebo"]
        self._clean_world(task)
        if not gazebo.run(paused=True):
            raise RuntimeError("Failed to execute a paused Gazebo run")
        self._populate_world(task, self.randomize_model_description(task=task))
        if not gazebo.run(paused=True):
            raise RuntimeError("Failed to execute a paused Gazebo run")

    # ModelDescriptionRandomizer
    def randomize_model_description(self, task, **kwargs) -> str:
        return misc.string_to_file(self._get_sdf_randomizer(task).sample())

    def _get_sdf_randomizer(self, task) -> SDFRandomizer:
        if self._sdf_randomizer is not None:
            return self._sdf_randomizer
        # this backend loads the URDF itself (no URDF -> SDF conversion)
        randomizer = SDFRandomizer(sdf_model=cartpole.CartPole.get_model_file())
        randomizer.rng = task.np_random
        randomizer.new_randomization() \
            .at_xpath("*/link/inertial/mass") \
            .method(Method.Additive) \
            .sampled_from(Distribution.Uniform, UniformParams(low=-0.2, high=0.2)) \
            .force_positive() \
            .add()
        randomizer.process_data()
        assert len(randomizer.get_active_randomizations()) > 0
        self._sdf_randomizer = randomizer
        return randomizer

    @staticmethod
    def _clean_world(task) -> None:
        if task.model_name is not None and task.model_name in task.world.model_names():
            if not task.world.to_gazebo().remove_model(task.model_name):
                raise RuntimeError("Failed to remove the cartpole from the world")

    @staticmethod
    def _populate_world(task, cartpole_model: str = None) -> None:
        model = cartpole.CartPole(world=task.world, model_file=cartpole_model)
        task.model_name = model.name()


class CartpoleEnvRandomizer(gazebo_env_randomizer.GazeboEnvRandomizer, CartpoleRandomizersMixin):
    """Randomized CartPole environment (a gym.Wrapper over the GazeboRuntime)."""

    def __init__(self, env, num_physics_rollouts: int = 0):
        CartpoleRandomizersMixin.__init__(self, randomize_physics_after_rollouts=num_physics_rollouts)
        gazebo_env_randomizer.GazeboEnvRandomizer.__init__(self, env=env, physics_randomizer=self)
