"""gym.Wrapper that prepares the world of a GazeboRuntime on every reset
(reference: python/gym_ignition/randomizers/gazebo_env_randomizer.py:72-103)."""

import abc
from typing import Callable, Union

from mwstep import gym_module

from ..runtimes import gazebo_runtime
from ..utils import logger
from . import abc as rabc
from .physics import dart

_gym = gym_module()


class GazeboEnvRandomizer(_gym.Wrapper, rabc.TaskRandomizer, abc.ABC):
    def __init__(self, env: Union[str, Callable], physics_randomizer=None, **kwargs):
        physics_randomizer = physics_randomizer or dart.DART()
        self._env_option = env
        self._kwargs = dict(kwargs, physics_engine=physics_randomizer.get_engine())
        _gym.Wrapper.__init__(self, self._make(env, **self._kwargs))
        self._physics_randomizer = physics_randomizer

    def reset(self, **kwargs):
        if self._physics_randomizer.physics_expired():
            seed, rng = self.env.task.seed, self.env.task.np_random
            self.env.close()
            self.env = self._make(self._env_option, **self._kwargs)
            self.env.seed(seed=seed)
            self.env.task.np_random = rng
        self._physics_randomizer.increase_rollout_counter()
        self.randomize_task(task=self.env.task, gazebo=self.env.gazebo, **kwargs)
        if not self.env.gazebo.run(paused=True):
            raise RuntimeError("Failed to execute a paused Gazebo run")
        return self.env.reset()

    @staticmethod
    def _make(env, **kwargs):
        with logger.gym_verbosity(level=_gym.logger.WARN):
            made = _gym.make(env, **kwargs) if isinstance(env, str) else env(**kwargs)
        if not isinstance(made.unwrapped, gazebo_runtime.GazeboRuntime):
            raise ValueError("The environment to wrap is not a GazeboRuntime")
        return made
