"""The decision-making Task interface (reference: python/gym_ignition/base/task.py:15-237).

A Task only talks to ScenarI/O objects (``world.get_model(...).get_joint(...)``);
it is unaware that the simulator behind them is the MI355X stepper.
"""

import abc
from typing import Dict, Optional, Tuple

import numpy as np

from mwstep import gym_module

_gym = gym_module()


class Task(abc.ABC):
    action_space = None
    observation_space = None

    def __init__(self, agent_rate: float) -> None:
        self._world = None
        self.agent_rate = agent_rate
        # RNG of the task: every random choice of a task must come from here
        self.np_random, self.seed = _gym.utils.seeding.np_random()

    @property
    def world(self):
        if self._world is None:
            raise Exception("The world was never stored")
        return self._world

    @world.setter
    def world(self, world) -> None:
        if world is None or str(world.name) == "":
            raise ValueError("World not valid")
        self._world = world

    def has_world(self) -> bool:
        return self._world is not None and str(self._world.name) != ""

    # ---- interface implemented by concrete tasks
    @abc.abstractmethod
    def create_spaces(self) -> Tuple[object, object]:
        """Return (action_space, observation_space)."""

    @abc.abstractmethod
    def reset_task(self) -> None:
        """Bring the task to its initial state (called by env.reset)."""

    @abc.abstractmethod
    def set_action(self, action) -> None:
        """Turn the action into simulator references (start of env.step)."""

    @abc.abstractmethod
    def get_observation(self) -> np.ndarray:
        """Observation after the simulator step."""

    @abc.abstractmethod
    def get_reward(self) -> float:
        """Scalar reward of the last step."""

    @abc.abstractmethod
    def is_done(self) -> bool:
        """Termination flag of the last step."""

    def get_info(self) -> Dict:
        return {}

    def seed_task(self, seed: Optional[int] = None):
        """Seed the task RNG and both spaces; returns [seed]."""
        if seed is None:
            seed = np.random.randint(2 ** 32 - 1)
        self.np_random, self.seed = _gym.utils.seeding.np_random(seed)
        self.action_space.seed(self.seed)
        self.observation_space.seed(self.seed)
        return [self.seed]
