"""Runtime: the gym.Env that executes a Task (reference: python/gym_ignition/base/runtime.py:10-81)."""

import abc

from mwstep import gym_module

_gym = gym_module()


class Runtime(_gym.Env, abc.ABC):
    def __init__(self, task, agent_rate: float):
        self.task = task
        self.agent_rate = agent_rate

    @abc.abstractmethod
    def timestamp(self) -> float:
        """Simulated time (simulated runtimes) or host time (real-time runtimes)."""
