"""Randomizer interfaces (reference: python/gym_ignition/randomizers/abc.py)."""

import abc


class TaskRandomizer(abc.ABC):
    @abc.abstractmethod
    def randomize_task(self, task, **kwargs) -> None:
        """Prepare the world of `task` for a new rollout."""


class PhysicsRandomizer(abc.ABC):
    def __init__(self, randomize_after_rollouts_num: int = 0):
        self._every = randomize_after_rollouts_num
        self._rollouts = 0

    @abc.abstractmethod
    def get_engine(self):
        ...

    def increase_rollout_counter(self) -> None:
        self._rollouts += 1

    def physics_expired(self) -> bool:
        return self._every != 0 and self._rollouts > 0 and self._rollouts % self._every == 0
