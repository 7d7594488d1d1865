"""Randomizer interfaces (reference: python/gym_ignition/randomizers/abc.py)."""

import abc


class TaskRandomizer(abc.ABC):
    @abc.abstractmethod
    def randomize_task(self, task, **kwargs) -> None:
        """Prepare the world of `task` for a new rollout."""


class PhysicsRandomizer(abc.ABC):
    """Physics of a task's world, re-created every `randomize_after_rollouts_num`
    rollouts (0: never) by GazeboEnvRandomizer.reset()."""

    def __init__(self, randomize_after_rollouts_num: int = 0):
        self._every = randomize_after_rollouts_num
        self._rollouts = 0

    @abc.abstractmethod
    def randomize_physics(self, task, **kwargs) -> None:
        """Configure (and randomize) the physics of the task's world."""

    @abc.abstractmethod
    def get_engine(self):
        """The physics engine of the rollout (PhysicsEngine_dart)."""

    def increase_rollout_counter(self) -> None:
        self._rollouts += 1

    def physics_expired(self) -> bool:
        return self._every != 0 and self._rollouts > 0 and self._rollouts % self._every == 0


class ModelRandomizer(abc.ABC):
    @abc.abstractmethod
    def randomize_model(self, task, **kwargs):
        """Randomize the model of `task` already in the world."""


class ModelDescriptionRandomizer(abc.ABC):
    @abc.abstractmethod
    def randomize_model_description(self, task, **kwargs) -> str:
        """Return the path of a randomized model description file."""
