"""Environment registrations (ids, rates and episode limits of the reference's
python/gym_ignition_environments/__init__.py:14-52)."""

import numpy

from mwstep import gym_module

from . import models, randomizers, tasks  # noqa: F401

_gym = gym_module()
_max_float = float(numpy.finfo(numpy.float32).max)

_ENVS = {
    "Pendulum-Gazebo-v0": tasks.pendulum_swingup.PendulumSwingUp,
    "CartPoleDiscreteBalancing-Gazebo-v0": tasks.cartpole_discrete_balancing.CartPoleDiscreteBalancing,
    "CartPoleContinuousBalancing-Gazebo-v0": tasks.cartpole_continuous_balancing.CartPoleContinuousBalancing,
    "CartPoleContinuousSwingup-Gazebo-v0": tasks.cartpole_continuous_swingup.CartPoleContinuousSwingup,
}

_registered = {s.id for s in _gym.envs.registry.all()} if hasattr(_gym.envs.registry, "all") else set()
for _id, _task_cls in _ENVS.items():
    if _id in _registered:
        continue
    _gym.envs.registration.register(
        id=_id,
        entry_point="gym_ignition.runtimes.gazebo_runtime:GazeboRuntime",
        max_episode_steps=5000,
        kwargs={"task_cls": _task_cls, "agent_rate": 1000, "physics_rate": 1000,
                "real_time_factor": _max_float})
