"""Pendulum swing-up on the `pivot` joint (reference:
python/gym_ignition_environments/tasks/pendulum_swingup.py).

The reward reads the joint force target after the run; the physics system
zero-fills force commands after every step (Physics.cpp:2250-2254), so that
term is zero -- kept as-is for parity.
"""

import abc

import numpy as np
from scenario import core as scenario_core

from mwstep import gym_module
from gym_ignition.base import task

_gym = gym_module()


class PendulumSwingUp(task.Task, abc.ABC):
    max_speed = 10.0
    max_torque = 50.0

    def __init__(self, agent_rate: float, **kwargs):
        task.Task.__init__(self, agent_rate=agent_rate)
        self.model_name = None

    def _pivot(self):
        return self.world.get_model(self.model_name).get_joint("pivot")

    def create_spaces(self):
        action_space = _gym.spaces.Box(low=-self.max_torque, high=self.max_torque, shape=(1,),
                                       dtype=np.float32)
        high = np.array([1.0, 1.0, self.max_speed])
        return action_space, _gym.spaces.Box(low=-high, high=high, dtype=np.float32)

    def set_action(self, action) -> None:
        if not self._pivot().set_generalized_force_target(action.tolist()[0]):
            raise RuntimeError("Failed to set the force to the pendulum")

    def get_observation(self) -> np.ndarray:
        pivot = self._pivot()
        q, dq = pivot.position(), pivot.velocity()
        return np.array([np.cos(q), np.sin(q), dq])

    def is_done(self) -> bool:
        return not self.observation_space.contains(self.get_observation())

    def get_reward(self) -> float:
        pivot = self._pivot()
        q, dq, tau = pivot.position(), pivot.velocity(), pivot.generalized_force_target()
        cost = (100.0 if self.is_done() else 0.0) + q ** 2 + 0.1 * dq ** 2 + 0.001 * tau ** 2
        return -cost

    def reset_task(self) -> None:
        if self.model_name not in self.world.model_names():
            raise RuntimeError("The pendulum model was not inserted in the world")
        pivot = self._pivot()
        if not pivot.set_control_mode(scenario_core.JointControlMode_force):
            raise RuntimeError("Failed to change the control mode of the pendulum")
        cos_q, sin_q, dq = self.observation_space.sample()
        if not pivot.to_gazebo().reset(float(np.arctan2(sin_q, cos_q)), float(dq)):
            raise RuntimeError("Failed to reset the pendulum state")
