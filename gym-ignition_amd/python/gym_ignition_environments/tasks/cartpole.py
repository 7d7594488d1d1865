"""CartPole tasks on the `linear` (cart) and `pivot` (pole) joints.

Behaviour follows the reference tasks
(python/gym_ignition_environments/tasks/cartpole_discrete_balancing.py,
cartpole_continuous_balancing.py, cartpole_continuous_swingup.py):
observation [x, dx, q, dq], termination when the observation leaves the reset
space, and the per-variant action, reward and reset distributions.  The same
logic runs batched on the device in mwstep's VecEnv (kernels.hip).
"""

import abc

import numpy as np
from scenario import core as scenario_core

from mwstep import gym_module
from gym_ignition.base import task

_gym = gym_module()


class _CartPole(task.Task, abc.ABC):
    # (x, dx, q, dq) limits of the reset space; the observation space is 1.2x
    x_limit = 2.4
    dx_limit = 20.0
    q_limit = np.deg2rad(12)
    dq_limit = np.deg2rad(3 * 360)

    def __init__(self, agent_rate: float, reward_cart_at_center: bool = True, **kwargs):
        task.Task.__init__(self, agent_rate=agent_rate)
        self.model_name = None
        self.reset_space = None
        self._reward_cart_at_center = reward_cart_at_center

    # -- spaces
    @abc.abstractmethod
    def _action_space(self):
        ...

    def create_spaces(self):
        high = np.array([self.x_limit, self.dx_limit, self.q_limit, self.dq_limit])
        self.reset_space = _gym.spaces.Box(low=-high, high=high, dtype=np.float32)
        obs_space = _gym.spaces.Box(low=-1.2 * high, high=1.2 * high, dtype=np.float32)
        return self._action_space(), obs_space

    # -- action
    @abc.abstractmethod
    def _force(self, action) -> float:
        ...

    def set_action(self, action) -> None:
        cart = self.world.get_model(self.model_name).get_joint("linear")
        if not cart.set_generalized_force_target(self._force(action)):
            raise RuntimeError("Failed to set the force to the cart")

    # -- observation / termination
    def get_observation(self) -> np.ndarray:
        model = self.world.get_model(self.model_name)
        q, x = model.joint_positions(["pivot", "linear"])
        dq, dx = model.joint_velocities(["pivot", "linear"])
        return np.array([x, dx, q, dq])

    def is_done(self) -> bool:
        return not self.reset_space.contains(self.get_observation())

    # -- reset
    @abc.abstractmethod
    def _initial_state(self):
        """Return (x, dx, q, dq) drawn from the task RNG."""

    def reset_task(self) -> None:
        if self.model_name not in self.world.model_names():
            raise RuntimeError("Cartpole model not found in the world")
        model = self.world.get_model(self.model_name)
        if not model.get_joint("linear").set_control_mode(scenario_core.JointControlMode_force):
            raise RuntimeError("Failed to change the control mode of the cartpole")
        x, dx, q, dq = self._initial_state()
        gz = model.to_gazebo()
        ok = gz.reset_joint_positions([x, q], ["linear", "pivot"])
        ok = gz.reset_joint_velocities([dx, dq], ["linear", "pivot"]) and ok
        if not ok:
            raise RuntimeError("Failed to reset the cartpole state")


class CartPoleDiscreteBalancing(_CartPole):
    force_mag = 20.0

    def _action_space(self):
        return _gym.spaces.Discrete(2)

    def _force(self, action) -> float:
        return self.force_mag if action == 1 else -self.force_mag

    def get_reward(self) -> float:
        reward = 0.0 if self.is_done() else 1.0
        if self._reward_cart_at_center:
            x, dx, _, _ = self.get_observation()
            reward = reward - 0.10 * np.abs(x) - 0.10 * np.abs(dx) - 10.0 * (x >= 0.9 * self.x_limit)
        return reward

    def _initial_state(self):
        x, dx, q, dq = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        return x, dx, q, dq


class CartPoleContinuousBalancing(_CartPole):
    max_force = 50.0

    def _action_space(self):
        return _gym.spaces.Box(low=np.array([-self.max_force]), high=np.array([self.max_force]),
                               dtype=np.float32)

    def _force(self, action) -> float:
        return action.tolist()[0]

    def get_reward(self) -> float:
        reward = 0.0 if self.is_done() else 1.0
        if self._reward_cart_at_center:
            x, dx, _, _ = self.get_observation()
            reward = reward - 0.10 * np.abs(x) - 0.10 * np.abs(dx) - 10.0 * (x >= self.x_limit)
        return reward

    def _initial_state(self):
        x, dx, q, dq = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        return x, dx, q, dq


class CartPoleContinuousSwingup(_CartPole):
    max_force = 200.0
    q_limit = np.deg2rad(5 * 360)

    def _action_space(self):
        return _gym.spaces.Box(low=np.array([-self.max_force]), high=np.array([self.max_force]),
                               dtype=np.float32)

    def _force(self, action) -> float:
        return action.tolist()[0]

    def get_reward(self) -> float:
        model = self.world.get_model(self.model_name)
        q = model.get_joint("pivot").position()
        x = model.get_joint("linear").position()
        dx = model.get_joint("linear").velocity()
        # upright pole -> 1, hanging pole -> 0; penalise cart speed and the rail ends
        return (np.cos(q) + 1) / 2 - 0.1 * (dx ** 2) - 10.0 * (x >= 0.8 * self.x_limit)

    def _initial_state(self):
        q = np.pi - np.deg2rad(self.np_random.uniform(low=-60, high=60))
        x, dx, dq = self.np_random.uniform(low=-0.05, high=0.05, size=(3,))
        return x, dx, q, dq
