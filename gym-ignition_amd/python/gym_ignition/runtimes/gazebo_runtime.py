"""GazeboRuntime: gym.Env over one simulator + one world, stepping on MI355X.

Public surface and behaviour of the reference runtime
(``/root/reference/python/gym_ignition/runtimes/gazebo_runtime.py:13-267``):
the simulator is created lazily with ``steps_per_run = physics_rate /
agent_rate``, a world (with a ground plane when no SDF world is given) is
inserted and initialised, the physics engine is enabled, and ``step`` runs
set_action -> run() -> observation / reward / done / info.
"""

import numpy as np

from mwstep import get_model_file, gym_module
from scenario import gazebo as scenario_gazebo

from ..base import runtime as _runtime
from ..base import task as _task
from ..utils import logger
from ..utils import scenario as scenario_utils

_gym = gym_module()


class GazeboRuntime(_runtime.Runtime):
    metadata = {"render.modes": ["human"]}

    def __init__(self, task_cls: type, agent_rate: float, physics_rate: float,
                 real_time_factor: float, physics_engine=scenario_gazebo.PhysicsEngine_dart,
                 world: str = None, **kwargs):
        self._gazebo = None
        self._world = None
        self._physics_rate = physics_rate
        self._real_time_factor = real_time_factor
        self._physics_engine = physics_engine
        self._world_sdf = world
        self._world_name = None

        task = task_cls(agent_rate=agent_rate, **kwargs)
        if not isinstance(task, _task.Task):
            raise RuntimeError("The task is not compatible with the runtime")
        super().__init__(task=task, agent_rate=agent_rate)

        _ = self.gazebo  # builds simulator + world
        self.action_space, self.observation_space = self.task.create_spaces()
        self.task.action_space = self.action_space
        self.task.observation_space = self.observation_space
        self.seed()

    # -- Runtime
    def timestamp(self) -> float:
        return self.world.time()

    # -- gym.Env
    def step(self, action):
        if not self.action_space.contains(action):
            logger.warn("The action does not belong to the action space")
        self.task.set_action(action)
        if not self.gazebo.run():
            raise AssertionError("Failed to step gazebo")
        obs = self.task.get_observation()
        assert isinstance(obs, np.ndarray)
        if not self.observation_space.contains(obs):
            logger.warn("The observation does not belong to the observation space")
        reward = self.task.get_reward()
        assert isinstance(reward, float), "Failed to get the reward"
        done = self.task.is_done()
        return obs, reward, done, self.task.get_info()

    def reset(self):
        self.task.reset_task()
        if not self.gazebo.run(paused=True):
            raise RuntimeError("Failed to run Gazebo")
        obs = self.task.get_observation()
        assert isinstance(obs, np.ndarray)
        if not self.observation_space.contains(obs):
            logger.warn("The observation does not belong to the observation space")
        return obs

    def render(self, mode: str = "human", **kwargs) -> None:
        if mode != "human":
            raise ValueError(f"Render mode '{mode}' not supported")
        if not self.gazebo.gui():
            raise RuntimeError("Failed to render the environment")

    def close(self) -> None:
        if not self.gazebo.close():
            raise RuntimeError("Failed to close Gazebo")

    def seed(self, seed: int = None):
        if not self.task.has_world():
            raise RuntimeError("The world has never been created")
        return self.task.seed_task(seed)

    # -- lazily built simulator and world
    @property
    def gazebo(self) -> scenario_gazebo.GazeboSimulator:
        if self._gazebo is not None:
            assert self._gazebo.initialized()
            return self._gazebo
        ratio = self._physics_rate / self.agent_rate
        if ratio != int(ratio):
            logger.warn(f"Rounding the number of iterations to {int(ratio)} from the nominal {ratio}")
        self._gazebo = scenario_gazebo.GazeboSimulator(1.0 / self._physics_rate,
                                                       self._real_time_factor, int(ratio))
        _ = self.world
        assert self._gazebo.initialized()
        return self._gazebo

    @property
    def world(self) -> scenario_gazebo.World:
        if self._world is not None:
            return self._world
        if self._gazebo is None:
            raise RuntimeError("Gazebo has not yet been created")
        if self._gazebo.initialized():
            raise RuntimeError("Gazebo was already initialized, cannot insert world")
        if self._world_sdf is None:
            self._world_sdf = ""
            self._world_name = scenario_utils.get_unique_world_name("default")
        else:
            base = scenario_gazebo.get_world_name_from_sdf(self._world_sdf)
            self._world_name = scenario_utils.get_unique_world_name(base)
        if not self._gazebo.insert_world_from_sdf(self._world_sdf, self._world_name):
            raise RuntimeError("Failed to load SDF world")
        if not self._gazebo.initialize() or not self._gazebo.initialized():
            raise RuntimeError("Failed to initialize Gazebo")
        world = self._gazebo.get_world(self._world_name)
        if self._world_sdf == "" and not world.insert_model(get_model_file("ground_plane")):
            raise RuntimeError("Failed to insert the ground plane")
        self.task.world = world
        world.set_physics_engine(engine=self._physics_engine)
        self._world = world
        return world
