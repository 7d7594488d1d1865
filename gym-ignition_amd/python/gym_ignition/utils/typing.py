"""Type aliases of the gym_ignition API (reference: python/gym_ignition/utils/typing.py)."""

from typing import Dict, List, NewType, Tuple, Union

import numpy as np

from mwstep import gym_module

_gym = gym_module()

Done = NewType("Done", bool)
Info = NewType("Info", Dict)
Reward = NewType("Reward", float)
Observation = NewType("Observation", np.ndarray)
Action = NewType("Action", Union[np.ndarray, np.number])
SeedList = NewType("SeedList", List[int])
State = NewType("State", Tuple[Observation, Reward, Done, Info])
ActionSpace = NewType("ActionSpace", _gym.spaces.Space)
ObservationSpace = NewType("ObservationSpace", _gym.spaces.Space)
