"""Model files shipped with the build (gym_ignition_models is not available
offline; see the provenance header of every file under gym-ignition_amd/models)."""

import os

MODELS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                          "models")

_FILES = {
    "cartpole": "cartpole.urdf",
    "pendulum": "pendulum.urdf",
    "panda": "panda.urdf",
    "cube": "cube.urdf",
    "quadruped": "quadruped.urdf",
    "humanoid32": "humanoid32.urdf",
    "ground_plane": "ground_plane.sdf",
}


def get_model_file(name: str) -> str:
    """Counterpart of ``gym_ignition_models.get_model_file``."""
    if name not in _FILES:
        raise ValueError(f"model {name!r} is not shipped; available: {sorted(_FILES)}")
    return os.path.join(MODELS_DIR, _FILES[name])


def get_robot_names():
    return sorted(_FILES)


# Panda JointController gains at 1 kHz, as the reference sets them
# (python/gym_ignition_environments/models/panda.py:48-58,
#  tests/test_scenario/test_pid_controllers.py:20-30): (P, I, D)
PANDA_PID_GAINS_1000HZ = {
    "panda_joint1": (50.0, 0.0, 20.0),
    "panda_joint2": (10000.0, 0.0, 500.0),
    "panda_joint3": (100.0, 0.0, 10.0),
    "panda_joint4": (1000.0, 0.0, 50.0),
    "panda_joint5": (100.0, 0.0, 10.0),
    "panda_joint6": (100.0, 0.0, 10.0),
    "panda_joint7": (10.0, 0.5, 0.1),
    "panda_finger_joint1": (100.0, 0.0, 50.0),
    "panda_finger_joint2": (100.0, 0.0, 50.0),
}
