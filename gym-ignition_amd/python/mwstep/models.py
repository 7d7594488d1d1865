"""Model files shipped with the build (gym_ignition_models is not available
offline; see the provenance header of every file under gym-ignition_amd/models)."""

import os

MODELS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                          "models")

_FILES = {
    "cartpole": "cartpole.urdf",
    "pendulum": "pendulum.urdf",
    "panda": "panda.urdf",
    "ground_plane": "ground_plane.sdf",
}


def get_model_file(name: str) -> str:
    """Counterpart of ``gym_ignition_models.get_model_file``."""
    if name not in _FILES:
        raise ValueError(f"model {name!r} is not shipped; available: {sorted(_FILES)}")
    return os.path.join(MODELS_DIR, _FILES[name])


def get_robot_names():
    return sorted(_FILES)
