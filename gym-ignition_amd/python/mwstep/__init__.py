"""mwstep -- MI355X many-worlds articulated-body stepper (host side).

Layers:
  native   ctypes binding of the C ABI in include/mwstep.h (libmwstep.so)
  sim      Simulator: N worlds of one model, ScenarI/O-style accessors
  vecenv   VecEnv: device-resident batched gym tasks (torch tensors)
  models   model files shipped with the build
The ScenarI/O / gym_ignition mirrors live in the sibling packages
``scenario``, ``gym_ignition`` and ``gym_ignition_environments``.
"""

from .models import get_model_file  # noqa: F401

__version__ = "0.1.0"


def gym_module():
    """The real ``gym`` if importable, else the bundled restatement."""
    try:
        import gym  # type: ignore
        return gym
    except ImportError:
        from . import gymcompat
        return gymcompat


def __getattr__(name):
    if name == "Simulator":
        from .sim import Simulator
        return Simulator
    if name == "VecEnv":
        from .vecenv import VecEnv
        return VecEnv
    raise AttributeError(name)
