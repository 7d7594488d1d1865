"""Logging helpers (reference: python/gym_ignition/utils/logger.py).  Messages go
through gym's logger; ``set_level`` also sets the ScenarI/O verbosity."""

import contextlib

from mwstep import gym_module

_gym = gym_module()


def debug(msg: str) -> None:
    _gym.logger.debug(msg)


def info(msg: str) -> None:
    _gym.logger.info(msg)


def warn(msg: str) -> None:
    _gym.logger.warn(msg)


def error(msg: str) -> None:
    _gym.logger.error(msg)


def set_level(level: int) -> None:
    from scenario import gazebo
    _gym.logger.set_level(level)
    table = {_gym.logger.DEBUG: gazebo.Verbosity_debug, _gym.logger.INFO: gazebo.Verbosity_info,
             _gym.logger.WARN: gazebo.Verbosity_warning, _gym.logger.ERROR: gazebo.Verbosity_error}
    gazebo.set_verbosity(table.get(level, gazebo.Verbosity_suppress_all))


@contextlib.contextmanager
def gym_verbosity(level: int):
    old = _gym.logger.level if hasattr(_gym.logger, "level") else None
    _gym.logger.set_level(level)
    try:
        yield
    finally:
        if old is not None:
            _gym.logger.set_level(old)
