from . import logger, scenario, typing  # noqa: F401
