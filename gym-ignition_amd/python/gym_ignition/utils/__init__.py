from . import logger, misc, scenario, typing  # noqa: F401
