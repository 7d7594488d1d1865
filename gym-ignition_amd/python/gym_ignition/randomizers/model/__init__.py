from . import sdf  # noqa: F401
