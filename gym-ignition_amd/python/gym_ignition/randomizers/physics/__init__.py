from . import dart  # noqa: F401
