from . import runtime, task  # noqa: F401
