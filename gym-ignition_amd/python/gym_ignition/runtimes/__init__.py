from . import gazebo_runtime  # noqa: F401
