from . import abc, gazebo_env_randomizer, physics  # noqa: F401
