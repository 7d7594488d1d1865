from . import abc, gazebo_env_randomizer, model, physics  # noqa: F401
