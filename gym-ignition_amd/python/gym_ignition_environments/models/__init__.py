from . import cartpole, pendulum  # noqa: F401
