from . import cartpole, panda, pendulum  # noqa: F401
