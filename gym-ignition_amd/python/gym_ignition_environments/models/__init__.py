from . import cartpole, icub, panda, pendulum  # noqa: F401
