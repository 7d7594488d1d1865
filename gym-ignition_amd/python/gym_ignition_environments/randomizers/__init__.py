from . import cartpole, cartpole_no_rand, pendulum_no_rand  # noqa: F401
