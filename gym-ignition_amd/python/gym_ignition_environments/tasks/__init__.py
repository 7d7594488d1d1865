from . import (cartpole, cartpole_continuous_balancing, cartpole_continuous_swingup,  # noqa: F401
               cartpole_discrete_balancing, pendulum, pendulum_swingup)
