# module path kept for gym entry points / imports of the reference layout
from .pendulum import PendulumSwingUp  # noqa: F401
