# module path kept for gym entry points / imports of the reference layout
from .cartpole import CartPoleDiscreteBalancing  # noqa: F401
