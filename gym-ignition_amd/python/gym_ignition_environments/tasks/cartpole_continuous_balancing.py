# module path kept for gym entry points / imports of the reference layout
from .cartpole import CartPoleContinuousBalancing  # noqa: F401
