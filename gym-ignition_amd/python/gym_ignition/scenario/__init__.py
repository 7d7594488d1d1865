from . import model_wrapper, model_with_file  # noqa: F401
