from mwstep import get_model_file

from gym_ignition.scenario import model_with_file, model_wrapper

from ._insert import insert


class Pendulum(model_wrapper.ModelWrapper, model_with_file.ModelWithFile):
    """The shipped pendulum (base `support`, joint `pivot`) inserted into a world."""

    def __init__(self, world, position=(0.0, 0.0, 0.0), orientation=(1.0, 0, 0, 0),
                 model_file: str = None):
        model = insert(world, "pendulum", model_file or self.get_model_file(), position, orientation)
        super().__init__(model=model)

    @classmethod
    def get_model_file(cls) -> str:
        return get_model_file("pendulum")
