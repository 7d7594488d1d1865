import abc


class ModelWithFile(abc.ABC):
    """Models that know the file (URDF/SDF) they are built from."""

    @classmethod
    @abc.abstractmethod
    def get_model_file(cls) -> str:
        ...
