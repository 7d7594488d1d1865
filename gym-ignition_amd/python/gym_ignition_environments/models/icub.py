import abc
from typing import List

from mwstep import get_model_file
from mwstep.models import ICUB_INITIAL_POSITIONS

from gym_ignition.scenario import model_with_file, model_wrapper

from ._insert import insert


class ICubGazeboABC(model_wrapper.ModelWrapper, abc.ABC):
    """The reference's iCub wrapper (python/gym_ignition_environments/models/
    icub.py:12-77): inserts the model under a unique "icub" name at the given
    pose and resets its 32 joints to the wrapper's initial posture by name
    through Model::resetJointPositions (here the ScenarI/O mirror over the
    C-ABI).  The shipped model (models/icub.urdf, make_icub.py) has the
    reference's joint names, DOFS / NUM_JOINTS / NUM_LINKS."""

    DOFS = 32
    NUM_LINKS = 39
    NUM_JOINTS = 32

    initial_positions = dict(ICUB_INITIAL_POSITIONS)

    def __init__(self, world, position: List[float], orientation: List[float], model_file: str = None):
        model = insert(world, "icub", model_file or self.get_model_file(), position, orientation)
        super().__init__(model=model)
        q0 = list(self.initial_positions.values())
        joint_names = list(self.initial_positions.keys())
        assert self.dofs() == len(q0) == len(joint_names)
        ok_q0 = self.to_gazebo().reset_joint_positions(q0, joint_names)
        assert ok_q0, "Failed to set initial position"


class ICubGazebo(ICubGazeboABC, model_with_file.ModelWithFile):
    """icub.py:80-99: inserted at (0, 0, 0.572), wxyz (0, 0, 0, 1)."""

    def __init__(self, world, position: List[float] = (0.0, 0.0, 0.572),
                 orientation: List[float] = (0, 0, 0, 1.0), model_file: str = None):
        super().__init__(world=world, position=position, orientation=orientation, model_file=model_file)

    @classmethod
    def get_model_file(cls) -> str:
        # the reference asks gym_ignition_models for "iCubGazeboV2_5" (absent
        # offline): the shipped iCub-class stand-in
        return get_model_file("icub")


class ICubGazeboSimpleCollisions(ICubGazeboABC):
    """icub.py:102-120: the same wrapper for the simple-collision model; the
    shipped model's collisions are already one box per foot."""

    def __init__(self, world, position: List[float] = (0.0, 0.0, 0.572),
                 orientation: List[float] = (0, 0, 0, 1.0), model_file: str = None):
        super().__init__(world=world, position=position, orientation=orientation, model_file=model_file)

    @classmethod
    def get_model_file(cls) -> str:
        return get_model_file("icub")
