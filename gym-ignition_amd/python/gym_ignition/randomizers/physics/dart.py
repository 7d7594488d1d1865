from scenario import gazebo as scenario_gazebo

from ..abc import PhysicsRandomizer


class DART(PhysicsRandomizer):
    """No physics randomization; the engine name routes to the HIP stepper."""

    def __init__(self):
        super().__init__(randomize_after_rollouts_num=0)

    def randomize_physics(self, task, **kwargs) -> None:
        return None

    def get_engine(self):
        return scenario_gazebo.PhysicsEngine_dart
