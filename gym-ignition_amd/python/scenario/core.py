"""``scenario.core`` names (enums and value types) of the ScenarI/O API.

Numbering and semantics follow
``/root/reference/cpp/scenario/core/include/scenario/core/Joint.h:25-75`` and
``utils.h`` (Pose, PID, Limit) as exposed through SWIG with snake_case names
(``bindings/core/core.i:70``).
"""

from __future__ import annotations

import math
from typing import Sequence

# JointType (Joint.h:25-31)
JointType_invalid = 0
JointType_fixed = 1
JointType_revolute = 2
JointType_prismatic = 3
JointType_ball = 4

# JointControlMode (Joint.h:37-75)
JointControlMode_invalid = 0
JointControlMode_idle = 1
JointControlMode_force = 2
JointControlMode_velocity = 3
JointControlMode_velocity_follower_dart = 4
JointControlMode_position = 5
JointControlMode_position_interpolated = 6


class Pose:
    """Position [x, y, z] and orientation quaternion [w, x, y, z]."""

    def __init__(self, position: Sequence[float] = (0.0, 0.0, 0.0),
                 orientation: Sequence[float] = (1.0, 0.0, 0.0, 0.0)):
        if len(position) != 3 or len(orientation) != 4:
            raise ValueError("Pose needs 3 position and 4 (wxyz) orientation elements")
        self.position = tuple(float(v) for v in position)
        self.orientation = tuple(float(v) for v in orientation)

    @staticmethod
    def identity() -> "Pose":
        return Pose()

    def __eq__(self, other) -> bool:
        return isinstance(other, Pose) and self.position == other.position and \
            self.orientation == other.orientation

    def __repr__(self):
        return f"Pose(position={list(self.position)}, orientation={list(self.orientation)})"


class Limit:
    def __init__(self, min: float = -math.inf, max: float = math.inf):  # noqa: A002
        self.min = float(min)
        self.max = float(max)

    def __repr__(self):
        return f"Limit(min={self.min}, max={self.max})"


class PID:
    """PID gains and limits (ignition::math::PID parameters)."""

    def __init__(self, p: float = 0.0, i: float = 0.0, d: float = 0.0, i_max: float = -1.0,
                 i_min: float = 0.0, cmd_max: float = -1.0, cmd_min: float = 0.0,
                 cmd_offset: float = 0.0):
        self.p, self.i, self.d = float(p), float(i), float(d)
        self.i_max, self.i_min = float(i_max), float(i_min)
        self.cmd_max, self.cmd_min = float(cmd_max), float(cmd_min)
        self.cmd_offset = float(cmd_offset)

    def __repr__(self):
        return f"PID(p={self.p}, i={self.i}, d={self.d})"


# Default PID of every joint (Joint.cpp:63)
DEFAULT_PID = PID(1.0, 0.1, 0.01, -1.0, 0.0, -1.0, 0.0, 0.0)


def __getattr__(name):
    # The abstract core interfaces are the gazebo classes themselves in this
    # build; `to_gazebo()` on any of them returns the same object.
    if name in ("World", "Model", "Joint"):
        from . import gazebo
        return getattr(gazebo, name)
    raise AttributeError(name)
