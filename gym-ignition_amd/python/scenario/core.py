"""``scenario.core`` names (enums and value types) of the ScenarI/O API.

Numbering and semantics follow
``/root/reference/cpp/scenario/core/include/scenario/core/Joint.h:25-75`` and
``utils.h`` (Pose, PID, Limit) as exposed through SWIG with snake_case names
(``bindings/core/core.i:70``).
"""

from __future__ import annotations

import math
from typing import Sequence

import numpy as np

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


class JointLimit:
    """core::JointLimit (utils.h): per-DoF min / max vectors."""

    def __init__(self, min=(), max=()):  # noqa: A002
        self.min = [float(v) for v in min]
        self.max = [float(v) for v in max]

    def __repr__(self):
        return f"JointLimit(min={self.min}, max={self.max})"


class PID:
    """scenario::core::PID (cpp/scenario/core/include/scenario/core/Joint.h:505-523):
    gains plus command / integral limits, with the SWIG binding's undercase
    member names (bindings/core/core.i:69-70).  Defaults leave every limit open."""

    _LOWEST = -float(np.finfo(np.float64).max)
    _MAX = float(np.finfo(np.float64).max)

    def __init__(self, p: float = 0.0, i: float = 0.0, d: float = 0.0):
        self.p, self.i, self.d = float(p), float(i), float(d)
        self.cmd_min, self.cmd_max, self.cmd_offset = self._LOWEST, self._MAX, 0.0
        self.i_min, self.i_max = self._LOWEST, self._MAX

    def to_list(self):
        """{p, i, d, cmd_min, cmd_max, cmd_offset, i_min, i_max} (mwstep.h order)."""
        return [self.p, self.i, self.d, self.cmd_min, self.cmd_max, self.cmd_offset, self.i_min, self.i_max]

    @classmethod
    def from_list(cls, v) -> "PID":
        pid = cls(v[0], v[1], v[2])
        pid.cmd_min, pid.cmd_max, pid.cmd_offset, pid.i_min, pid.i_max = (float(x) for x in v[3:8])
        return pid

    def __repr__(self):
        return f"PID(p={self.p}, i={self.i}, d={self.d})"


# Default PID of every joint: ignition::math::PID(1, 0.1, 0.01, -1, 0, -1, 0, 0)
# (Joint.cpp:63) as returned by Joint::pid() (fromIgnitionPID)
DEFAULT_PID = PID.from_list([1.0, 0.1, 0.01, 0.0, -1.0, 0.0, 0.0, -1.0])


class ContactPoint:
    """scenario::core::ContactPoint (Link.h / utils.h): world-frame point,
    normal, force and torque on the body, penetration depth."""

    def __init__(self, position=(0.0, 0.0, 0.0), normal=(0.0, 0.0, 0.0), force=(0.0, 0.0, 0.0),
                 torque=(0.0, 0.0, 0.0), depth: float = 0.0):
        self.position = [float(x) for x in position]
        self.normal = [float(x) for x in normal]
        self.force = [float(x) for x in force]
        self.torque = [float(x) for x in torque]
        self.depth = float(depth)


class Contact:
    """scenario::core::Contact: the points between two bodies (scoped link names)."""

    def __init__(self, body_a: str = "", body_b: str = "", points=()):
        self.body_a = body_a
        self.body_b = body_b
        self.points = list(points)


def __getattr__(name):
    # The abstract core interfaces are the gazebo classes themselves in this
    # build; `to_gazebo()` on any of them returns the same object.
    if name in ("World", "Model", "Joint"):
        from . import gazebo
        return getattr(gazebo, name)
    raise AttributeError(name)
