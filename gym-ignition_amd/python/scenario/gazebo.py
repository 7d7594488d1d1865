"""``scenario.gazebo`` -- ScenarI/O simulator API backed by the HIP stepper.

Same names and return conventions as the reference's SWIG module
(``/root/reference/bindings/gazebo/gazebo.i``): lifecycle calls and setters
return ``bool`` and log the reason of a failure, getters raise
``RuntimeError`` (the SWIG mapping of ``scenario::gazebo::exceptions``).

Where the reference keeps entity state in one ign-gazebo ECM per world and
steps each with DART on the CPU, a ``GazeboSimulator`` here owns one native
scene (``mwstep.scene.Scene``, include/mwscene.h) whose worlds are the
simulator's worlds: every model of every world lives in HBM, models of one
world collide with each other and with the world's ground plane, and one
``run()`` steps all worlds in one kernel launch (GazeboSimulator.cpp:435-488,
Physics.cpp:1832-1834).  A model inserted with the same name, file and pose
into several worlds shares one model slot of the scene (its joint parameters,
PID gains and controller period are the slot's); state, commands, targets,
control modes, resets and wrenches are per world.  Component semantics that
callers can observe are kept:

  * resets and commands take effect on the next ``run()`` (paused or not),
    and getters return the state refreshed by the last run
    (``Physics.cpp:1330-1440, 2226-2345``);
  * a joint force target is consumed by one physics step and reads back as
    zero after the run (``Physics.cpp:2250-2254``);
  * ``World.time()`` is the simulated time written by the physics system, so it
    stays 0 until ``set_physics_engine`` and then follows the server iterations
    (``Physics.cpp:656-666``; ``tests/test_scenario/test_world.py:149-219``).
"""

from __future__ import annotations

import collections
import math
import os
import re
import sys
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import core

PhysicsEngine_dart = 0

Verbosity_suppress_all, Verbosity_error, Verbosity_warning = 0, 1, 2
Verbosity_info, Verbosity_debug = 3, 4
_verbosity = Verbosity_warning


def set_verbosity(level: int = Verbosity_warning) -> None:
    global _verbosity
    _verbosity = int(level)


def _err(msg: str) -> None:
    if _verbosity >= Verbosity_error:
        print(f"[ERROR] {msg}", file=sys.stderr)


def _warn(msg: str) -> None:
    if _verbosity >= Verbosity_warning:
        print(f"[WARNING] {msg}", file=sys.stderr)


def _device() -> int:
    return int(os.environ.get("MWSTEP_DEVICE", "0"))


# slot-wide components of a scene model (Model._comp / _set_component): keys
# ("pid", dof), ("param", dof, which), ("period",)
def _read_component(view, key):
    if key[0] == "pid":
        return tuple(float(v) for v in view.pid(key[1]))
    if key[0] == "param":
        return float(view.joint_param(key[1], key[2]))
    return float(view.controller_period())


def _write_component(view, key, value) -> None:
    if key[0] == "pid":
        view.set_pid(key[1], list(value))
    elif key[0] == "param":
        view.set_joint_param(key[1], key[2], value)
    else:
        view.set_controller_period(value)


# ---------------------------------------------------------------- SDF helpers
_EMPTY_WORLD = """<?xml version="1.0" ?>
<sdf version="1.6">
    <world name="default">
        <physics default="true" type="dart">
        </physics>
    </world>
</sdf>"""


def get_empty_world() -> str:
    """SDF of an empty world named "default" (utils.cpp:171-196)."""
    return _EMPTY_WORLD


_MESH_URDF = re.compile(r'(<mesh\b[^>]*?\bfilename\s*=\s*")([^"]+)(")')
_MESH_SDF = re.compile(r'(<mesh\b[^>]*>(?:(?!</mesh>).)*?<uri>\s*)([^<]+?)(\s*</uri>)', re.S)


def _absolute_mesh_uris(text: str, base_dir: str) -> str:
    """Relative mesh URIs of a model read from a file resolve against the
    file's directory, as the reference's asFullPath(uri, sdf FilePath) does
    (Physics.cpp:905); the model compiler gets the text with absolute paths."""
    def fix(m):
        uri = m.group(2).strip()
        if uri.startswith(("/", "model://", "package://", "file://")):
            return m.group(0)
        return m.group(1) + os.path.join(base_dir, uri) + m.group(3)
    return _MESH_SDF.sub(fix, _MESH_URDF.sub(fix, text))


def _read(path_or_string: str) -> str:
    if path_or_string.lstrip().startswith("<"):
        return path_or_string
    with open(path_or_string) as f:
        return f.read()


def _sdf_model_pose(root) -> core.Pose:
    """<model><pose>x y z roll pitch yaw</pose> as a Pose (wxyz)."""
    pe = root.find("model/pose")
    v = [float(x) for x in pe.text.split()] if pe is not None and pe.text and pe.text.strip() else [0.0] * 6
    cr, sr = math.cos(v[3] / 2), math.sin(v[3] / 2)
    cp, sp = math.cos(v[4] / 2), math.sin(v[4] / 2)
    cy, sy = math.cos(v[5] / 2), math.sin(v[5] / 2)
    q = [cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
         cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy]
    return core.Pose(v[:3], q)


def get_world_name_from_sdf(sdf: str, world_index: int = 0) -> str:
    root = ET.fromstring(_read(sdf).strip())
    worlds = root.findall("world")
    return worlds[world_index].get("name", "") if world_index < len(worlds) else ""


def get_model_name_from_sdf(sdf: str, model_index: int = 0) -> str:
    root = ET.fromstring(_read(sdf).strip())
    if root.tag == "robot":
        return root.get("name", "")
    models = root.findall("model")
    return models[model_index].get("name", "") if model_index < len(models) else ""


# ---------------------------------------------------------------------- Joint
class Joint:
    """One degree of freedom of an articulated model (all joints are 1-dof)."""

    def __init__(self, model: "Model", dof: int, name: str):
        self._model = model
        self._dof = dof
        self._name = name

    # -- identity
    def to_gazebo(self) -> "Joint":
        return self

    def valid(self) -> bool:
        return self._model.valid()

    def name(self, scoped: bool = False) -> str:
        return f"{self._model.name()}::{self._name}" if scoped else self._name

    def type(self) -> int:
        return self._model._sim.joint_type(self._dof)

    def dofs(self) -> int:
        return 1

    def _check_dof(self, dof: int) -> None:
        if dof != 0:
            raise RuntimeError(f"DOF mismatch: joint '{self._name}' has 1 DoF, requested #{dof}")

    # -- state (refreshed by the last run)
    def _read(self, what: str) -> float:
        return float(self._model._get(what, [self._dof])[0])

    def position(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self._read("q")

    def velocity(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self._read("qd")

    def acceleration(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self._read("qdd")

    def generalized_force(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self._read("force")

    def joint_position(self) -> List[float]:
        return [self.position()]

    def joint_velocity(self) -> List[float]:
        return [self.velocity()]

    def joint_acceleration(self) -> List[float]:
        return [self.acceleration()]

    def joint_generalized_force(self) -> List[float]:
        return [self.generalized_force()]

    # -- control
    def control_mode(self) -> int:
        return self._model._sim.control_mode(0, self._dof)

    def set_control_mode(self, mode: int) -> bool:
        return self._model.set_joint_control_mode(mode, [self._name])

    def pid(self) -> core.PID:
        # Joint::pid (Joint.cpp:470-476)
        return core.PID.from_list(self._model._comp(("pid", self._dof)))

    def set_pid(self, pid: core.PID) -> bool:
        # Joint::setPID (Joint.cpp:479-525): output limits looser than the
        # effort limit are replaced by +-effort (what the scene stores too)
        try:
            g = [float(v) for v in pid.to_list()]
            from mwstep import native as N
            maxf = self._model._comp(("param", self._dof, N.PARAM_MAX_GENERALIZED_FORCE))
            if g[3] < -maxf or g[4] > maxf:
                g[3], g[4] = -maxf, maxf
            self._model._set_component(("pid", self._dof), tuple(g))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def set_generalized_force_target(self, force: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._model.set_joint_generalized_force_targets([force], [self._name])

    def generalized_force_target(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return float(self._model._get("force_target", [self._dof])[0])

    def set_velocity_target(self, velocity: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._model.set_joint_velocity_targets([velocity], [self._name])

    def velocity_target(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return float(self._model._get("velocity_target", [self._dof])[0])

    def set_position_target(self, position: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._model.set_joint_position_targets([position], [self._name])

    def position_target(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return float(self._model._get("position_target", [self._dof])[0])

    # -- resets (applied by the next run)
    def reset_position(self, position: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._model.reset_joint_positions([position], [self._name])

    def reset_velocity(self, velocity: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._model.reset_joint_velocities([velocity], [self._name])

    def reset(self, position: float = 0.0, velocity: float = 0.0, dof: int = 0) -> bool:
        return self.reset_position(position, dof) and self.reset_velocity(velocity, dof)

    # -- parameters (only while the model was just created)
    def _set_param(self, which: int, value: float) -> bool:
        try:
            self._model._set_component(("param", self._dof, which), float(value))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def _param(self, which: int) -> float:
        return self._model._comp(("param", self._dof, which))

    def set_coulomb_friction(self, value: float) -> bool:
        from mwstep import native as N
        return self._set_param(N.PARAM_COULOMB_FRICTION, value)

    def set_viscous_friction(self, value: float) -> bool:
        from mwstep import native as N
        return self._set_param(N.PARAM_VISCOUS_FRICTION, value)

    def coulomb_friction(self) -> float:
        from mwstep import native as N
        return self._param(N.PARAM_COULOMB_FRICTION)

    def viscous_friction(self) -> float:
        from mwstep import native as N
        return self._param(N.PARAM_VISCOUS_FRICTION)

    def max_generalized_force(self, dof: int = 0) -> float:
        from mwstep import native as N
        self._check_dof(dof)
        v = self._param(N.PARAM_MAX_GENERALIZED_FORCE)
        return math.inf if v >= 1e299 else v

    def set_max_generalized_force(self, max_force: float, dof: int = 0) -> bool:
        from mwstep import native as N
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        return self._set_param(N.PARAM_MAX_GENERALIZED_FORCE, max_force)

    # acceleration targets: stored for controllers, no effect on the physics
    # (JointAccelerationTarget, Joint.cpp:747-845)
    def set_acceleration_target(self, acceleration: float, dof: int = 0) -> bool:
        if dof != 0:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        self._model._acc_targets[self._name] = float(acceleration)
        return True

    def acceleration_target(self, dof: int = 0) -> float:
        self._check_dof(dof)
        if self._name not in self._model._acc_targets:
            raise RuntimeError(f"Joint '{self._name}' has no acceleration target")
        return self._model._acc_targets[self._name]

    # vectorised (multi-DoF) forms of the per-DoF accessors (core/Joint.h)
    def joint_position_target(self) -> List[float]:
        return [self.position_target()]

    def joint_velocity_target(self) -> List[float]:
        return [self.velocity_target()]

    def joint_acceleration_target(self) -> List[float]:
        return [self.acceleration_target()]

    def joint_generalized_force_target(self) -> List[float]:
        return [self.generalized_force_target()]

    def joint_max_generalized_force(self) -> List[float]:
        return [self.max_generalized_force()]

    def set_joint_position_target(self, target: Sequence[float]) -> bool:
        return len(target) == 1 and self.set_position_target(target[0])

    def set_joint_velocity_target(self, target: Sequence[float]) -> bool:
        return len(target) == 1 and self.set_velocity_target(target[0])

    def set_joint_acceleration_target(self, target: Sequence[float]) -> bool:
        return len(target) == 1 and self.set_acceleration_target(target[0])

    def set_joint_generalized_force_target(self, target: Sequence[float]) -> bool:
        return len(target) == 1 and self.set_generalized_force_target(target[0])

    def set_joint_max_generalized_force(self, max_force: Sequence[float]) -> bool:
        return len(max_force) == 1 and self.set_max_generalized_force(max_force[0])

    def position_limit(self, dof: int = 0) -> core.Limit:
        from mwstep import native as N
        self._check_dof(dof)
        lo = self._param(N.PARAM_POSITION_LIMIT_MIN)
        hi = self._param(N.PARAM_POSITION_LIMIT_MAX)
        return core.Limit(-math.inf if lo <= -1e299 else lo, math.inf if hi >= 1e299 else hi)

    def joint_position_limit(self) -> core.Limit:
        return self.position_limit()


# ------------------------------------------------------------------ BallJoint
# A ball joint (core::JointType::Ball, 3 dofs, Joint.cpp:318-331) runs in
# DART's BallJoint coordinates natively (csrc/chain_dyn.hpp ball_part, oracle.c
# ball_part): its three internal dofs `<name>#x/#y/#z` ARE the rotation vector
# of the joint rotation (positions), the child's angular velocity in the child
# frame (velocities, accelerations) and the child-frame torque (forces); the
# kernels integrate the positions on SO(3), R <- R exp(dt w).  No angle
# parameterisation, so no gimbal singularity.
def rotvec_from_R(R) -> np.ndarray:
    """log map of SO(3) (the rotation vector, DART BallJoint positions)"""
    c = max(-1.0, min(1.0, (np.trace(R) - 1.0) / 2.0))
    th = math.acos(c)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    if th < 1e-7:
        return 0.5 * w
    if math.pi - th < 1e-6:
        # near pi: the axis from the symmetric part
        A = (R + np.eye(3)) / 2.0
        k = int(np.argmax(np.diag(A)))
        ax = A[:, k] / math.sqrt(max(A[k, k], 1e-300))
        return th * ax / np.linalg.norm(ax)
    return th / (2.0 * math.sin(th)) * w


def R_from_rotvec(r) -> np.ndarray:
    r = np.asarray(r, dtype=float)
    th = float(np.linalg.norm(r))
    if th < 1e-12:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


class BallJoint(Joint):
    """A 3-dof ball joint: its three internal dofs in DART's coordinates."""

    def __init__(self, model: "Model", dof: int, name: str):
        super().__init__(model, dof, name)
        self._idx = [dof, dof + 1, dof + 2]
        self._names = [f"{name}#x", f"{name}#y", f"{name}#z"]

    def type(self) -> int:
        return core.JointType_ball

    def dofs(self) -> int:
        return 3

    def _check_dof(self, dof: int) -> None:
        if not 0 <= dof < 3:
            raise RuntimeError(f"DOF mismatch: joint '{self._name}' has 3 DoFs, requested #{dof}")

    def _vals(self, what: str) -> List[float]:
        return np.asarray(self._model._get(what, self._idx), dtype=float).tolist()

    # -- state in DART's BallJoint coordinates
    def joint_position(self) -> List[float]:
        return self._vals("q")

    def joint_velocity(self) -> List[float]:
        return self._vals("qd")

    def joint_acceleration(self) -> List[float]:
        return self._vals("qdd")

    def joint_generalized_force(self) -> List[float]:
        return self._vals("force")

    def joint_generalized_force_target(self) -> List[float]:
        return self._vals("force_target")

    def position(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self.joint_position()[dof]

    def velocity(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self.joint_velocity()[dof]

    def acceleration(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self.joint_acceleration()[dof]

    def generalized_force(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self.joint_generalized_force()[dof]

    def generalized_force_target(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return self.joint_generalized_force_target()[dof]

    def _to_internal(self, what: str, v) -> np.ndarray:
        if what not in ("reset_q", "reset_qd", "force_target"):
            raise RuntimeError(f"Joint '{self._name}' (ball) does not support {what}")
        v = np.asarray(v, dtype=float)
        if what == "reset_q" and float(np.linalg.norm(v)) > math.pi:
            # DART keeps the rotation vector's angle in [0, pi]
            v = rotvec_from_R(R_from_rotvec(v))
        return v

    def set_joint_generalized_force_target(self, target: Sequence[float]) -> bool:
        return len(target) == 3 and self._model.set_joint_generalized_force_targets(list(target), [self._name])

    def set_generalized_force_target(self, force: float, dof: int = 0) -> bool:
        if not 0 <= dof < 3:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        t = self.joint_generalized_force_target()
        t[dof] = float(force)
        return self.set_joint_generalized_force_target(t)

    def reset_joint_position(self, position: Sequence[float]) -> bool:
        return len(position) == 3 and self._model.reset_joint_positions(list(position), [self._name])

    def reset_joint_velocity(self, velocity: Sequence[float]) -> bool:
        return len(velocity) == 3 and self._model.reset_joint_velocities(list(velocity), [self._name])

    def reset_position(self, position: float, dof: int = 0) -> bool:
        if not 0 <= dof < 3:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        p = self.joint_position()
        p[dof] = float(position)
        return self.reset_joint_position(p)

    def reset_velocity(self, velocity: float, dof: int = 0) -> bool:
        if not 0 <= dof < 3:
            _err(f"Joint '{self._name}' does not have DoF#{dof}")
            return False
        v = self.joint_velocity()
        v[dof] = float(velocity)
        return self.reset_joint_velocity(v)

    def reset(self, position: float = 0.0, velocity: float = 0.0, dof: int = 0) -> bool:
        return self.reset_position(position, dof) and self.reset_velocity(velocity, dof)

    # -- JointController and limits: not defined for ball joints
    # (JointController.cpp:323-327 skips them; Joint.cpp:876-900 warns)
    def set_control_mode(self, mode: int) -> bool:
        if mode not in (core.JointControlMode_force, core.JointControlMode_idle):
            _err(f"Type of joint '{self._name}' not supported by the JointController")
            return False
        return self._model.set_joint_control_mode(mode, [self._name])

    def control_mode(self) -> int:
        return self._model._sim.control_mode(0, self._dof)

    def _unsupported(self, what: str) -> bool:
        _err(f"Joint '{self._name}' (ball) has no {what}")
        return False

    def set_position_target(self, position: float, dof: int = 0) -> bool:
        return self._unsupported("position target")

    def set_velocity_target(self, velocity: float, dof: int = 0) -> bool:
        return self._unsupported("velocity target")

    def set_joint_position_target(self, target: Sequence[float]) -> bool:
        return self._unsupported("position target")

    def set_joint_velocity_target(self, target: Sequence[float]) -> bool:
        return self._unsupported("velocity target")

    def position_limit(self, dof: int = 0) -> core.Limit:
        self._check_dof(dof)
        return core.Limit(-math.inf, math.inf)

    def joint_position_limit(self) -> core.Limit:
        return core.JointLimit([-math.inf] * 3, [math.inf] * 3)

    def max_generalized_force(self, dof: int = 0) -> float:
        self._check_dof(dof)
        return math.inf

    def joint_max_generalized_force(self) -> List[float]:
        return [math.inf] * 3


# ---------------------------------------------------------------------- Model
class Model:
    """An articulated model (one native simulator with a single world)."""

    def __init__(self, world: "World", name: str, sim, pose: core.Pose):
        self._world = world
        self._name = name
        self._sim = sim
        self._pose = pose
        # ScenarI/O joints: a ball joint's three internal dofs are one Joint
        self._joints: Dict[str, Joint] = {}
        self._jnames: List[str] = []
        self._ball: Dict[str, BallJoint] = {}
        names = list(sim.joint_names)
        i = 0
        while i < len(names):
            n = names[i]
            if n.endswith("#x") and i + 2 < len(names) and sim.joint_type(i) == 4 and names[i + 2] == n[:-2] + "#z":
                j = BallJoint(self, i, n[:-2])
                self._ball[j._name] = j
                i += 3
            else:
                j = Joint(self, i, n)
                i += 1
            self._joints[j._name] = j
            self._jnames.append(j._name)
        self._pending_vel = None
        self._export = None  # exported model rows (link forward kinematics)
        self._history: Optional[collections.deque] = None
        self._acc_targets: Dict[str, float] = {}   # JointAccelerationTarget (no physics effect)
        self._base_targets: Dict[str, list] = {}   # Base*Target components (no physics effect)

    # -- identity
    def to_gazebo(self) -> "Model":
        return self

    def valid(self) -> bool:
        return self._sim is not None

    def name(self) -> str:
        return self._name

    def dofs(self, joint_names: Sequence[str] = ()) -> int:
        if not joint_names:
            return self._sim.dofs
        return sum(self._joints[n].dofs() if n in self._joints else 1 for n in joint_names)

    def joint_names(self, scoped: bool = False) -> List[str]:
        return [f"{self._name}::{n}" if scoped else n for n in self._jnames]

    def get_joint(self, joint_name: str) -> Joint:
        if joint_name not in self._joints:
            raise RuntimeError(f"Joint '{joint_name}' not found in model '{self._name}'")
        return self._joints[joint_name]

    def joints(self, joint_names: Sequence[str] = ()) -> List[Joint]:
        return [self.get_joint(n) for n in (joint_names or self._jnames)]

    def base_frame(self) -> str:
        return self._sim.base_frame

    def nr_of_joints(self) -> int:
        return len(self._jnames)

    def nr_of_links(self) -> int:
        return len(self.link_names())

    def _file_mass(self) -> float:
        """Sum of the <inertial><mass> of every link in the model file (URDF:
        links without <inertial> weigh 0; SDF: sdformat's default mass 1)."""
        import xml.etree.ElementTree as ET
        text = getattr(self, "_text", None)
        if not text:
            return 0.0
        root = ET.fromstring(text)
        if root.tag == "robot":
            return float(sum(float(m.get("value", "0")) for m in root.findall("link/inertial/mass")))
        model = root if root.tag == "model" else root.find("model")
        total = 0.0
        for link in model.findall("link") if model is not None else []:
            m = link.find("inertial/mass")
            total += float(m.text) if m is not None else 1.0
        return total

    def total_mass(self, link_names: Sequence[str] = ()) -> float:
        # Model::totalMass (Model.cpp:413-425): the sum of Link::mass over the
        # links (every link of the model by default)
        return float(sum(self.get_link(n).mass() for n in (link_names or self.link_names())))

    def links_in_contact(self) -> List[str]:
        # Model::linksInContact (Model.cpp:725-736)
        return [n for n in self.link_names() if self.get_link(n).in_contact()]

    def joint_limits(self, joint_names: Sequence[str] = ()) -> core.JointLimit:
        # Model::jointLimits (Model.cpp:797-815): serialised position limits
        lims = [j.position_limit() for j in self.joints(joint_names)]
        return core.JointLimit([lm.min for lm in lims], [lm.max for lm in lims])

    def set_joint_acceleration_targets(self, accelerations: Sequence[float],
                                       joint_names: Sequence[str] = ()) -> bool:
        names = list(joint_names) or list(self._jnames)
        if len(accelerations) != len(names):
            _err("Wrong number of elements (joint_dofs=%d)" % len(names))
            return False
        for n in names:
            if n not in self._joints:
                _err(f"Joint '{n}' not found in model '{self._name}'")
                return False
        for n, a in zip(names, accelerations):
            self._acc_targets[n] = float(a)
        return True

    def joint_acceleration_targets(self, joint_names: Sequence[str] = ()) -> List[float]:
        return [self.get_joint(n).acceleration_target() for n in (joint_names or self._jnames)]

    # -- base targets (Model.cpp:1077-1246): stored for controllers, the
    # physics does not read them; a getter of a target never set raises
    def set_base_pose_target(self, position: Sequence[float], orientation: Sequence[float]) -> bool:
        self._base_targets["pose"] = [list(map(float, position)), list(map(float, orientation))]
        return True

    def set_base_position_target(self, position: Sequence[float]) -> bool:
        orientation = self._base_targets.get("pose", [None, [1.0, 0.0, 0.0, 0.0]])[1]
        return self.set_base_pose_target(position, orientation)

    def set_base_orientation_target(self, orientation: Sequence[float]) -> bool:
        position = self._base_targets.get("pose", [[0.0, 0.0, 0.0], None])[0]
        return self.set_base_pose_target(position, orientation)

    def set_base_world_velocity_target(self, linear: Sequence[float], angular: Sequence[float]) -> bool:
        return self.set_base_world_linear_velocity_target(linear) and \
            self.set_base_world_angular_velocity_target(angular)

    def set_base_world_linear_velocity_target(self, linear: Sequence[float]) -> bool:
        self._base_targets["lin_vel"] = list(map(float, linear))
        return True

    def set_base_world_angular_velocity_target(self, angular: Sequence[float]) -> bool:
        self._base_targets["ang_vel"] = list(map(float, angular))
        return True

    def set_base_world_linear_acceleration_target(self, linear: Sequence[float]) -> bool:
        self._base_targets["lin_acc"] = list(map(float, linear))
        return True

    def set_base_world_angular_acceleration_target(self, angular: Sequence[float]) -> bool:
        self._base_targets["ang_acc"] = list(map(float, angular))
        return True

    def _base_target(self, key: str, what: str):
        if key not in self._base_targets:
            raise RuntimeError(f"model '{self._name}' has no {what} target")
        return self._base_targets[key]

    def base_position_target(self) -> List[float]:
        return list(self._base_target("pose", "base pose")[0])

    def base_orientation_target(self) -> List[float]:
        return list(self._base_target("pose", "base pose")[1])

    def base_world_linear_velocity_target(self) -> List[float]:
        return list(self._base_target("lin_vel", "base linear velocity"))

    def base_world_angular_velocity_target(self) -> List[float]:
        return list(self._base_target("ang_vel", "base angular velocity"))

    def base_world_linear_acceleration_target(self) -> List[float]:
        return list(self._base_target("lin_acc", "base linear acceleration"))

    def base_world_angular_acceleration_target(self) -> List[float]:
        return list(self._base_target("ang_acc", "base angular acceleration"))

    def base_position(self) -> List[float]:
        # Model::basePosition (Model.cpp:976-984); a fixed base stays at its insertion pose
        if self._sim.floating:
            return self._sim.base_pose()[0, :3].tolist()
        return list(self._pose.position)

    def base_orientation(self) -> List[float]:
        # Model::baseOrientation (Model.cpp:986-994), wxyz
        if self._sim.floating:
            return self._sim.base_pose()[0, 3:].tolist()
        return list(self._pose.orientation)

    def base_world_linear_velocity(self) -> List[float]:
        return self._sim.base_velocity()[0, :3].tolist() if self._sim.floating else [0.0, 0.0, 0.0]

    def base_world_angular_velocity(self) -> List[float]:
        return self._sim.base_velocity()[0, 3:].tolist() if self._sim.floating else [0.0, 0.0, 0.0]

    def _base_R(self) -> np.ndarray:
        w, x, y, z = self.base_orientation()
        return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                         [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                         [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])

    def base_body_linear_velocity(self) -> List[float]:
        # Model::baseBodyLinearVelocity (Model.cpp:996-1008)
        return (self._base_R().T @ np.array(self.base_world_linear_velocity())).tolist()

    def base_body_angular_velocity(self) -> List[float]:
        return (self._base_R().T @ np.array(self.base_world_angular_velocity())).tolist()

    def _floating_only(self, what: str) -> bool:
        if not self._sim.floating:
            _err(f"{what}: the model '{self._name}' has a fixed base")
            return False
        return True

    def reset_base_pose(self, position: Sequence[float], orientation: Sequence[float]) -> bool:
        # Model::resetBasePose (Model.cpp:256-289): applied by the next run
        if not self._floating_only("reset_base_pose"):
            return False
        if len(position) != 3 or len(orientation) != 4:
            _err("Wrong size of the base pose")
            return False
        try:
            self._sim.reset_base_pose(list(position) + list(orientation))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def reset_base_position(self, position: Sequence[float]) -> bool:
        # Model.cpp:291-294: with the CURRENT orientation
        return self.reset_base_pose(position, self.base_orientation())

    def reset_base_orientation(self, orientation: Sequence[float]) -> bool:
        # Model.cpp:296-299: with the CURRENT position
        return self.reset_base_pose(self.base_position(), orientation)

    def reset_base_world_velocity(self, linear: Sequence[float], angular: Sequence[float]) -> bool:
        # Model::resetBaseWorldVelocity (Model.cpp:343-400)
        if not self._floating_only("reset_base_world_velocity"):
            return False
        try:
            self._sim.reset_base_velocity(list(linear) + list(angular))
            self._pending_vel = (list(linear), list(angular))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def reset_base_world_linear_velocity(self, linear: Sequence[float]) -> bool:
        # Model.cpp:301-320: keeps an angular velocity already reset in this run
        angular = self._pending_vel[1] if self._pending_vel else self.base_world_angular_velocity()
        return self.reset_base_world_velocity(linear, angular)

    def reset_base_world_angular_velocity(self, angular: Sequence[float]) -> bool:
        linear = self._pending_vel[0] if self._pending_vel else self.base_world_linear_velocity()
        return self.reset_base_world_velocity(linear, angular)

    # -- links and contacts (Link.cpp): the base link and the link of every joint
    def link_names(self, scoped: bool = False) -> List[str]:
        # Model::linkNames (Model.cpp:479-520); links lumped by fixed joints do not exist
        # unless the file keeps them (sdformat's preserveFixedJoint: _preserved_links);
        # a ball joint's internal massless links (`<joint>#x`, `#y`) are not links
        names = [self._sim.base_frame] + [n for n in self._sim.link_names if not self._internal_link(n)]
        names += list(self._preserved_links())
        return [f"{self._name}::{n}" for n in names] if scoped else names

    def get_link(self, link_name: str) -> "Link":
        if link_name == self._sim.base_frame:
            return Link(self, link_name, -1)
        if link_name in self._sim.link_names and not self._internal_link(link_name):
            return Link(self, link_name, self._sim.link_names.index(link_name))
        kept = self._preserved_links().get(link_name)
        if kept is not None:
            return Link(self, link_name, kept[0], offset=kept[1:3])
        raise RuntimeError(f"Link '{link_name}' not found in model '{self._name}'")

    def _preserved_links(self) -> Dict[str, tuple]:
        """Links welded to their parent by a fixed joint that the URDF asks
        sdformat to keep (`<gazebo reference="<joint>"><preserveFixedJoint>
        true</preserveFixedJoint></gazebo>`, e.g. the iCub's force/torque
        sensor frames): still links of the model (Model::linkNames, Link
        getters) although the physics lumps their inertia into the parent
        body (the model compiler, as DART's welded bodies move rigidly).
        name -> (owner body, R, p of the link frame in the owner body's
        frame, the link's own mass, has collisions, its COM in its frame)."""
        cache = self.__dict__.get("_preserved")
        if cache is not None:
            return cache
        out: Dict[str, tuple] = {}
        text = getattr(self, "_text", None)
        root = None
        if text:
            try:
                root = ET.fromstring(text.strip())
            except ET.ParseError:
                root = None
        if root is not None and root.tag == "robot":
            keep = {g.get("reference") for g in root.findall("gazebo")
                    if (g.findtext("preserveFixedJoint") or "").strip().lower() in ("true", "1")}
            compiled = {self._sim.base_frame: -1}
            compiled.update({n: i for i, n in enumerate(self._sim.link_names)})
            links = {lk.get("name"): lk for lk in root.findall("link")}
            pending = [j for j in root.findall("joint") if j.get("type") == "fixed" and j.get("name") in keep]
            progress = True
            while pending and progress:
                progress = False
                for j in list(pending):
                    parent, child = j.find("parent").get("link"), j.find("child").get("link")
                    if parent in compiled:
                        owner, R0, p0 = compiled[parent], np.eye(3), np.zeros(3)
                    elif parent in out:
                        owner, R0, p0 = out[parent][:3]
                    else:
                        continue
                    R, pj = _urdf_origin(j.find("origin"))
                    lk = links.get(child)
                    m = lk.find("inertial/mass") if lk is not None else None
                    com = _urdf_origin(lk.find("inertial/origin"))[1] if lk is not None else np.zeros(3)
                    out[child] = (owner, R0 @ R, p0 + R0 @ pj, float(m.get("value")) if m is not None else 0.0,
                                  lk is not None and lk.find("collision") is not None, com)
                    pending.remove(j)
                    progress = True
            # a body whose own link has no collision while exactly one kept
            # link on it has: the body's contacts are that link's (the iCub's
            # soles sit on the foot F/T-sensor frame)
            owned = {}
            for name, (owner, _R, _p, _m, col, _c) in out.items():
                if col:
                    owned.setdefault(owner, []).append(name)
            own_col = {compiled[n]: (links[n].find("collision") is not None) for n in compiled if n in links}
            self._contact_link = {b: ns[0] for b, ns in owned.items() if len(ns) == 1 and not own_col.get(b, False)}
        else:
            self._contact_link = {}
        self._preserved = out
        return out

    def links(self, link_names: Sequence[str] = ()) -> List["Link"]:
        return [self.get_link(n) for n in (link_names or self.link_names())]

    def _link_state(self, body: int):
        """World pose (R, p) and world velocity (linear of the link origin,
        angular) of `body` (-1 = base) by forward kinematics of the exported
        model (joint origin E, r, axis per body) from the base state."""
        R = self._base_R()
        p = np.array(self.base_position(), dtype=float)
        v = np.array(self.base_world_linear_velocity(), dtype=float)
        w = np.array(self.base_world_angular_velocity(), dtype=float)
        if body < 0:
            return R, p, v, w
        if self._export is None:
            n = self._sim.dofs
            self._export = self._sim.export_model()[:34 * n].reshape(n, 34)
        rows = self._export
        path = []
        k = body
        while k >= 0:
            path.append(k)
            k = int(rows[k, 33])
        q = self._sim.get("q")[0]
        qd = self._sim.get("qd")[0]
        for j in reversed(path):
            row = rows[j]
            E, r, a = row[2:11].reshape(3, 3), row[11:14], row[14:17]
            if row[0] == 0:  # revolute: Rodrigues about the child-frame axis
                c, sn = np.cos(q[j]), np.sin(q[j])
                K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
                Rr, pr = E @ (np.eye(3) + sn * K + (1 - c) * K @ K), r
            else:
                Rr, pr = E, r + q[j] * (E @ a)
            pn = p + R @ pr
            v = v + np.cross(w, pn - p)
            R = R @ Rr
            if row[0] == 0:
                w = w + R @ a * qd[j]
            else:
                v = v + R @ a * qd[j]
            p = pn
        return R, p, v, w

    def _link_acc(self, body: int):
        """World linear acceleration of the link origin and world angular
        acceleration of `body` from the joint accelerations of the last run
        (Physics.cpp:1948-2079 reads them from DART's link frames).  The base
        of a fixed-base model does not accelerate; a floating base's
        acceleration is not read back by this backend."""
        if self._sim.floating:
            raise RuntimeError("link accelerations of floating-base models are not available in this backend")
        R = self._base_R()
        p = np.array(self.base_position(), dtype=float)
        v = np.zeros(3)
        w = np.zeros(3)
        a = np.zeros(3)
        al = np.zeros(3)
        if body < 0:
            return a, al
        if self._export is None:
            n = self._sim.dofs
            self._export = self._sim.export_model()[:34 * n].reshape(n, 34)
        rows = self._export
        path = []
        k = body
        while k >= 0:
            path.append(k)
            k = int(rows[k, 33])
        q = self._sim.get("q")[0]
        qd = self._sim.get("qd")[0]
        qdd = self._sim.get("qdd")[0]
        for j in reversed(path):
            row = rows[j]
            E, r, ax = row[2:11].reshape(3, 3), row[11:14], row[14:17]
            if row[0] == 0:
                c, sn = np.cos(q[j]), np.sin(q[j])
                K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
                Rr, pr = E @ (np.eye(3) + sn * K + (1 - c) * K @ K), r
            else:
                Rr, pr = E, r + q[j] * (E @ ax)
            pn = p + R @ pr
            d = pn - p
            # rigid transport from the parent origin, then the joint's own terms
            a = a + np.cross(al, d) + np.cross(w, np.cross(w, d))
            v = v + np.cross(w, d)
            R = R @ Rr
            u = R @ ax  # joint axis in the world (fixed in parent and child)
            if row[0] == 0:
                al = al + u * qdd[j] + np.cross(w, u * qd[j])
                w = w + u * qd[j]
            else:
                a = a + u * qdd[j] + 2.0 * np.cross(w, u * qd[j])
                v = v + u * qd[j]
            p = pn
        return a, al

    def contacts_enabled(self) -> bool:
        return self._sim.contacts_enabled()

    def enable_contacts(self, enable: bool = True) -> bool:
        # Model::enableContacts (Model.cpp:686-700): a flag of this world's
        # view of the slot (the scene detects every world's contacts)
        self._sim.enable_contacts(enable)
        return True

    def contacts(self, link_names: Sequence[str] = ()) -> List[core.Contact]:
        # Model::contacts (Model.cpp:739-755): the contacts of every (selected) link
        out: List[core.Contact] = []
        for ln in (link_names or self.link_names()):
            out.extend(self.get_link(ln).contacts())
        return out

    def controller_period(self) -> float:
        # Model::controllerPeriod (Model.cpp:581-587)
        return self._comp(("period",))

    def set_controller_period(self, period: float) -> bool:
        # Model::setControllerPeriod (Model.cpp:589-602)
        try:
            if not (float(period) > 0.0):
                raise RuntimeError("The controller period must be greater than zero")
            self._set_component(("period",), float(period))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    # -- slot-wide components: PID gains, joint parameters, controller period
    def _comp(self, key):
        """The component `key` of this world's model: a change recorded
        since the last run, else the scene slot's value."""
        if self._sim is None:
            raise RuntimeError(f"model '{self._name}' was removed")
        pend = self.__dict__.get("_pending_comp")
        if pend and key in pend:
            return pend[key]
        return _read_component(self._sim, key)

    def _set_component(self, key, value) -> None:
        """Joint::setPID / setCoulombFriction / setViscousFriction /
        setMaxGeneralizedForce, Model::setControllerPeriod.  These components
        belong to a scene slot, which the same model inserted into several
        worlds shares; the reference keeps them per world (one ECM per
        world).  A model alone in its slot changes the slot at once.  A model
        sharing its slot records the change (a change back to the slot's
        value cancels it), and the next run() groups the slot's models by
        their recorded changes: the worlds that made none -- or, if every
        world changed something, the largest group of identical changes --
        keep the slot, every other group of identical changes moves to one
        slot of its own (GazeboSimulator._resolve_components).  So N worlds
        that each insert a Panda and call set_pid on every joint end up in
        one slot, changed once."""
        if self._sim is None:
            raise RuntimeError(f"model '{self._name}' was removed")
        sim = self._world._simulator
        if not sim._slot_shared(self):
            _write_component(self._sim, key, value)
            return
        if key[0] == "param":
            # validate now (the reference's setter fails at once): a model that
            # was already stepped refuses parameter changes
            _write_component(self._sim, key, _read_component(self._sim, key))
        pend = self.__dict__.setdefault("_pending_comp", {})
        if value == _read_component(self._sim, key):
            pend.pop(key, None)
        else:
            pend[key] = value

    def _internal_link(self, n: str) -> bool:
        return bool(self._ball) and (n.endswith("#x") or n.endswith("#y")) and n[:-2] in self._ball

    # -- vectorised joint data (serialised in the requested name order)
    def _dofs(self, names: Sequence[str]):
        if not self._ball:
            return self._sim.dof_indices(list(names) if names else None)
        out = []
        for n in (names or self._jnames):
            b = self._ball.get(n)
            out.extend(b._names if b is not None else [n])
        return self._sim.dof_indices(out)

    def _ball_list(self, what: str, joint_names: Sequence[str]) -> List[float]:
        # models with ball joints: a ball joint's three dofs hold DART's
        # BallJoint coordinates (no conversion)
        return self._get(what, self._dofs(joint_names)).tolist()

    def _get(self, what: str, dof_idx) -> np.ndarray:
        if self._sim is None:
            raise RuntimeError(f"model '{self._name}' was removed")
        if dof_idx is not None:
            dof_idx = np.asarray(dof_idx, dtype=np.int32)
        ov = self.__dict__.get("_state_override")
        if ov and what in ov:
            # moved to a slot of its own since the last run: the state it carried
            return ov[what].copy() if dof_idx is None else ov[what][dof_idx]
        return self._sim.get(what, 0, 1, dof_idx)[0]

    def _state_list(self, what: str, joint_names: Sequence[str]) -> List[float]:
        # the per-env path reads the same joints several times per env step
        # (observation, reward, termination): memoised per joint-state
        # generation of the scene (every run and mutator starts a new one)
        if self._sim is None:
            raise RuntimeError(f"model '{self._name}' was removed")
        if self._ball:
            return self._ball_list(what, joint_names)
        gen = self._sim.scene.gen
        key = (what, tuple(joint_names) if joint_names else ())
        memo = self.__dict__.setdefault("_memo", {})
        hit = memo.get(key)
        if hit is not None and hit[0] == gen:
            return list(hit[1])
        val = self._get(what, self._dofs(joint_names)).tolist()
        if len(memo) > 64:
            memo.clear()
        memo[key] = (gen, val)
        return list(val)

    def joint_positions(self, joint_names: Sequence[str] = ()) -> List[float]:
        return self._state_list("q", joint_names)

    def joint_velocities(self, joint_names: Sequence[str] = ()) -> List[float]:
        return self._state_list("qd", joint_names)

    def joint_accelerations(self, joint_names: Sequence[str] = ()) -> List[float]:
        if self._ball:
            return self._ball_list("qdd", joint_names)
        return self._get("qdd", self._dofs(joint_names)).tolist()

    def joint_generalized_forces(self, joint_names: Sequence[str] = ()) -> List[float]:
        if self._ball:
            return self._ball_list("force", joint_names)
        return self._get("force", self._dofs(joint_names)).tolist()

    def joint_generalized_force_targets(self, joint_names: Sequence[str] = ()) -> List[float]:
        if self._ball:
            return self._ball_list("force_target", joint_names)
        return self._get("force_target", self._dofs(joint_names)).tolist()

    def joint_velocity_targets(self, joint_names: Sequence[str] = ()) -> List[float]:
        return self._get("velocity_target", self._dofs(joint_names)).tolist()

    def joint_position_targets(self, joint_names: Sequence[str] = ()) -> List[float]:
        return self._get("position_target", self._dofs(joint_names)).tolist()

    def _set(self, what: str, values, joint_names: Sequence[str]) -> bool:
        try:
            if self._ball:
                # ball joints: 3 values each, in DART's BallJoint coordinates
                names = list(joint_names) or list(self._jnames)
                n = self.dofs(names)
                if len(values) != n:
                    _err(f"Wrong number of elements (joint_dofs={n})")
                    return False
                vals, k = [], 0
                for nm in names:
                    b = self._ball.get(nm)
                    if b is not None:
                        vals.extend(b._to_internal(what, values[k:k + 3]).tolist())
                        k += 3
                    else:
                        vals.append(values[k])
                        k += 1
                values = vals
                joint_names = names
            idx = self._dofs(joint_names)
            n = self._sim.dofs if idx is None else len(idx)
            if len(values) != n:
                _err(f"Wrong number of elements (joint_dofs={n})")
                return False
            self._sim.set(what, [list(values)], 0, 1, idx)
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def set_joint_generalized_force_targets(self, forces, joint_names: Sequence[str] = ()) -> bool:
        return self._set("force_target", forces, joint_names)

    def set_joint_velocity_targets(self, velocities, joint_names: Sequence[str] = ()) -> bool:
        return self._set("velocity_target", velocities, joint_names)

    def set_joint_position_targets(self, positions, joint_names: Sequence[str] = ()) -> bool:
        return self._set("position_target", positions, joint_names)

    def reset_joint_positions(self, positions, joint_names: Sequence[str] = ()) -> bool:
        return self._set("reset_q", positions, joint_names)

    def reset_joint_velocities(self, velocities, joint_names: Sequence[str] = ()) -> bool:
        return self._set("reset_qd", velocities, joint_names)

    def set_joint_control_mode(self, mode: int, joint_names: Sequence[str] = ()) -> bool:
        try:
            self._sim.set_control_mode(int(mode), 0, 1, self._dofs(joint_names))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    # -- history of applied joint forces (HistoryOfAppliedJointForces component)
    def enable_history_of_applied_joint_forces(self, enable: bool = True,
                                               max_history_size_per_joint: int = 100) -> bool:
        if enable:
            if self._history is None:
                self._history = collections.deque(maxlen=max_history_size_per_joint * self.dofs())
        else:
            self._history = None
        return True

    def history_of_applied_joint_forces_enabled(self) -> bool:
        return self._history is not None

    def history_of_applied_joint_forces(self, joint_names: Sequence[str] = ()) -> List[float]:
        if self._history is None:
            return []
        h = np.array(self._history).reshape(-1, self.dofs())
        idx = self._dofs(joint_names)
        return (h if idx is None else h[:, idx]).reshape(-1).tolist()

    # -- stepping (called by GazeboSimulator.run)
    def _run(self, paused: bool) -> None:
        # bookkeeping before the world's scene runs (GazeboSimulator.run)
        if self._history is not None and not paused:
            self._history.extend(self._get("force_target", None).tolist())
        self._pending_vel = None
        self.__dict__.pop("_state_override", None)

    def _close(self) -> None:
        if self._sim is not None:
            self._world._simulator._remove_model(self._sim)
            self._sim = None


class Link:
    """A link of a model (Link.cpp): pose, velocity and contacts."""

    def __init__(self, model: "Model", name: str, body: int = -1, offset=None):
        self._model = model
        self._name = name
        self._body = body  # -1 = the base link, i = the link moved by joint i
        # a link kept on a fixed joint (Model._preserved_links): its frame in the body's
        self._offset = offset

    def _state(self):
        """World R, p, v (of the link origin), w of this link."""
        R, p, v, w = self._model._link_state(self._body)
        if self._offset is None:
            return R, p, v, w
        Ro, po = self._offset
        d = R @ po
        return R @ Ro, p + d, v + np.cross(w, d), w

    def _acc(self):
        a, al = self._model._link_acc(self._body)
        if self._offset is None:
            return a, al
        R, _, _, w = self._model._link_state(self._body)
        d = R @ self._offset[1]
        return a + np.cross(al, d) + np.cross(w, np.cross(w, d)), al

    def _contact_owner(self) -> bool:
        """Whether this link reports its body's contacts: a body's own link
        does unless a kept link on it carries the body's collisions."""
        m = self._model
        m._preserved_links()
        delegate = m._contact_link.get(self._body)
        return (delegate == self._name) if delegate is not None else self._offset is None

    def to_gazebo(self) -> "Link":
        return self

    def name(self, scoped: bool = False) -> str:
        return f"{self._model.name()}::{self._name}" if scoped else self._name

    def mass(self) -> float:
        # Link::mass (Link.cpp:198-204) of the compiled body: links welded by
        # fixed joints are lumped into one body (their masses summed), except
        # the links the file keeps (Model._preserved_links), which have their own
        kept = self._model._preserved_links()
        if self._offset is not None:
            return kept[self._name][3]
        mine = sum(v[3] for v in kept.values() if v[0] == self._body)
        ex = self._model._sim.export_model()
        n = self._model._sim.dofs
        if self._body >= 0:
            return float(ex[34 * self._body + 17]) - mine
        if self._model._sim.floating:
            return float(ex[34 * n + 3]) - mine
        # a welded base is not part of the dynamics: its (lumped) mass is what
        # the model file holds beyond the moving bodies
        return max(self._model._file_mass() - sum(float(ex[34 * b + 17]) for b in range(n)), 0.0)

    def position(self) -> List[float]:
        return self._state()[1].tolist()

    def orientation(self) -> List[float]:
        # wxyz of the link rotation
        return _quat_from_R(self._state()[0])

    def world_linear_velocity(self) -> List[float]:
        return self._state()[2].tolist()

    def world_angular_velocity(self) -> List[float]:
        return self._state()[3].tolist()

    # body-fixed (link frame) velocities and accelerations: W_R_L^T times the
    # world ones (Link.cpp bodyLinearVelocity & co., ign-gazebo issue 87 note)
    def body_linear_velocity(self) -> List[float]:
        R, _, v, _ = self._state()
        return (R.T @ v).tolist()

    def body_angular_velocity(self) -> List[float]:
        R, _, _, w = self._state()
        return (R.T @ w).tolist()

    def world_linear_acceleration(self) -> List[float]:
        return self._acc()[0].tolist()

    def world_angular_acceleration(self) -> List[float]:
        return self._acc()[1].tolist()

    def body_linear_acceleration(self) -> List[float]:
        return (self._state()[0].T @ self._acc()[0]).tolist()

    def body_angular_acceleration(self) -> List[float]:
        return (self._state()[0].T @ self._acc()[1]).tolist()

    def contacts_enabled(self) -> bool:
        return self._model.contacts_enabled()

    def enable_contact_detection(self, enable: bool) -> bool:
        return self._model.enable_contacts(enable)

    def contacts(self) -> List[core.Contact]:
        # Link::contacts (Link.cpp:365-434): the points of one body pair are
        # merged into one Contact, body_a = this link; the other body is a
        # link of another model of the world or the ground plane
        sim = self._model._sim
        if not sim.contacts_enabled() or not self._contact_owner():
            return []
        rows = sim.contact_rows()
        groups: "collections.OrderedDict[tuple, list]" = collections.OrderedDict()
        for r in rows:
            if int(r[10]) != self._body:
                continue
            groups.setdefault((int(r[11]), int(r[12])), []).append(r)
        out = []
        world = self._model._world
        for (om, ol), pts in groups.items():
            if om < 0:
                other = world._ground_name or "ground_plane::link"
            else:
                other = world._link_name_of(om, ol)
            cps = [core.ContactPoint(r[0:3], r[3:6], r[6:9], (0.0, 0.0, 0.0), r[9]) for r in pts]
            out.append(core.Contact(self.name(scoped=True), other, cps))
        return out

    def in_contact(self) -> bool:
        return len(self.contacts()) > 0

    # -- external wrenches (Link::applyWorldForce / Torque / Wrench[ToCoM],
    # Link.cpp:484-560): world force at the link origin and world torque,
    # applied from the next physics step until simTime >= now + duration
    def apply_world_wrench(self, force: Sequence[float], torque: Sequence[float], duration: float = 0.0) -> bool:
        if len(force) != 3 or len(torque) != 3:
            _err("The force and the torque must have 3 elements")
            return False
        try:
            torque = np.asarray(torque, dtype=float)
            if self._offset is not None:
                # a kept link's origin is off its body's: move the force there
                R, p, _, _ = self._model._link_state(self._body)
                torque = torque + np.cross(R @ self._offset[1], np.asarray(force, dtype=float))
            self._model._sim.apply_world_wrench(self._body, list(force) + torque.tolist(), float(duration))
            return True
        except RuntimeError as e:
            _err(str(e))
            return False

    def apply_world_force(self, force: Sequence[float], duration: float = 0.0) -> bool:
        return self.apply_world_wrench(force, [0.0, 0.0, 0.0], duration)

    def apply_world_torque(self, torque: Sequence[float], duration: float = 0.0) -> bool:
        return self.apply_world_wrench([0.0, 0.0, 0.0], torque, duration)

    def apply_world_wrench_to_com(self, force: Sequence[float], torque: Sequence[float],
                                  duration: float = 0.0) -> bool:
        # the force acts at the COM: its moment about the link origin is added
        # (W_R_L L_o_I) x f (Link.cpp:534-560)
        ex = self._model._sim.export_model()
        n = self._model._sim.dofs
        if self._offset is not None:   # a kept link: its own inertial origin
            com = self._model._preserved_links()[self._name][5]
        else:
            com = ex[34 * n + 4:34 * n + 7] if self._body < 0 else ex[34 * self._body + 18:34 * self._body + 21]
        R = self._state()[0]
        t = np.asarray(torque, dtype=float) + np.cross(R @ com, np.asarray(force, dtype=float))
        return self.apply_world_wrench(force, t.tolist(), duration)

    def contact_wrench(self) -> List[float]:
        # Link::contactWrench (Link.cpp:436-482): sum of forces and of (p - o_L) x f
        o = np.array(self.position())
        f = np.zeros(3)
        t = np.zeros(3)
        for c in self.contacts():
            for p in c.points:
                fp = np.array(p.force)
                f += fp
                t += np.cross(np.array(p.position) - o, fp)
        return np.concatenate([f, t]).tolist()


def _urdf_origin(el) -> tuple:
    """(R, p) of a URDF <origin xyz rpy> (fixed-axis roll, pitch, yaw)."""
    if el is None:
        return np.eye(3), np.zeros(3)
    p = np.array([float(v) for v in (el.get("xyz") or "0 0 0").split()])
    r, pi, y = (float(v) for v in (el.get("rpy") or "0 0 0").split())
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(pi), math.sin(pi), math.cos(y), math.sin(y)
    R = np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                  [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                  [-sp, cp * sr, cp * cr]])
    return R, p


def _quat_from_R(R: np.ndarray) -> List[float]:
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        k = 0.5 / np.sqrt(tr + 1.0)
        q = [0.25 / k, (R[2, 1] - R[1, 2]) * k, (R[0, 2] - R[2, 0]) * k, (R[1, 0] - R[0, 1]) * k]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        k = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        q = [(R[2, 1] - R[1, 2]) / k, 0.25 * k, (R[0, 1] + R[1, 0]) / k, (R[0, 2] + R[2, 0]) / k]
    elif R[1, 1] > R[2, 2]:
        k = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        q = [(R[0, 2] - R[2, 0]) / k, (R[0, 1] + R[1, 0]) / k, 0.25 * k, (R[1, 2] + R[2, 1]) / k]
    else:
        k = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
        q = [(R[1, 0] - R[0, 1]) / k, (R[0, 2] + R[2, 0]) / k, (R[1, 2] + R[2, 1]) / k, 0.25 * k]
    return [float(x) for x in q]


class StaticModel:
    """A model without degrees of freedom (e.g. the ground plane)."""

    def __init__(self, name: str, pose: core.Pose):
        self._name = name
        self._pose = pose

    def to_gazebo(self):
        return self

    def valid(self) -> bool:
        return True

    def name(self) -> str:
        return self._name

    def dofs(self, joint_names: Sequence[str] = ()) -> int:
        return 0

    def joint_names(self, scoped: bool = False) -> List[str]:
        return []

    def base_position(self) -> List[float]:
        return list(self._pose.position)

    def base_orientation(self) -> List[float]:
        return list(self._pose.orientation)

    def _run(self, paused: bool) -> None:
        pass

    def _close(self) -> None:
        pass


# ---------------------------------------------------------------------- World
class World:
    """One world of the simulator: world index `_index` of the simulator's scene."""

    def __init__(self, simulator: "GazeboSimulator", name: str, index: int):
        self._simulator = simulator
        self._name = name
        self._index = index
        self._models: "collections.OrderedDict[str, object]" = collections.OrderedDict()
        self._physics = False
        self._time_ns = 0
        self._gravity = [0.0, 0.0, -9.8]
        self._ground_mu = None     # a static model with a plane collision is in the world
        self._ground_name = None
        # removed models stay listed until the next (paused or unpaused) run
        # processes the removal request (World::removeModel, World.cpp:432-453)
        self._removing: List[str] = []

    def to_gazebo(self) -> "World":
        return self

    @property
    def name(self):
        # usable both as attribute-like `world.name` checks and as `world.name()`
        return _NameProxy(self._name)

    def time(self) -> float:
        return self._time_ns / 1e9

    def gravity(self) -> List[float]:
        return list(self._gravity)

    def set_gravity(self, gravity: Sequence[float]) -> bool:
        if len(gravity) != 3:
            _err("The gravity must have 3 elements")
            return False
        self._gravity = [float(g) for g in gravity]
        try:
            self._simulator._set_gravity(self, self._gravity)
        except RuntimeError as e:
            _err(str(e))
            return False
        return True

    def model_names(self) -> List[str]:
        return list(self._models.keys()) + [n for n in self._removing if n not in self._models]

    def get_model(self, model_name: str):
        if model_name not in self._models:
            raise RuntimeError(f"Model '{model_name}' not found in world '{self._name}'")
        return self._models[model_name]

    def models(self, model_names: Sequence[str] = ()) -> list:
        return [self.get_model(n) for n in (model_names or self.model_names())]

    def _link_name_of(self, slot: int, link: int) -> str:
        """scoped name of link `link` (-1 base) of the model in scene slot `slot`"""
        for name, m in self._models.items():
            if isinstance(m, Model) and m._sim is not None and m._sim.m == slot:
                sim = m._sim
                m._preserved_links()   # a body's collisions may sit on a kept link
                return f"{name}::{m._contact_link.get(link, sim.base_frame if link < 0 else sim.link_names[link])}"
        return f"model{slot}::link{link}"

    def set_physics_engine(self, engine: int = PhysicsEngine_dart) -> bool:
        if engine != PhysicsEngine_dart:
            _err("Physics engine not supported")
            return False
        if self._physics:
            _err("The physics engine was already inserted in this world")
            return False
        self._physics = True
        # the Physics system starts stepping the models already in the world
        for m in self._models.values():
            if isinstance(m, Model):
                self._simulator._scene.set_present(m._sim.m, 2, self._index, 1)
        return True

    def insert_model(self, model_file: str, pose: core.Pose = None, override_model_name: str = "") -> bool:
        try:
            text = _read(model_file)
        except OSError as e:
            _err(f"Failed to read model file: {e}")
            return False
        if os.path.isfile(model_file):
            text = _absolute_mesh_uris(text, os.path.dirname(os.path.abspath(model_file)))
        return self.insert_model_from_string(text, pose, override_model_name)

    def insert_model_from_string(self, model_string: str, pose: core.Pose = None,
                                 override_model_name: str = "") -> bool:
        if not self._simulator.initialized():
            _err("The simulator was not initialized")
            return False
        pose = pose or core.Pose.identity()
        try:
            root = ET.fromstring(model_string.strip())
        except ET.ParseError as e:
            _err(f"Failed to parse the model: {e}")
            return False
        if root.tag == "robot":
            name = override_model_name or root.get("name", "model")
        else:
            m = root.find("model")
            if m is None:
                _err("The SDF does not contain a <model>")
                return False
            name = override_model_name or m.get("name", "model")
        if name in self._models:
            _err(f"Model '{name}' already exists in world '{self._name}'")
            return False
        static = root.tag != "robot" and (root.find("model/static") is not None and
                                          root.find("model/static").text.strip().lower() in ("1", "true"))
        solid = [g for g in root.findall("model/link/collision/geometry")
                 if any(g.find(t) is not None for t in ("box", "sphere", "cylinder", "mesh"))]
        if static and not solid:
            if root.findall("model/joint"):
                _err("static SDF models with joints are not supported by this build")
                return False
            self._models[name] = StaticModel(name, pose)
            plane = root.find("model/link/collision/geometry/plane")
            if plane is not None:
                # the ground plane of the world: every model collides with it
                mu_el = root.find("model/link/collision/surface/friction/ode/mu")
                self._ground_mu = float(mu_el.text) if mu_el is not None else 1.0
                link = root.find("model/link")
                self._ground_name = f"{name}::{link.get('name', 'link')}"
                self._simulator._set_ground(self, True, self._ground_mu)
            return True
        # a static model with box / sphere / cylinder / mesh collisions is a welded
        # collider of the scene (the model compiler welds its links to the world)
        if root.tag != "robot" and [float(v) for v in (*pose.position, *pose.orientation)] == [0, 0, 0, 1, 0, 0, 0]:
            # the identity keeps the SDF model's own <pose> (World.cpp:169-177)
            pose = _sdf_model_pose(root)
        try:
            view = self._simulator._place_model(self, model_string,
                                                list(pose.position) + list(pose.orientation), name)
        except RuntimeError as e:
            _err(f"Failed to insert model '{name}': {e}")
            return False
        self._models[name] = Model(self, name, view, pose)
        self._models[name]._text = model_string
        return True

    def remove_model(self, model_name: str) -> bool:
        if model_name not in self._models:
            _err(f"Model '{model_name}' not found in world '{self._name}'")
            return False
        removed = self._models.pop(model_name)
        removed._close()
        self._removing.append(model_name)
        if self._ground_name is not None and self._ground_name.split("::")[0] == model_name:
            self._ground_mu = self._ground_name = None
            self._simulator._set_ground(self, False, 1.0)
        return True

    # called by GazeboSimulator.run before the scene steps
    def _update(self, paused: bool, sim_time_ns: int) -> None:
        self._removing.clear()
        if not self._physics:
            return
        self._time_ns = sim_time_ns
        for m in self._models.values():
            m._run(paused)

    def _close(self) -> None:
        for m in self._models.values():
            m._close()
        self._models.clear()


class _NameProxy(str):
    """A str that can also be called: the reference exposes World.name() while
    gym_ignition's Task checks ``world.name == ""``."""

    def __call__(self) -> str:
        return str(self)


# ------------------------------------------------------------ GazeboSimulator
class GazeboSimulator:
    """Lifecycle of a set of worlds stepped in lockstep (GazeboSimulator.h):
    all of them are the worlds of one native scene, stepped by one launch."""

    def __init__(self, step_size: float = 0.001, rtf: float = 1.0, steps_per_run: int = 1):
        self._step_size = float(step_size)
        self._rtf = float(rtf)
        self._steps_per_run = int(steps_per_run)
        self._initialized = False
        self._worlds: "collections.OrderedDict[str, World]" = collections.OrderedDict()
        self._pending_worlds: List[str] = []
        self._iterations = 0
        self._scene = None
        self._slots: List[tuple] = []   # per scene slot: (name, text, pose) of its current model

    def step_size(self) -> float:
        return self._step_size

    def real_time_factor(self) -> float:
        return self._rtf

    def steps_per_run(self) -> int:
        return self._steps_per_run

    def initialized(self) -> bool:
        return self._initialized

    def insert_world_from_sdf(self, world_file: str = "", world_name: str = "") -> bool:
        if self._initialized:
            _err("Worlds can be inserted only before initializing the simulator")
            return False
        if world_file:
            try:
                name = world_name or get_world_name_from_sdf(world_file)
            except (OSError, ET.ParseError) as e:
                _err(f"Failed to load the SDF world: {e}")
                return False
        else:
            name = world_name or "default"
        if name in self._pending_worlds:
            _err(f"World '{name}' already exists")
            return False
        self._pending_worlds.append(name)
        return True

    def insert_worlds_from_sdf(self, world_file: str, world_names: Sequence[str] = ()) -> bool:
        try:
            root = ET.fromstring(_read(world_file).strip())
        except (OSError, ET.ParseError) as e:
            _err(f"Failed to load the SDF worlds: {e}")
            return False
        names = [w.get("name", "") for w in root.findall("world")]
        if world_names:
            if len(world_names) != len(names):
                _err("The number of world names does not match the worlds in the SDF")
                return False
            names = list(world_names)
        return all(self.insert_world_from_sdf("", n) for n in names)

    def initialize(self) -> bool:
        if self._initialized:
            return True
        # helpers.cpp:391-400 and GazeboSimulator.cpp:578-582
        if self._step_size <= 0:
            _err("The physics step size must be positive")
            return False
        if self._rtf <= 0:
            _err("The real-time factor must be positive")
            return False
        if self._steps_per_run <= 0:
            _err("The number of steps per run must be positive")
            return False
        if not self._pending_worlds:
            self._pending_worlds.append("default")
        from mwstep.scene import Scene
        try:
            self._scene = Scene(n_worlds=len(self._pending_worlds), step_size=self._step_size,
                                steps_per_run=self._steps_per_run, rtf=self._rtf, device=_device(), pgs_iters=50)
            self._scene.set_ground_plane(False, 1.0)
        except RuntimeError as e:
            _err(f"Failed to create the simulator: {e}")
            return False
        for i, n in enumerate(self._pending_worlds):
            self._worlds[n] = World(self, n, i)
        self._initialized = True
        return True

    # ---- scene slots (internal)
    def _place_model(self, world: World, text: str, pose: List[float], name: str):
        """World::insertModel into `world`: reuse the slot holding the same
        model (name, file, pose; any pose for a floating model) if it is not
        in that world yet, else a free
        slot of the same tree (an env randomizer's per-episode model), else a
        new slot; returns the SceneView of the model in that world."""
        from mwstep.scene import SceneView
        sc, w = self._scene, world._index
        key = (name, text, tuple(round(float(v), 12) for v in pose))
        slot = None
        for m, k in enumerate(self._slots):
            if k == key and not sc.present(m, w):
                slot = m
                break
        moved = False
        if slot is None:
            # a floating model's insert pose is only its initial base state:
            # the slot of the same model (name, file) at another pose serves
            # this world too, its base reset to this pose (N worlds inserting
            # one robot at randomised poses take one slot, not N)
            for m, k in enumerate(self._slots):
                if len(k) == 3 and k[:2] == key[:2] and sc.models[m]["floating"] and not sc.present(m, w):
                    slot, moved = m, True
                    break
        if slot is not None:
            sc.set_present(slot, 1, w, 1)
            if moved:
                sc.reset_base_pose(slot, np.asarray(pose, dtype=np.float64).reshape(1, 7), w, 1)
        else:
            for m, k in enumerate(self._slots):
                if not any(sc.present(m, ww) for ww in range(sc.n_worlds)):
                    try:
                        sc.replace_model(m, text, pose, f"{name}#{m}")
                    except RuntimeError:
                        continue
                    self._slots[m] = key
                    slot = m
                    sc.set_present(slot, 1, w, 1)
                    break
        if slot is None:
            slot = sc.insert_model(text, pose, f"{name}#{len(self._slots)}", worlds=(w, 1))
            self._slots.append(key)
        if not world._physics:
            sc.set_present(slot, 0, w, 1)   # placed, not stepped until the Physics system is inserted
        return SceneView(sc, slot, w)

    def _slot_models(self, m: int) -> List["Model"]:
        return [o for wd in self._worlds.values() for o in wd._models.values()
                if isinstance(o, Model) and o._sim is not None and o._sim.m == m]

    def _slot_shared(self, model: "Model") -> bool:
        return any(o is not model for o in self._slot_models(model._sim.m))

    def _resolve_components(self) -> None:
        """Apply the slot-wide component changes that models sharing a slot
        recorded since the last run (Model._set_component): per slot, the
        models are grouped by their recorded changes; the group without
        changes (else the largest group) keeps the slot and its changes are
        applied to it once, every other group moves to one new slot."""
        slots = sorted({o._sim.m for wd in self._worlds.values() for o in wd._models.values()
                        if isinstance(o, Model) and o._sim is not None and o.__dict__.get("_pending_comp")})
        for m in slots:
            models = self._slot_models(m)
            groups: Dict[tuple, List[Model]] = {}
            for o in models:
                k = tuple(sorted((o.__dict__.get("_pending_comp") or {}).items()))
                groups.setdefault(k, []).append(o)
            keep = () if () in groups else max(groups, key=lambda k: len(groups[k]))
            for k, grp in groups.items():
                if k != keep:
                    self._move_models(grp, m, dict(k))
            view = groups[keep][0]._sim
            for key, value in keep:
                _write_component(view, key, value)
            for o in models:
                o.__dict__.pop("_pending_comp", None)

    def _move_models(self, models: List["Model"], m: int, changes: dict) -> None:
        """Move the models of several worlds, all sharing slot m, to one new
        slot whose components are slot m's with `changes` applied, carrying
        each world's state (joint state, targets, control modes, base).  If
        the scene has no room for another slot, the changes go to slot m
        itself (every world sharing it sees them) with a warning."""
        from mwstep import native as N
        from mwstep.scene import SceneView
        sc = self._scene
        old = models[0]._sim
        name, text, pose = self._slots[m][:3]
        nd = sc.models[m]["dofs"]
        floating = sc.models[m]["floating"]
        pkeys = (N.PARAM_COULOMB_FRICTION, N.PARAM_VISCOUS_FRICTION, N.PARAM_MAX_GENERALIZED_FORCE)
        comps = {("pid", d): _read_component(old, ("pid", d)) for d in range(nd)}
        comps.update({("param", d, k): _read_component(old, ("param", d, k)) for d in range(nd) for k in pkeys})
        comps[("period",)] = _read_component(old, ("period",))
        comps.update(changes)
        # each world's state and per-world components, read before the move
        carried = []
        for mdl in models:
            v = mdl._sim
            carried.append(dict(
                present=sc.present(m, v.w), q=v.get("q"), qd=v.get("qd"), qdd=v.get("qdd"),
                tgt={k: v.get(k) for k in ("position_target", "velocity_target", "force_target")},
                modes=[v.control_mode(v.w, d) for d in range(nd)], contacts=v.contacts_enabled(),
                base=(v.base_pose(), v.base_velocity()) if floating else None))
        w0 = models[0]._sim.w
        try:
            slot = sc.insert_model(text, list(pose), f"{name}#{len(self._slots)}", worlds=(w0, 1))
        except RuntimeError as e:
            _warn(f"No room for another scene slot ({e}): the component change of model '{name}' "
                  f"applies to every world sharing its slot")
            for key, value in changes.items():
                _write_component(old, key, value)
            return
        self._slots.append((name, text, tuple(pose), "own", tuple(mdl._sim.w for mdl in models)))  # never shared again
        first = SceneView(sc, slot, w0)
        # slot-wide components first (a parameter change rebuilds the slot)
        for key in sorted(k for k in comps if k[0] == "param"):
            _write_component(first, key, comps[key])
        for d in range(nd):
            _write_component(first, ("pid", d), comps[("pid", d)])
        _write_component(first, ("period",), comps[("period",)])
        for mdl, c in zip(models, carried):
            w = mdl._sim.w
            if w != w0:
                sc.set_present(slot, 1, w, 1)
            view = SceneView(sc, slot, w)
            for d in range(nd):
                view.set_control_mode(c["modes"][d], dofs=[d])
            view.enable_contacts(c["contacts"])
            view.set("reset_q", c["q"])
            view.set("reset_qd", c["qd"])
            for k, v in c["tgt"].items():
                for d in range(nd):
                    if k == "force_target" and v[0, d] == 0.0:
                        continue
                    try:  # the targets the dof's control mode accepts
                        view.set(k, v[:, d:d + 1], dofs=[d])
                    except RuntimeError:
                        pass
            if floating:
                view.reset_base_pose(c["base"][0])
                view.reset_base_velocity(c["base"][1])
            sc.set_present(m, 0, w, 1)
            if not c["present"]:  # placed without the Physics system: not stepped yet
                sc.set_present(slot, 0, w, 1)
            mdl._sim = view
            mdl._export = None
            # until the next run applies the resets, the getters read the carried state
            mdl._state_override = {"q": c["q"][0].copy(), "qd": c["qd"][0].copy(), "qdd": c["qdd"][0].copy()}

    def _remove_model(self, view) -> None:
        if self._scene is not None:
            self._scene.set_present(view.m, 0, view.w, 1)

    def _set_ground(self, world: World, enabled: bool, mu: float) -> None:
        # the plane's presence and friction are per world
        if enabled:
            self._scene.set_world_friction(mu, world._index, 1)
        self._scene.set_world_ground(enabled, world._index, 1)

    def _set_gravity(self, world: World, g: List[float]) -> None:
        # World::setGravity: this world's Gravity component only (World.cpp:301-319)
        self._scene.set_world_gravity(g, world._index, 1)

    def world_names(self) -> List[str]:
        return list(self._worlds.keys())

    def get_world(self, world_name: str = "") -> World:
        if not self._initialized:
            raise RuntimeError("The simulator was not initialized")
        if not world_name:
            return next(iter(self._worlds.values()))
        if world_name not in self._worlds:
            raise RuntimeError(f"World '{world_name}' not found")
        return self._worlds[world_name]

    def run(self, paused: bool = False) -> bool:
        if not self._initialized:
            _err("The simulator was not initialized")
            return False
        if not paused:
            self._iterations += self._steps_per_run
        t_ns = self._iterations * int(round(self._step_size * 1e9))
        try:
            self._resolve_components()
            for w in self._worlds.values():
                w._update(paused, t_ns)
            self._scene.run(paused)
        except RuntimeError as e:
            _err(f"The server couldn't execute the step: {e}")
            return False
        return True

    def gui(self, verbosity: int = -1) -> bool:
        _warn("The GUI is not part of this build")
        return False

    def pause(self) -> bool:
        return True

    def running(self) -> bool:
        return False

    def close(self) -> bool:
        for w in self._worlds.values():
            w._close()
        self._worlds.clear()
        if self._scene is not None:
            self._scene.close()
            self._scene = None
        self._initialized = False
        return True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
