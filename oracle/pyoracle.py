"""ctypes front-end of the fp64 CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``gym-ignition_amd/``) never imports it.

It carries its own URDF reader (``xml.etree``) so that the model the oracle
steps is compiled independently of the product's C++ model compiler; a test
cross-checks the two compilations.  URDF semantics follow what sdformat does
on URDF import for the reference (fixed joints lumped into their parent link,
``world`` link => fixed base), as used by
``/root/reference/python/gym_ignition/runtimes/gazebo_runtime.py:249-262``.
"""

from __future__ import annotations

import ctypes
import math
import os
import subprocess
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OR_MAXB = 48
PASSIVE, FORCE, SERVO = 0, 1, 2
TASK_CARTPOLE_DISCRETE = 0
TASK_CARTPOLE_CONTINUOUS_BALANCING = 1
TASK_CARTPOLE_CONTINUOUS_SWINGUP = 2
TASK_PENDULUM_SWINGUP = 3


class OrModel(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32),
        ("jtype", ctypes.c_int32 * OR_MAXB),
        ("limited", ctypes.c_int32 * OR_MAXB),
        ("parent", ctypes.c_int32 * OR_MAXB),
        ("pad_", ctypes.c_int32),
        ("gravity_base", ctypes.c_double * 3),
        ("E", (ctypes.c_double * 9) * OR_MAXB),
        ("r", (ctypes.c_double * 3) * OR_MAXB),
        ("axis", (ctypes.c_double * 3) * OR_MAXB),
        ("mass", ctypes.c_double * OR_MAXB),
        ("com", (ctypes.c_double * 3) * OR_MAXB),
        ("Ic", (ctypes.c_double * 6) * OR_MAXB),
        ("damping", ctypes.c_double * OR_MAXB),
        ("friction", ctypes.c_double * OR_MAXB),
        ("lower", ctypes.c_double * OR_MAXB),
        ("upper", ctypes.c_double * OR_MAXB),
        ("effort", ctypes.c_double * OR_MAXB),
        ("vel_limit", ctypes.c_double * OR_MAXB),
    ]


class OrPidGains(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("p", "i", "d", "imax", "imin", "cmdmax", "cmdmin", "offset")]


class OrPidState(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("perr_last", "ierr", "cmd")]


OR_MAXSHAPES = 8
OR_MAXCONTACTS = 8 * OR_MAXSHAPES


class OrFreeModel(ctypes.Structure):
    _fields_ = [
        ("mass", ctypes.c_double),
        ("com", ctypes.c_double * 3),
        ("Ic", ctypes.c_double * 6),
        ("n_shapes", ctypes.c_int32),
        ("ground", ctypes.c_int32),
        ("shape_type", ctypes.c_int32 * OR_MAXSHAPES),
        ("shape_size", (ctypes.c_double * 3) * OR_MAXSHAPES),
        ("shape_R", (ctypes.c_double * 9) * OR_MAXSHAPES),
        ("shape_p", (ctypes.c_double * 3) * OR_MAXSHAPES),
        ("gravity", ctypes.c_double * 3),
        ("mu", ctypes.c_double),
        ("mesh_npts", ctypes.c_int32 * OR_MAXSHAPES),
        ("mesh_pt", ((ctypes.c_double * 3) * 8) * OR_MAXSHAPES),
    ]


class OrFreeState(ctypes.Structure):
    _fields_ = [("p", ctypes.c_double * 3), ("R", ctypes.c_double * 9),
                ("w", ctypes.c_double * 3), ("v", ctypes.c_double * 3)]


OR_MAXFS = 16
OR_MAXFC = 8 * OR_MAXFS
OR_MESH_MAXP = 16   # oracle.h: support points per mesh
OR_WARM_WORDS = 3 * OR_MAXFC + 3 * OR_MAXB   # oracle.h OR_WARM_WORDS


class OrFloatModel(ctypes.Structure):
    _fields_ = [
        ("tree", OrModel),
        ("base_mass", ctypes.c_double),
        ("base_com", ctypes.c_double * 3),
        ("base_Ic", ctypes.c_double * 6),
        ("n_shapes", ctypes.c_int32),
        ("ground", ctypes.c_int32),
        ("shape_body", ctypes.c_int32 * OR_MAXFS),
        ("shape_type", ctypes.c_int32 * OR_MAXFS),
        ("shape_size", (ctypes.c_double * 3) * OR_MAXFS),
        ("shape_R", (ctypes.c_double * 9) * OR_MAXFS),
        ("shape_p", (ctypes.c_double * 3) * OR_MAXFS),
        ("gravity", ctypes.c_double * 3),
        ("mu", ctypes.c_double),
        ("shape_npts", ctypes.c_int32 * OR_MAXFS),
        ("shape_pts", ((ctypes.c_double * 3) * OR_MESH_MAXP) * OR_MAXFS),
    ]


class OrFloatState(ctypes.Structure):
    _fields_ = [("p", ctypes.c_double * 3), ("R", ctypes.c_double * 9), ("V", ctypes.c_double * 6),
                ("q", ctypes.c_double * OR_MAXB), ("qd", ctypes.c_double * OR_MAXB)]


class OrTask(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("steps_per_run", ctypes.c_int32),
        ("max_episode_steps", ctypes.c_int32),
        ("reward_cart_at_center", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("randomize", ctypes.c_int32),
        ("world0", ctypes.c_int32),
        ("mass_low", ctypes.c_double),
        ("mass_high", ctypes.c_double),
        ("gravity_mean", ctypes.c_double),
        ("gravity_std", ctypes.c_double),
        ("gdir", ctypes.c_double * 3),
    ]


def build() -> str:
    """Compile liboracle.so in place (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))
        ):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        D = ctypes.POINTER(ctypes.c_double)
        I32 = ctypes.POINTER(ctypes.c_int32)
        U32 = ctypes.POINTER(ctypes.c_uint32)
        U8 = ctypes.POINTER(ctypes.c_uint8)
        M = ctypes.POINTER(OrModel)
        T = ctypes.POINTER(OrTask)
        L.or_aba.argtypes = [M, D, D, D, ctypes.c_double, D]
        L.or_crba.argtypes = [M, D, D]
        L.or_rnea.argtypes = [M, D, D, D, D]
        L.or_step.argtypes = [M, ctypes.c_double, D, D, I32, D, ctypes.c_int, D, D]
        L.or_step.restype = ctypes.c_int
        L.or_pgs.argtypes = [ctypes.c_int, D, D, D, D, D, ctypes.c_int]
        L.or_free_step.argtypes = [ctypes.POINTER(OrFreeModel), ctypes.c_double, ctypes.POINTER(OrFreeState),
                                   ctypes.c_int, D, D, D, D]
        L.or_free_step.restype = ctypes.c_int
        FM, FS = ctypes.POINTER(OrFloatModel), ctypes.POINTER(OrFloatState)
        L.or_float_step.argtypes = [FM, ctypes.c_double, FS, I32, D, ctypes.c_int, D, D, D, I32]
        L.or_float_step.restype = ctypes.c_int
        L.or_float_step_warm.argtypes = [FM, ctypes.c_double, FS, I32, D, ctypes.c_int, ctypes.c_double, D, D, D,
                                         D, I32]
        L.or_float_step_warm.restype = ctypes.c_int
        L.or_scene_step.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, I32, D, D, ctypes.c_int,
                                    D, I32]
        L.or_scene_step.restype = ctypes.c_int
        L.or_float_dynamics.argtypes = [FM, FS, D, D]
        G, PS = ctypes.POINTER(OrPidGains), ctypes.POINTER(OrPidState)
        L.or_pid_rollout.argtypes = [M, ctypes.c_double, ctypes.c_int, ctypes.c_int, D, D, D, D, ctypes.c_double,
                                     G, PS, ctypes.c_int]
        L.or_float_pid_rollout.argtypes = [FM, ctypes.c_double, ctypes.c_int, FS, D, G, PS, ctypes.c_int]
        L.or_pid_update.argtypes = [ctypes.POINTER(OrPidGains), ctypes.POINTER(OrPidState),
                                    ctypes.c_double, ctypes.c_double]
        L.or_pid_update.restype = ctypes.c_double
        L.or_philox.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, U32]
        L.or_philox_raw.argtypes = [U32, U32, U32]
        L.or_task_reset_state.argtypes = [T, ctypes.c_uint32, ctypes.c_uint32, D, D]
        L.or_task_sample_physics.argtypes = [M, T, ctypes.c_uint32, ctypes.c_uint32, D, D]
        L.or_vec_step.argtypes = [M, T, ctypes.c_int, D, D, ctypes.c_void_p, U32, U32, D, D,
                                  U8, D, ctypes.c_int]
        L.or_vec_reset.argtypes = [M, T, ctypes.c_int, D, D, U32, U32, D]
        L.or_vec_rollout.argtypes = [M, T, ctypes.c_int, ctypes.c_int, D, D, ctypes.c_void_p,
                                     U32, U32, D, D, U8, D, ctypes.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray, ct=ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(ct))


# --------------------------------------------------------------------------
# independent URDF reader
# --------------------------------------------------------------------------

def _rpy(rpy: Sequence[float]) -> np.ndarray:
    r, p, y = rpy
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _quat_wxyz(q: Sequence[float]) -> np.ndarray:
    w, x, y, z = q
    n = math.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / n, x / n, y / n, z / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def _vec(el, attr, default):
    if el is None or el.get(attr) is None:
        return np.array(default, dtype=float)
    return np.array([float(v) for v in el.get(attr).split()], dtype=float)


@dataclass
class _Link:
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    I: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about COM, link frame
    # collision shapes in the link frame: (type 0 box / 1 sphere, size (half extents / radius), R, p)
    shapes: list = field(default_factory=list)


@dataclass
class _Joint:
    name: str
    jtype: str
    parent: str
    child: str
    R: np.ndarray
    p: np.ndarray
    axis: np.ndarray
    lower: float = -math.inf
    upper: float = math.inf
    effort: float = math.inf
    velocity: float = math.inf
    damping: float = 0.0
    friction: float = 0.0


def _merge(parent: _Link, child: _Link, R: np.ndarray, p: np.ndarray) -> _Link:
    """Rigidly merge `child` (pose R, p in parent) into `parent`."""
    shapes = list(parent.shapes) + [(t, sz, R @ SR, R @ sp + p) for (t, sz, SR, sp) in child.shapes]
    out = _merge_inertia(parent, child, R, p)
    out.shapes = shapes
    return out


def _merge_inertia(parent: _Link, child: _Link, R: np.ndarray, p: np.ndarray) -> _Link:
    m = parent.mass + child.mass
    if m <= 0.0:
        return _Link()
    c_child = R @ child.com + p
    com = (parent.mass * parent.com + child.mass * c_child) / m
    I_child = R @ child.I @ R.T

    def shift(I, mass, d):
        return I + mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

    I = shift(parent.I, parent.mass, parent.com - com) + shift(I_child, child.mass, c_child - com)
    return _Link(m, com, I)


@dataclass
class ChainModel:
    joint_names: List[str]
    base_link: str
    model: OrModel
    base_R: np.ndarray
    base_p: np.ndarray
    floating: bool = False
    free: Optional[OrFreeModel] = None
    # collision shapes of the moving bodies: (body, type, size, R, p) in the body frame
    body_shapes: list = field(default_factory=list)
    # the base link's shapes (type, size, R, p) and inertial (mass, com, I about the com)
    base_shapes: list = field(default_factory=list)
    base_inertial: tuple = None

    @property
    def n(self) -> int:
        return self.model.n


def _mat_to_rpy(R: np.ndarray) -> np.ndarray:
    """Inverse of _rpy (R = Rz(y) Ry(p) Rx(r))."""
    p = math.asin(max(-1.0, min(1.0, -R[2, 0])))
    return np.array([math.atan2(R[2, 1], R[2, 2]), p, math.atan2(R[1, 0], R[0, 0])])


def _sdf_pose(el) -> np.ndarray:
    """4x4 homogeneous transform of the <pose> child of `el` (x y z r p y)."""
    T = np.eye(4)
    pe = el.find("pose") if el is not None else None
    if pe is not None and pe.text and pe.text.strip():
        v = [float(x) for x in pe.text.split()]
        T[:3, :3] = _rpy(v[3:6])
        T[:3, 3] = v[:3]
    return T


def _sdf_val(el, path, default):
    e = el.find(path) if el is not None else None
    return float(e.text) if e is not None and e.text and e.text.strip() else default


def _origin(T: np.ndarray) -> str:
    xyz = " ".join(repr(float(v)) for v in T[:3, 3])
    rpy = " ".join(repr(float(v)) for v in _mat_to_rpy(T[:3, :3]))
    return f'<origin xyz="{xyz}" rpy="{rpy}"/>'


def sdf_to_urdf(text: str, pose_xyz=(0.0, 0.0, 0.0), pose_wxyz=(1.0, 0.0, 0.0, 0.0)):
    """Rewrite an SDF <model> as the URDF that describes the same multibody,
    for the oracle's URDF reader (independent of the product's C++ SDF
    front-end).  SDF 1.6 frames: link pose in the model frame, joint pose in
    the child link frame, axis in the joint frame unless
    use_parent_model_frame; <limit>/<dynamics> inside <axis>; sdformat's
    inertial defaults (mass 1, unit inertia).  The URDF child-link frame is
    the joint frame, the root link's frame the model frame.  Returns (urdf,
    xyz, wxyz): the model pose (the insertion pose unless it is the
    identity, World.cpp:169-177)."""
    root = ET.fromstring(text.strip())
    me = root.find("model")
    Tm = _sdf_pose(me)
    if tuple(pose_xyz) == (0.0, 0.0, 0.0) and tuple(pose_wxyz) == (1.0, 0.0, 0.0, 0.0):
        w, x, y, z = _rot_to_quat(Tm[:3, :3])
        pose_xyz, pose_wxyz = tuple(Tm[:3, 3]), (w, x, y, z)
    X = {le.get("name"): _sdf_pose(le) for le in me.findall("link")}
    F = {n: np.eye(4) for n in X}
    F["world"] = np.eye(4)
    jts = me.findall("joint")
    for je in jts:
        F[je.find("child").text.strip()] = X[je.find("child").text.strip()] @ _sdf_pose(je)
    out = [f'<robot name="{me.get("name", "model")}">']
    st = me.find("static")
    static = st is not None and st.text is not None and st.text.strip() in ("1", "true")
    # a static model: its root links are welded to the world at the model frame
    roots = [n for n in X if n not in {je.find("child").text.strip() for je in jts}] if static else []
    if static or any(je.find("parent").text.strip() == "world" for je in jts):
        out.append('<link name="world"/>')
    for n in roots:
        out.append(f'<joint name="__static_{n}" type="fixed"><origin xyz="0 0 0" rpy="0 0 0"/>'
                   f'<parent link="world"/><child link="{n}"/></joint>')
    for le in me.findall("link"):
        n = le.get("name")
        C = np.linalg.inv(F[n]) @ X[n]          # SDF link frame in the URDF link frame
        ine = le.find("inertial")
        Ti = C @ _sdf_pose(ine)
        m = _sdf_val(ine, "mass", 1.0)
        ie = ine.find("inertia") if ine is not None else None
        g = lambda k, d: _sdf_val(ie, k, d)
        I = np.array([[g("ixx", 1.0), g("ixy", 0.0), g("ixz", 0.0)],
                      [g("ixy", 0.0), g("iyy", 1.0), g("iyz", 0.0)],
                      [g("ixz", 0.0), g("iyz", 0.0), g("izz", 1.0)]])
        I = Ti[:3, :3] @ I @ Ti[:3, :3].T
        xyz = " ".join(repr(float(v)) for v in Ti[:3, 3])
        f = lambda v: repr(float(v))
        out.append(f'<link name="{n}"><inertial><origin xyz="{xyz}" rpy="0 0 0"/><mass value="{f(m)}"/>'
                   f'<inertia ixx="{f(I[0,0])}" ixy="{f(I[0,1])}" ixz="{f(I[0,2])}" iyy="{f(I[1,1])}" '
                   f'iyz="{f(I[1,2])}" izz="{f(I[2,2])}"/></inertial>')
        for ce in le.findall("collision"):
            Tc = C @ _sdf_pose(ce)
            box, sph = ce.find("geometry/box/size"), ce.find("geometry/sphere/radius")
            cyl = ce.find("geometry/cylinder")
            if box is not None:
                geo = f'<box size="{box.text.strip()}"/>'
            elif sph is not None:
                geo = f'<sphere radius="{sph.text.strip()}"/>'
            elif cyl is not None:
                geo = (f'<cylinder radius="{_sdf_val(cyl, "radius", 0.5)!r}" '
                       f'length="{_sdf_val(cyl, "length", 1.0)!r}"/>')
            elif ce.find("geometry/mesh/uri") is not None:
                me = ce.find("geometry/mesh")
                sc = me.find("scale")
                geo = (f'<mesh filename="{me.find("uri").text.strip()}" '
                       f'scale="{sc.text.strip() if sc is not None else "1 1 1"}"/>')
            else:
                continue
            out.append(f'<collision>{_origin(Tc)}<geometry>{geo}</geometry></collision>')
        out.append("</link>")
    for je in jts:
        pa, ch, jt = je.find("parent").text.strip(), je.find("child").text.strip(), je.get("type")
        O = np.linalg.inv(F[pa]) @ F[ch]
        if jt == "ball":
            # a spherical pair = three continuous joints about x, y, z of the
            # joint frame at one point, two massless links between them
            # (DART's BallJoint moves the child the same way; only the
            # coordinates differ: rotation vector there, X-Y-Z angles here)
            nm = je.get("name")
            ax = je.find("axis")
            dyn = (f'<dynamics damping="{float(_sdf_val(ax, "dynamics/damping", 0.0))!r}" '
                   f'friction="{float(_sdf_val(ax, "dynamics/friction", 0.0))!r}"/>')
            chain = [(pa, f"{nm}#x", O, "1 0 0"), (f"{nm}#x", f"{nm}#y", np.eye(4), "0 1 0"),
                     (f"{nm}#y", ch, np.eye(4), "0 0 1")]
            for k, (jp, jc, Oj, axs) in enumerate(chain):
                if k < 2:
                    out.append(f'<link name="{jc}"/>')
                out.append(f'<joint name="{nm}#{"xyz"[k]}" type="continuous">{_origin(Oj)}'
                           f'<parent link="{jp}"/><child link="{jc}"/><axis xyz="{axs}"/>'
                           f'<limit effort="inf" velocity="inf"/>{dyn}</joint>')
            continue
        body = [f'<joint name="{je.get("name")}" type="{{TYPE}}">', _origin(O),
                f'<parent link="{pa}"/><child link="{ch}"/>']
        if jt != "fixed":
            ax = je.find("axis")
            xe = ax.find("xyz") if ax is not None else None
            a = np.array([float(v) for v in xe.text.split()]) if xe is not None else np.array([0.0, 0.0, 1.0])
            upm = ax is not None and ax.find("use_parent_model_frame") is not None and \
                ax.find("use_parent_model_frame").text.strip() in ("1", "true")
            if upm or (xe is not None and xe.get("expressed_in") == "__model__"):
                a = F[ch][:3, :3].T @ a
            body.append(f'<axis xyz="{" ".join(repr(float(v)) for v in a)}"/>')
            lo, hi = _sdf_val(ax, "limit/lower", -1e16), _sdf_val(ax, "limit/upper", 1e16)
            eff, vel = _sdf_val(ax, "limit/effort", -1.0), _sdf_val(ax, "limit/velocity", -1.0)
            eff, vel = (eff if eff >= 0 else math.inf), (vel if vel >= 0 else math.inf)
            lim = f'effort="{float(eff)!r}" velocity="{float(vel)!r}"'
            if jt == "revolute" and lo <= -1e16 and hi >= 1e16:
                jt = "continuous"
            if jt == "prismatic":
                lo, hi = (-math.inf if lo <= -1e16 else lo), (math.inf if hi >= 1e16 else hi)
            if jt != "continuous":
                lim += f' lower="{float(lo)!r}" upper="{float(hi)!r}"'
            body.append(f"<limit {lim}/>")
            body.append(f'<dynamics damping="{float(_sdf_val(ax, "dynamics/damping", 0.0))!r}" '
                        f'friction="{float(_sdf_val(ax, "dynamics/friction", 0.0))!r}"/>')
        body[0] = body[0].replace("{TYPE}", jt)
        out.append("".join(body) + "</joint>")
    out.append("</robot>")
    return "".join(out), tuple(pose_xyz), tuple(pose_wxyz)


def _rot_to_quat(R: np.ndarray):
    """Unit quaternion (w, x, y, z) of a rotation matrix (Shepperd)."""
    t = np.trace(R)
    if t > 0:
        s = 2.0 * math.sqrt(1.0 + t)
        return (0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s)
    i = int(np.argmax(np.diag(R)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = 2.0 * math.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k])
    q = [0.0] * 4
    q[0] = (R[k, j] - R[j, k]) / s
    q[1 + i] = 0.25 * s
    q[1 + j] = (R[j, i] + R[i, j]) / s
    q[1 + k] = (R[k, i] + R[i, k]) / s
    return tuple(q)


# --------------------------------------------------------------------------
# mesh collisions (Physics.cpp:897-931 attaches the loaded mesh with the
# collision pose and the SDF <scale>): restated independently of the model
# compiler's csrc/mesh.cpp -- STL (binary / ASCII) and OBJ vertices, the
# support points along 26 fixed directions (8 cube corners, 12 edges, 6 faces;
# the first vertex of the maximum), then along 136 Fibonacci-sphere directions
# while fewer than OR_MESH_MAXP distinct ones were found, and the
# bounding box in the mesh frame (the shape frame is moved to its centre).
# --------------------------------------------------------------------------
_MESH_DIRS = np.array([(-1, -1, -1), (-1, -1, 1), (-1, 1, -1), (-1, 1, 1), (1, -1, -1), (1, -1, 1), (1, 1, -1),
                       (1, 1, 1), (-1, -1, 0), (-1, 1, 0), (1, -1, 0), (1, 1, 0), (-1, 0, -1), (-1, 0, 1),
                       (1, 0, -1), (1, 0, 1), (0, -1, -1), (0, -1, 1), (0, 1, -1), (0, 1, 1), (-1, 0, 0),
                       (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)], dtype=float)


def mesh_vertices(path: str) -> np.ndarray:
    """[V, 3] vertices of an STL (binary or ASCII) or Wavefront OBJ file."""
    low = path.lower()
    with open(path, "rb") as f:
        data = f.read()
    if low.endswith(".stl"):
        if len(data) >= 84:
            n = int(np.frombuffer(data[80:84], dtype="<u4")[0])
            if len(data) == 84 + 50 * n:
                rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)),
                                                               ("a", "<u2")]), count=n)
                return rec["v"].reshape(-1, 3).astype(float)
        toks = data.decode("ascii", "replace").split()
        v = [[float(toks[i + 1]), float(toks[i + 2]), float(toks[i + 3])]
             for i, t in enumerate(toks) if t == "vertex"]
    elif low.endswith(".dae"):
        v = _dae_vertices(path, data)
    elif low.endswith(".obj"):
        v = [[float(x) for x in ln.split()[1:4]] for ln in data.decode("ascii", "replace").splitlines()
             if ln.startswith(("v ", "v\t"))]
    else:
        raise ValueError(f"mesh '{path}': only STL, OBJ and COLLADA collision meshes are supported")
    if not v:
        raise ValueError(f"mesh '{path}' has no vertices")
    return np.array(v, dtype=float)


def _dae_vertices(path: str, data: bytes) -> list:
    """COLLADA as ign-common's ColladaLoader reads it for MeshManager::Load:
    POSITION sources of the geometries the visual scene's nodes instantiate,
    under the node chains' transforms (matrix / translate / rotate in degrees /
    scale, in document order), times <unit meter>; no instancing node: every
    geometry as stored; <up_axis> not applied."""
    root = ET.fromstring(data)
    for el in root.iter():
        el.tag = el.tag.split("}", 1)[-1]
    unit = root.find("asset/unit")
    unit = float(unit.get("meter", "1")) if unit is not None else 1.0
    geoms = []
    for g in root.findall("library_geometries/geometry"):
        me = g.find("mesh")
        vt = me.find("vertices") if me is not None else None
        if vt is None:
            continue
        src = ""
        for i in vt.findall("input"):
            if i.get("semantic") == "POSITION" and i.get("source"):
                src = i.get("source")[1:]
        pts = []
        for so in me.findall("source"):
            fa = so.find("float_array")
            if so.get("id") != src or fa is None:
                continue
            ac = so.find("technique_common/accessor")
            stride = int(float(ac.get("stride", "3"))) if ac is not None else 3
            f = [float(x) for x in (fa.text or "").split()]
            pts += [f[k:k + 3] for k in range(0, len(f) - 2, stride)]
        geoms.append((g.get("id", ""), pts))
    out, inst = [], [False]

    def walk(nd, M):
        for k in nd:
            f = [float(x) for x in (k.text or "").split()]
            T = np.eye(4)
            if k.tag == "matrix" and len(f) == 16:
                T = np.array(f).reshape(4, 4)
            elif k.tag == "translate" and len(f) == 3:
                T[:3, 3] = f
            elif k.tag == "scale" and len(f) == 3:
                T[0, 0], T[1, 1], T[2, 2] = f
            elif k.tag == "rotate" and len(f) == 4:
                n = math.sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2])
                x, y, z, a = f[0] / n, f[1] / n, f[2] / n, f[3] * math.pi / 180.0
                c, s_, t = math.cos(a), math.sin(a), 1.0 - math.cos(a)
                T[:3, :3] = [[t * x * x + c, t * x * y - s_ * z, t * x * z + s_ * y],
                             [t * x * y + s_ * z, t * y * y + c, t * y * z - s_ * x],
                             [t * x * z - s_ * y, t * y * z + s_ * x, t * z * z + c]]
            else:
                continue
            M = M @ T
        for ig in nd.findall("instance_geometry"):
            url = ig.get("url", "")
            for gid, pts in geoms:
                if url and gid == url[1:]:
                    inst[0] = True
                    out.extend((M[:3, :3] @ np.array(p) + M[:3, 3]).tolist() for p in pts)
        for ch in nd.findall("node"):
            walk(ch, M)

    scenes = root.findall("library_visual_scenes/visual_scene")
    want = root.find("scene/instance_visual_scene")
    want = want.get("url", "")[1:] if want is not None else ""
    vs = None
    for v in scenes:
        if vs is None or v.get("id") == want:
            vs = v
    if vs is not None:
        walk(vs, np.eye(4))
    if not inst[0]:
        out = [p for _, pts in geoms for p in pts]
    return [[x * unit for x in p] for p in out]


def resolve_mesh_uri(uri: str, model_dir: str = "") -> str:
    uri = uri.strip()
    if uri.startswith("file://"):
        return uri[7:]
    for pre in ("model://", "package://"):
        if uri.startswith(pre):
            rest = uri[len(pre):]
            for var in ("GZ_SIM_RESOURCE_PATH", "IGN_GAZEBO_RESOURCE_PATH", "SDF_PATH", "ROS_PACKAGE_PATH"):
                for d in os.environ.get(var, "").split(":"):
                    if d and os.path.exists(os.path.join(d, rest)):
                        return os.path.join(d, rest)
            if model_dir and "/" in rest and os.path.exists(os.path.join(model_dir, rest.split("/", 1)[1])):
                return os.path.join(model_dir, rest.split("/", 1)[1])
            raise ValueError(f"cannot resolve mesh URI '{uri}'")
    if uri.startswith("/") or not model_dir:
        return uri
    return os.path.join(model_dir, uri)


def mesh_shape(verts, scale, SR, sp):
    """(3, size, R, p) of a mesh collision: size = [half extents, support
    points (shape frame, flattened)]; p = the bounding-box centre."""
    v = np.asarray(verts, dtype=float) * np.asarray(scale, dtype=float)
    lo, hi = v.min(axis=0), v.max(axis=0)
    c, half = 0.5 * (lo + hi), 0.5 * (hi - lo)
    pick: List[int] = []
    for d in _MESH_DIRS:
        i = int(np.argmax(d[0] * v[:, 0] + d[1] * v[:, 1] + d[2] * v[:, 2]))
        if i not in pick and len(pick) < OR_MESH_MAXP:
            pick.append(i)
    golden = math.pi * (3.0 - math.sqrt(5.0))
    for k in range(136):   # room left: Fibonacci-sphere directions
        if len(pick) >= OR_MESH_MAXP:
            break
        z = 1.0 - (2.0 * k + 1.0) / 136.0
        r, phi = math.sqrt(1.0 - z * z), golden * k
        d = (r * math.cos(phi), r * math.sin(phi), z)
        i = int(np.argmax(d[0] * v[:, 0] + d[1] * v[:, 1] + d[2] * v[:, 2]))
        if i not in pick:
            pick.append(i)
    pts = v[pick] - c
    return (3, np.concatenate([half, pts.reshape(-1)]), SR, np.asarray(sp, dtype=float) + SR @ c)


def _ball_part(chain, i) -> int:
    """1, 2, 3 for the x / y / z part of a ball joint written by sdf_to_urdf, else 0"""
    nm = chain[i].name
    if len(nm) < 3 or nm[-2] != "#" or nm[-1] not in "xyz" or chain[i].jtype != "continuous":
        return 0
    k = "xyz".index(nm[-1])
    base = nm[:-2]
    first = i - k
    if first < 0 or first + 2 >= len(chain):
        return 0
    if all(chain[first + t].name == f"{base}#{'xyz'[t]}" for t in range(3)):
        return k + 1
    return 0


def load_urdf(path_or_string: str, pose_xyz=(0.0, 0.0, 0.0), pose_wxyz=(1.0, 0.0, 0.0, 0.0),
              gravity=(0.0, 0.0, -9.8)) -> ChainModel:
    text = path_or_string
    model_dir = ""
    if not path_or_string.lstrip().startswith("<"):
        with open(path_or_string) as f:
            text = f.read()
        model_dir = os.path.dirname(path_or_string) or "."
    root = ET.fromstring(text.strip())
    if root.tag == "sdf":
        text, pose_xyz, pose_wxyz = sdf_to_urdf(text, pose_xyz, pose_wxyz)
        root = ET.fromstring(text)
    links: Dict[str, _Link] = {}
    for le in root.findall("link"):
        L = _Link()
        ine = le.find("inertial")
        if ine is not None:
            o = ine.find("origin")
            Ro = _rpy(_vec(o, "rpy", [0, 0, 0]))
            L.com = _vec(o, "xyz", [0, 0, 0])
            L.mass = float(ine.find("mass").get("value"))
            ie = ine.find("inertia")
            g = lambda k: float(ie.get(k, "0"))
            Iin = np.array([[g("ixx"), g("ixy"), g("ixz")],
                            [g("ixy"), g("iyy"), g("iyz")],
                            [g("ixz"), g("iyz"), g("izz")]])
            L.I = Ro @ Iin @ Ro.T
        for ce in le.findall("collision"):
            o = ce.find("origin")
            geo = ce.find("geometry")
            box = geo.find("box") if geo is not None else None
            sph = geo.find("sphere") if geo is not None else None
            cyl = geo.find("cylinder") if geo is not None else None
            SR, sp = _rpy(_vec(o, "rpy", [0, 0, 0])), _vec(o, "xyz", [0, 0, 0])
            if box is not None:
                L.shapes.append((0, 0.5 * _vec(box, "size", [0, 0, 0]), SR, sp))
            elif sph is not None:
                L.shapes.append((1, np.array([float(sph.get("radius")), 0.0, 0.0]), SR, sp))
            elif cyl is not None:   # axis z: (radius, half length)
                L.shapes.append((2, np.array([float(cyl.get("radius")), 0.5 * float(cyl.get("length")), 0.0]),
                                 SR, sp))
            elif geo is not None and geo.find("mesh") is not None:
                me = geo.find("mesh")
                verts = mesh_vertices(resolve_mesh_uri(me.get("filename"), model_dir))
                L.shapes.append(mesh_shape(verts, _vec(me, "scale", [1, 1, 1]), SR, sp))
        links[le.get("name")] = L
    joints: List[_Joint] = []
    for je in root.findall("joint"):
        o = je.find("origin")
        ax = _vec(je.find("axis"), "xyz", [1, 0, 0])
        ax = ax / np.linalg.norm(ax)
        J = _Joint(je.get("name"), je.get("type"), je.find("parent").get("link"),
                   je.find("child").get("link"), _rpy(_vec(o, "rpy", [0, 0, 0])),
                   _vec(o, "xyz", [0, 0, 0]), ax)
        lim = je.find("limit")
        if lim is not None:
            J.effort = float(lim.get("effort", "inf"))
            J.velocity = float(lim.get("velocity", "inf"))
            if J.jtype in ("revolute", "prismatic"):
                J.lower = float(lim.get("lower", "0"))
                J.upper = float(lim.get("upper", "0"))
        dyn = je.find("dynamics")
        if dyn is not None:
            J.damping = float(dyn.get("damping", "0"))
            J.friction = float(dyn.get("friction", "0"))
        joints.append(J)

    children = {j.child for j in joints}
    roots = [n for n in links if n not in children]
    assert len(roots) == 1, roots
    root_link = roots[0]
    base_R = _quat_wxyz(pose_wxyz)
    base_p = np.array(pose_xyz, dtype=float)
    floating = root_link != "world"
    if not floating:
        wj = [j for j in joints if j.parent == "world"]
        assert wj, "nothing is attached to the world link"
        if len(wj) == 1 and wj[0].jtype == "fixed":
            base_p = base_p + base_R @ wj[0].p
            base_R = base_R @ wj[0].R
            root_link = wj[0].child
            joints = [j for j in joints if j is not wj[0]]
        # else: the massless world link is the fixed base, its joints hang from the model frame

    # lump fixed joints into their parent (sdformat URDF import behaviour)
    owner = {n: n for n in links}            # link -> body it was lumped into
    off_R = {n: np.eye(3) for n in links}     # pose of link in its owner
    off_p = {n: np.zeros(3) for n in links}
    changed = True
    while changed:
        changed = False
        for j in list(joints):
            if j.jtype != "fixed":
                continue
            po = owner[j.parent]
            R = off_R[j.parent] @ j.R
            p = off_R[j.parent] @ j.p + off_p[j.parent]
            links[po] = _merge(links[po], links[j.child], R, p)
            for ln in links:
                if owner[ln] == j.child:
                    owner[ln] = po
                    off_p[ln] = R @ off_p[ln] + p
                    off_R[ln] = R @ off_R[ln]
            joints.remove(j)
            changed = True
            break

    # moving joints form a tree from the base body, numbered depth-first with
    # children in declaration order (parent index < child index)
    chain: List[_Joint] = []
    parents: List[int] = []

    def visit(link: str, pidx: int) -> None:
        for j in [j for j in joints if owner[j.parent] == link]:
            assert len(chain) < len(joints), "the joints do not form a tree"
            chain.append(j)
            parents.append(pidx)
            visit(j.child, len(chain) - 1)

    visit(root_link, -1)
    assert len(chain) == len(joints), "moving joints not connected to the base"

    M = OrModel()
    M.n = len(chain)
    g_base = base_R.T @ np.array(gravity, dtype=float)
    for k in range(3):
        M.gravity_base[k] = g_base[k]
    for i, j in enumerate(chain):
        E = off_R[j.parent] @ j.R
        r = off_R[j.parent] @ j.p + off_p[j.parent]
        L = links[j.child]
        M.jtype[i] = 0 if j.jtype in ("revolute", "continuous") else 1
        # a ball joint (sdf_to_urdf: `<name>#x`, `#y`, `#z`, consecutive):
        # DART's BallJoint coordinates (oracle.c ball_part)
        part = _ball_part(chain, i)
        if part:
            M.jtype[i] = part << 4
        M.limited[i] = 1 if j.jtype in ("revolute", "prismatic") else 0
        M.parent[i] = parents[i]
        for k in range(9):
            M.E[i][k] = E.flat[k]
        for k in range(3):
            M.r[i][k] = r[k]
            M.axis[i][k] = j.axis[k]
            M.com[i][k] = L.com[k]
        M.mass[i] = L.mass
        Ic = L.I
        for k, v in enumerate([Ic[0, 0], Ic[1, 1], Ic[2, 2], Ic[0, 1], Ic[0, 2], Ic[1, 2]]):
            M.Ic[i][k] = v
        M.damping[i] = j.damping
        M.friction[i] = j.friction
        M.lower[i] = j.lower
        M.upper[i] = j.upper
        M.effort[i] = j.effort
        M.vel_limit[i] = j.velocity
    cm = ChainModel([j.name for j in chain], root_link, M, base_R, base_p)
    cm.floating = floating
    B0 = links[root_link]
    cm.base_shapes = list(B0.shapes)
    cm.base_inertial = (B0.mass, np.array(B0.com, dtype=float), np.array(B0.I, dtype=float))
    for i, j in enumerate(chain):
        for (t, sz, SR, sp) in links[j.child].shapes:
            cm.body_shapes.append((i, t, sz, SR, sp))
    if floating:
        B = links[root_link]
        F = OrFreeModel()
        F.mass = B.mass
        for k in range(3):
            F.com[k] = B.com[k]
            F.gravity[k] = gravity[k]
        for k, v in enumerate([B.I[0, 0], B.I[1, 1], B.I[2, 2], B.I[0, 1], B.I[0, 2], B.I[1, 2]]):
            F.Ic[k] = v
        solid = []   # a mesh splits into entries of <= 8 support points (one slot block each)
        for (t, sz, SR, sp) in B.shapes:
            if t != 3:
                solid.append((t, sz, SR, sp))
                continue
            pts = np.asarray(sz[3:]).reshape(-1, 3)
            for c0 in range(0, len(pts), 8):
                solid.append((3, np.concatenate([sz[:3], pts[c0:c0 + 8].reshape(-1)]), SR, sp))
        assert len(solid) <= OR_MAXSHAPES
        F.n_shapes = len(solid)
        for i, (t, sz, SR, sp) in enumerate(solid):
            if t == 3:
                pts = np.asarray(sz[3:]).reshape(-1, 3)
                F.mesh_npts[i] = len(pts)
                for c, pt in enumerate(pts):
                    for k in range(3):
                        F.mesh_pt[i][c][k] = pt[k]
            F.shape_type[i] = t
            for k in range(3):
                F.shape_size[i][k] = sz[k]
                F.shape_p[i][k] = sp[k]
            for k in range(9):
                F.shape_R[i][k] = SR.flat[k]
        F.mu = 1.0
        cm.free = F
    return cm


# --------------------------------------------------------------------------
# thin wrappers
# --------------------------------------------------------------------------

def aba(cm: ChainModel, q, qd, tau, dt_implicit=0.0) -> np.ndarray:
    q, qd, tau = (np.ascontiguousarray(x, dtype=np.float64) for x in (q, qd, tau))
    out = np.zeros(cm.n)
    lib().or_aba(ctypes.byref(cm.model), _p(q), _p(qd), _p(tau), dt_implicit, _p(out))
    return out


def crba(cm: ChainModel, q) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.float64)
    out = np.zeros((cm.n, cm.n))
    lib().or_crba(ctypes.byref(cm.model), _p(q), _p(out))
    return out


def rnea(cm: ChainModel, q, qd, qdd) -> np.ndarray:
    q, qd, qdd = (np.ascontiguousarray(x, dtype=np.float64) for x in (q, qd, qdd))
    out = np.zeros(cm.n)
    lib().or_rnea(ctypes.byref(cm.model), _p(q), _p(qd), _p(qdd), _p(out))
    return out


def step(cm: ChainModel, dt, q, qd, mode, cmd, pgs_iters=50):
    """One engine step; returns (q, qd, qdd, force, active_rows)."""
    q = np.array(q, dtype=np.float64)
    qd = np.array(qd, dtype=np.float64)
    mode = np.ascontiguousarray(mode, dtype=np.int32)
    cmd = np.ascontiguousarray(cmd, dtype=np.float64)
    qdd = np.zeros(cm.n)
    f = np.zeros(cm.n)
    nr = lib().or_step(ctypes.byref(cm.model), dt, _p(q), _p(qd), _p(mode, ctypes.c_int32),
                       _p(cmd), pgs_iters, _p(qdd), _p(f))
    return q, qd, qdd, f, nr


# scenario::core::PID defaults (cpp/scenario/core/include/scenario/core/utils/
# utils.h PID struct): cmd / integral limits open; Joint.cpp:63 DefaultPID is
# ignition::math::PID(1, 0.1, 0.01, -1, 0, -1, 0, 0) (empty ranges: no clamp).
_BIG = float(np.finfo(np.float64).max)


def pid_gains(p, i, d, imax=_BIG, imin=-_BIG, cmdmax=_BIG, cmdmin=-_BIG, offset=0.0) -> OrPidGains:
    return OrPidGains(p, i, d, imax, imin, cmdmax, cmdmin, offset)


DEFAULT_PID = (1.0, 0.1, 0.01, -1.0, 0.0, -1.0, 0.0, 0.0)


def pid_update(g: OrPidGains, s: OrPidState, err: float, dt: float) -> float:
    return lib().or_pid_update(ctypes.byref(g), ctypes.byref(s), err, dt)


IDLE, FORCE_MODE, VELOCITY_FOLLOWER_DART, POSITION, VELOCITY = 1, 2, 4, 5, 3


class ScenarioWorld:
    """fp64 restatement of one world of GazeboSimulator.run() with the
    ScenarI/O Physics + JointController systems (the checker of the HIP
    scenario kernel).  Per run, for every substep:
      JointController::PreUpdate (JointController.cpp:114-287): period gating
        on the simulated time in integer nanoseconds; Position / Velocity
        joints run the PID on error = current - target (:308) and write the
        force target; VelocityFollowerDart re-issues the velocity command;
      Physics::UpdatePhysics: SetForce (effort clip in the engine) / servo;
      engine step (or_step); UpdateSim zero-fills the force command
        (Physics.cpp:2250-2254), so a Force-mode target acts on one substep.
    Resets apply at the start of the next run (velocity, then position)."""

    def __init__(self, cm: ChainModel, dt: float, steps_per_run: int = 1, pgs_iters: int = 50):
        n = cm.n
        self.cm, self.dt, self.spr, self.pgs = cm, dt, steps_per_run, pgs_iters
        self.dt_ns = int(round(dt * 1e9))
        self.q, self.qd, self.qdd = np.zeros(n), np.zeros(n), np.zeros(n)
        self.mode = [IDLE] * n
        self.force = np.zeros(n)
        self.ptgt, self.vtgt = np.zeros(n), np.zeros(n)
        self.gains = [OrPidGains(*DEFAULT_PID) for _ in range(n)]
        self.state = [OrPidState() for _ in range(n)]
        self.period_ns = 2 ** 63 - 1          # Model.cpp:181-185: never, after the first update
        self.prev_ns = 0
        self.controller = False                # JointController inserted (Joint.cpp:376-404)
        self.iterations = 0
        self.reset_q, self.reset_qd = {}, {}

    # -- component writes (Joint.cpp) --
    def set_mode(self, dof, mode):
        self.mode[dof] = mode
        self.force[dof] = 0.0
        if mode in (POSITION,):
            self.ptgt[dof] = self.q[dof]
        if mode in (VELOCITY, VELOCITY_FOLLOWER_DART):
            self.vtgt[dof] = self.qd[dof]
        if mode in (POSITION, VELOCITY, VELOCITY_FOLLOWER_DART):
            self.controller = True
        self.state[dof] = OrPidState()

    def set_pid(self, dof, p, i, d, imax=_BIG, imin=-_BIG, cmdmax=_BIG, cmdmin=-_BIG, offset=0.0):
        e = self.cm.model.effort[dof]
        if cmdmin < -e or cmdmax > e:          # Joint.cpp:504-513
            cmdmin, cmdmax = -e, e
        self.gains[dof] = OrPidGains(p, i, d, imax, imin, cmdmax, cmdmin, offset)
        self.state[dof] = OrPidState()

    def reset_position(self, dof, v):
        self.reset_q[dof] = v
        self.state[dof] = OrPidState()

    def reset_velocity(self, dof, v):
        self.reset_qd[dof] = v
        self.state[dof] = OrPidState()

    def run(self, paused=False):
        for d, v in self.reset_qd.items():
            self.qd[d] = v
        for d, v in self.reset_q.items():
            self.q[d] = v
        self.reset_q, self.reset_qd = {}, {}
        if paused:
            self.force[:] = 0.0
            return
        n = self.cm.n
        for s in range(self.spr):
            sim_ns = (self.iterations + s + 1) * self.dt_ns
            compute = False
            if self.controller:
                elapsed = self.period_ns if self.prev_ns == 0 else sim_ns - self.prev_ns
                if elapsed >= self.period_ns:
                    self.prev_ns = sim_ns
                    compute = True
            mode = np.zeros(n, dtype=np.int32)
            cmd = np.zeros(n)
            for d in range(n):
                m = self.mode[d]
                if m in (POSITION, VELOCITY):
                    if compute:
                        cur = self.q[d] if m == POSITION else self.qd[d]
                        tgt = self.ptgt[d] if m == POSITION else self.vtgt[d]
                        pid_update(self.gains[d], self.state[d], cur - tgt, self.dt)
                    mode[d], cmd[d] = FORCE, self.state[d].cmd
                elif m == VELOCITY_FOLLOWER_DART:
                    mode[d], cmd[d] = SERVO, self.vtgt[d]
                elif m == FORCE_MODE:
                    mode[d], cmd[d] = FORCE, (self.force[d] if s == 0 else 0.0)
                else:
                    mode[d] = PASSIVE
            self.q, self.qd, self.qdd, _, _ = step(self.cm, self.dt, self.q, self.qd, mode, cmd, self.pgs)
        self.force[:] = 0.0
        self.iterations += self.spr


class FreeWorld:
    """fp64 floating rigid body on the ground plane (or_free_step): DART
    FreeJoint dynamics + ContactConstraint rows, the checker of the HIP
    free-body kernel.  Pose (p, R); twist in the body frame (w, v)."""

    def __init__(self, cm: ChainModel, dt: float = 1e-3, ground: bool = True, mu: float = 1.0,
                 pgs_iters: int = 100):
        assert cm.floating and cm.n == 0
        self.m = OrFreeModel()
        ctypes.pointer(self.m)[0] = cm.free
        self.m.ground = 1 if ground else 0
        self.m.mu = mu
        self.dt, self.pgs = dt, pgs_iters
        self.s = OrFreeState()
        self.set_pose(cm.base_p, cm.base_R)
        self.contacts = []

    def set_pose(self, p, R):
        for k in range(3):
            self.s.p[k] = p[k]
        for k in range(9):
            self.s.R[k] = np.asarray(R).flat[k]

    def set_twist(self, w_body, v_body):
        for k in range(3):
            self.s.w[k] = w_body[k]
            self.s.v[k] = v_body[k]

    @property
    def p(self):
        return np.array(self.s.p[:])

    @property
    def R(self):
        return np.array(self.s.R[:]).reshape(3, 3)

    @property
    def twist(self):
        return np.array(self.s.w[:]), np.array(self.s.v[:])

    def step(self):
        cp, cn, cf, cd = (np.zeros(3 * OR_MAXCONTACTS), np.zeros(3 * OR_MAXCONTACTS),
                          np.zeros(3 * OR_MAXCONTACTS), np.zeros(OR_MAXCONTACTS))
        nc = lib().or_free_step(ctypes.byref(self.m), self.dt, ctypes.byref(self.s), self.pgs,
                                _p(cp), _p(cn), _p(cf), _p(cd))
        self.contacts = [(cp[3 * i:3 * i + 3].copy(), cn[3 * i:3 * i + 3].copy(), cf[3 * i:3 * i + 3].copy(),
                          float(cd[i])) for i in range(nc)]
        return nc


def _mesh_points_as_spheres(shapes):
    """(body, type, size, R, p) list with every mesh replaced by zero-radius
    spheres at its support points (mw_sim's articulated floating models: the
    same ground contacts as the scene's mesh slots)"""
    out = []
    for (b, t, sz, SR, sp) in shapes:
        if t != 3:
            out.append((b, t, sz, SR, sp))
            continue
        for pt in np.asarray(sz[3:]).reshape(-1, 3):
            out.append((b, 1, np.zeros(3), np.eye(3), np.asarray(sp, dtype=float) + np.asarray(SR) @ pt))
    return out


class FloatWorld:
    """fp64 articulated floating-base model on the ground plane (or_float_step):
    DART FreeJoint root + the joint tree, dense CRBA/RNEA dynamics, contact
    rows on any body and joint rows -- the checker of the HIP floating-tree
    kernel.  Base pose (p, R), base twist V = [w; v] in the base frame."""

    def __init__(self, cm: ChainModel, dt: float = 1e-3, ground: bool = True, mu: float = 1.0,
                 pgs_iters: int = 100, pgs_tol: float = 0.0, warm_start: bool = False):
        assert cm.floating
        m = OrFloatModel()
        ctypes.pointer(m.tree)[0] = cm.model
        F = cm.free
        m.base_mass = F.mass
        for k in range(3):
            m.base_com[k] = F.com[k]
            m.gravity[k] = F.gravity[k]
        for k in range(6):
            m.base_Ic[k] = F.Ic[k]
        shapes = _mesh_points_as_spheres([(-1, *sh) for sh in cm.base_shapes] + list(cm.body_shapes))
        assert len(shapes) <= OR_MAXFS
        m.n_shapes = len(shapes)
        for i, (b, t, sz, SR, sp) in enumerate(shapes):
            m.shape_body[i] = b
            m.shape_type[i] = t
            for k in range(3):
                m.shape_size[i][k] = sz[k]
                m.shape_p[i][k] = sp[k]
            for k in range(9):
                m.shape_R[i][k] = np.asarray(SR).flat[k]
        m.ground = 1 if ground else 0
        m.mu = mu
        self.m, self.cm = m, cm
        self.dt, self.pgs = dt, pgs_iters
        # the kernels' solver options (or_float_step_warm): tolerance exit and
        # warm start from the previous step's impulses (by contact slot / joint row)
        self.pgs_tol = pgs_tol
        self.warm = np.zeros(OR_WARM_WORDS) if warm_start else None
        self.s = OrFloatState()
        self.set_pose(cm.base_p, cm.base_R)
        self.mode = np.zeros(cm.n, dtype=np.int32)
        self.cmd = np.zeros(cm.n)
        self.contacts = []

    def set_pose(self, p, R):
        for k in range(3):
            self.s.p[k] = p[k]
        for k in range(9):
            self.s.R[k] = np.asarray(R).flat[k]

    def set_twist(self, w_body, v_body):
        for k in range(3):
            self.s.V[k] = w_body[k]
            self.s.V[3 + k] = v_body[k]

    def set_joints(self, q, qd):
        for i in range(self.cm.n):
            self.s.q[i] = q[i]
            self.s.qd[i] = qd[i]

    @property
    def p(self):
        return np.array(self.s.p[:])

    @property
    def R(self):
        return np.array(self.s.R[:]).reshape(3, 3)

    @property
    def V(self):
        return np.array(self.s.V[:])

    @property
    def q(self):
        return np.array(self.s.q[:self.cm.n])

    @property
    def qd(self):
        return np.array(self.s.qd[:self.cm.n])

    def dynamics(self):
        nv = 6 + self.cm.n
        M, h = np.zeros(nv * nv), np.zeros(nv)
        lib().or_float_dynamics(ctypes.byref(self.m), ctypes.byref(self.s), _p(M), _p(h))
        return M.reshape(nv, nv), h

    def step(self, mode=None, cmd=None):
        mode = self.mode if mode is None else np.ascontiguousarray(mode, dtype=np.int32)
        cmd = self.cmd if cmd is None else np.ascontiguousarray(cmd, dtype=float)
        cp, cf, cd = np.zeros(3 * OR_MAXFC), np.zeros(3 * OR_MAXFC), np.zeros(OR_MAXFC)
        cb = np.zeros(OR_MAXFC, dtype=np.int32)
        if self.pgs_tol > 0.0 or self.warm is not None:
            nc = lib().or_float_step_warm(ctypes.byref(self.m), self.dt, ctypes.byref(self.s),
                                          _p(mode, ctypes.c_int32), _p(cmd), self.pgs, self.pgs_tol,
                                          _p(self.warm) if self.warm is not None else None,
                                          _p(cp), _p(cf), _p(cd), _p(cb, ctypes.c_int32))
        else:
            nc = lib().or_float_step(ctypes.byref(self.m), self.dt, ctypes.byref(self.s),
                                     _p(mode, ctypes.c_int32), _p(cmd), self.pgs, _p(cp), _p(cf), _p(cd),
                                     _p(cb, ctypes.c_int32))
        self.contacts = [(cp[3 * i:3 * i + 3].copy(), cf[3 * i:3 * i + 3].copy(), float(cd[i]), int(cb[i]))
                         for i in range(nc)]
        return nc


OR_SC_MAXM = 8
OR_SC_MAXC = 160


class OrSceneModel(ctypes.Structure):
    _fields_ = [("n_models", ctypes.c_int32), ("ground", ctypes.c_int32), ("mu", ctypes.c_double),
                ("gravity", ctypes.c_double * 3), ("floating", ctypes.c_int32 * OR_SC_MAXM),
                ("pad_", ctypes.c_int32), ("model", OrFloatModel * OR_SC_MAXM)]


class OrSceneState(ctypes.Structure):
    _fields_ = [("s", OrFloatState * OR_SC_MAXM)]


def collide(type_a, size_a, c_a, R_a, type_b, size_b, c_b, R_b):
    """or_collide: (normal from B into A, points [k][3], depths [k])."""
    n, pts, dep = np.zeros(3), np.zeros(12), np.zeros(4)
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=float).reshape(-1))
    k = lib().or_collide(int(type_a), _p(f(list(size_a) + [0] * (3 - len(size_a)))), _p(f(c_a)), _p(f(R_a)),
                         int(type_b), _p(f(list(size_b) + [0] * (3 - len(size_b)))), _p(f(c_b)), _p(f(R_b)),
                         _p(n), _p(pts), _p(dep))
    return n, pts[:3 * k].reshape(k, 3), dep[:k]


OR_HULL_MAXF, OR_HULL_MAXE = 32, 48


class OrHullInfo(ctypes.Structure):
    _fields_ = [("nv", ctypes.c_int32), ("nf", ctypes.c_int32), ("ne", ctypes.c_int32),
                ("n", (ctypes.c_double * 3) * OR_HULL_MAXF), ("d", ctypes.c_double * OR_HULL_MAXF),
                ("fnv", ctypes.c_int32 * OR_HULL_MAXF), ("fv", (ctypes.c_int32 * 16) * OR_HULL_MAXF),
                ("e", (ctypes.c_int32 * 2) * OR_HULL_MAXE), ("ef", (ctypes.c_int32 * 2) * OR_HULL_MAXE)]


def hull(points):
    """or_hull_build: the convex hull the mesh narrow phase uses for these
    support points -- dict(n [F, 3] outward normals, d [F], faces: list of
    vertex-index polygons (counter-clockwise seen from outside), edges [E, 2],
    edge_faces [E, 2]); None for a flat point set."""
    pts = np.ascontiguousarray(np.asarray(points, dtype=float).reshape(-1, 3))
    info = OrHullInfo()
    f = lib().or_hull_build
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(OrHullInfo)]
    nf = f(len(pts), _p(pts), ctypes.byref(info))
    if nf <= 0:
        return None
    return dict(n=np.array([info.n[i][:] for i in range(nf)]), d=np.array(info.d[:nf]),
                faces=[list(info.fv[i][:info.fnv[i]]) for i in range(nf)],
                edges=np.array([info.e[i][:] for i in range(info.ne)]),
                edge_faces=np.array([info.ef[i][:] for i in range(info.ne)]))


def collide_hull(type_a, size_a, pts_a, c_a, R_a, type_b, size_b, pts_b, c_b, R_b):
    """or_collide_hull (a mesh against a box or a mesh): (normal from B into
    A, points [k][3], depths [k]); pts_*: a mesh's support points (shape frame)."""
    n, pts, dep = np.zeros(3), np.zeros(12), np.zeros(4)
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=float).reshape(-1))
    pa = f(pts_a if pts_a is not None else np.zeros(3))
    pb = f(pts_b if pts_b is not None else np.zeros(3))
    k = lib().or_collide_hull(int(type_a), _p(f(size_a)), len(pa) // 3, _p(pa), _p(f(c_a)), _p(f(R_a)),
                              int(type_b), _p(f(size_b)), len(pb) // 3, _p(pb), _p(f(c_b)), _p(f(R_b)),
                              _p(n), _p(pts), _p(dep))
    return n, pts[:3 * k].reshape(k, 3), dep[:k]


class SceneWorld:
    """fp64 scene (or_scene_step): several models in one world, each on a
    fixed or floating base, ground plane, shape-pair contacts between models,
    external world wrenches.  models: list of ChainModel (from load_urdf with
    the insertion pose); a model is floating when its URDF root is not
    attached to "world"."""

    def __init__(self, models, dt=1e-3, ground=True, mu=1.0, pgs_iters=50, gravity=(0.0, 0.0, -9.8)):
        assert len(models) <= OR_SC_MAXM
        sm = OrSceneModel()
        sm.n_models = len(models)
        sm.ground = 1 if ground else 0
        sm.mu = mu
        for k in range(3):
            sm.gravity[k] = gravity[k]
        self.st = OrSceneState()
        for m, cm in enumerate(models):
            sm.floating[m] = 1 if cm.floating else 0
            fm = sm.model[m]
            ctypes.pointer(fm.tree)[0] = cm.model
            mass, com, I = cm.base_inertial
            fm.base_mass = mass
            for k in range(3):
                fm.base_com[k] = com[k]
                fm.gravity[k] = gravity[k]
            for k, v in enumerate([I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]):
                fm.base_Ic[k] = v
            shapes = [(-1, t, sz, SR, sp) for (t, sz, SR, sp) in cm.base_shapes] + list(cm.body_shapes)
            assert len(shapes) <= OR_MAXFS
            fm.n_shapes = len(shapes)
            for i, (b, t, sz, SR, sp) in enumerate(shapes):
                fm.shape_body[i] = b
                fm.shape_type[i] = t
                for k in range(3):
                    fm.shape_size[i][k] = sz[k]
                    fm.shape_p[i][k] = sp[k]
                for k in range(9):
                    fm.shape_R[i][k] = np.asarray(SR).flat[k]
                if t == 3:   # mesh: sz = half extents, then the support points
                    pts = np.asarray(sz[3:]).reshape(-1, 3)
                    fm.shape_npts[i] = len(pts)
                    for c, pt in enumerate(pts):
                        for k in range(3):
                            fm.shape_pts[i][c][k] = pt[k]
            s0 = self.st.s[m]
            for k in range(3):
                s0.p[k] = cm.base_p[k]
            for k in range(9):
                s0.R[k] = np.asarray(cm.base_R).flat[k]
        self.sm, self.models = sm, list(models)
        self.dt, self.pgs = dt, pgs_iters
        self.mode = np.zeros((OR_SC_MAXM, OR_MAXB), dtype=np.int32)
        self.cmd = np.zeros((OR_SC_MAXM, OR_MAXB))
        self.wrench = np.zeros((OR_SC_MAXM, 1 + OR_MAXB, 6))
        self.contacts = []

    def state(self, m):
        return self.st.s[m]

    def set_pose(self, m, p, R):
        s = self.st.s[m]
        for k in range(3):
            s.p[k] = p[k]
        for k in range(9):
            s.R[k] = np.asarray(R).flat[k]

    def set_twist(self, m, w_body, v_body):
        s = self.st.s[m]
        for k in range(3):
            s.V[k] = w_body[k]
            s.V[3 + k] = v_body[k]

    def set_joints(self, m, q, qd):
        s = self.st.s[m]
        for i in range(self.models[m].n):
            s.q[i] = q[i]
            s.qd[i] = qd[i]

    def p(self, m):
        return np.array(self.st.s[m].p[:])

    def R(self, m):
        return np.array(self.st.s[m].R[:]).reshape(3, 3)

    def V(self, m):
        return np.array(self.st.s[m].V[:])

    def q(self, m):
        return np.array(self.st.s[m].q[:self.models[m].n])

    def qd(self, m):
        return np.array(self.st.s[m].qd[:self.models[m].n])

    def step(self):
        c = np.zeros((OR_SC_MAXC, 10))
        who = np.zeros((OR_SC_MAXC, 4), dtype=np.int32)
        nc = lib().or_scene_step(ctypes.byref(self.sm), self.dt, ctypes.byref(self.st),
                                 _p(np.ascontiguousarray(self.mode), ctypes.c_int32),
                                 _p(np.ascontiguousarray(self.cmd)), _p(np.ascontiguousarray(self.wrench)),
                                 self.pgs, _p(c), _p(who, ctypes.c_int32))
        self.contacts = [(c[i].copy(), tuple(int(v) for v in who[i])) for i in range(nc)]
        return nc


PGS_CONVERGED = -1   # sweep budget: run the boxed LCP to its fixed point (oracle.h)


def pgs_stats():
    """(sweeps, last sweep's largest impulse change) of the latest LCP solve."""
    n, d = ctypes.c_int(0), ctypes.c_double(0.0)
    lib().or_pgs_stats(ctypes.byref(n), ctypes.byref(d))
    return n.value, d.value


def pid_rollout(cm: ChainModel, q, qd, q0, amp, freq, gains, T, dt=1e-3, pgs_iters=20, states=None):
    """T steps of W fixed-base worlds under the JointController PID (or_pid_rollout,
    C; releases the GIL): q, qd [W, n] updated in place; targets q0 + amp sin(2 pi f t)."""
    W, n = q.shape
    g = (OrPidGains * n)(*gains)
    st = states if states is not None else (OrPidState * (W * n))()
    lib().or_pid_rollout(ctypes.byref(cm.model), dt, W, T, _p(q), _p(qd), _p(np.ascontiguousarray(q0)),
                         _p(np.ascontiguousarray(amp, dtype=float)), freq, g, st, pgs_iters)
    return st


def float_pid_rollout(fw: "FloatWorld", target, gains, T, states=None):
    """T steps of one FloatWorld under the PID hold (or_float_pid_rollout, C)."""
    n = fw.cm.n
    g = (OrPidGains * n)(*gains)
    st = states if states is not None else (OrPidState * n)()
    lib().or_float_pid_rollout(ctypes.byref(fw.m), fw.dt, T, ctypes.byref(fw.s),
                               _p(np.ascontiguousarray(target, dtype=float)), g, st, fw.pgs)
    return st


def lcp_last():
    """The latest floating-tree LCP the oracle solved (test hook): dict of the
    Delassus matrix A (with CFM), rhs b, bounds lo/hi (friction rows: +-inf,
    bounded by mu x_normal), row kinds (0 normal, 1 friction, 2 box), mu and
    the solution x the step used, the rows' warm-record identities `wid`, the
    stage-1 impulses `x1` and the b-term magnitudes `bscale`
    (oracle.h or_lcp_last_rows); None when the step had no rows."""
    cap = 3 * 8 * 16 + 3 * 48
    A = np.zeros(cap * cap)
    b, lo, hi, x = (np.zeros(cap) for _ in range(4))
    kind = np.zeros(cap, np.int32)
    mu = ctypes.c_double(0.0)
    n = lib().or_lcp_last(cap, _p(A), _p(b), _p(lo), _p(hi), kind.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          _p(x), ctypes.byref(mu))
    if n <= 0:
        return None
    wid = np.zeros(cap, np.int32)
    x1, bscale = np.zeros(cap), np.zeros(cap)
    f = lib().or_lcp_last_rows
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double),
                  ctypes.POINTER(ctypes.c_double)]
    assert f(cap, wid.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _p(x1), _p(bscale)) == n
    return dict(A=A[:n * n].reshape(n, n).copy(), b=b[:n].copy(), lo=lo[:n].copy(), hi=hi[:n].copy(),
                kind=kind[:n].copy(), mu=mu.value, x=x[:n].copy(), wid=wid[:n].copy(), x1=x1[:n].copy(),
                bscale=bscale[:n].copy())


def set_lcp_perturbation(eps: float, seed: int = 0) -> None:
    """Conditioning probe (oracle.c or_set_lcp_perturbation): every exact LCP
    solve sees A with its symmetric entry pairs scaled by (1 + eps u), u in
    [-1, 1); eps = 0 turns it off."""
    f = lib().or_set_lcp_perturbation
    f.argtypes = [ctypes.c_double, ctypes.c_uint64]
    f(float(eps), int(seed))


def pgs(A, b, lo, hi, iters=100):
    A = np.ascontiguousarray(A, dtype=np.float64)
    b, lo, hi = (np.ascontiguousarray(x, dtype=np.float64) for x in (b, lo, hi))
    x = np.zeros(len(b))
    lib().or_pgs(len(b), _p(A), _p(b), _p(lo), _p(hi), _p(x), iters)
    return x


def philox(seed: int, world: int, episode: int) -> np.ndarray:
    out = (ctypes.c_uint32 * 4)()
    lib().or_philox(seed, world, episode, out)
    return np.array(list(out), dtype=np.uint32)


def philox_raw(ctr, key) -> np.ndarray:
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().or_philox_raw(_p(c, ctypes.c_uint32), _p(k, ctypes.c_uint32), _p(out, ctypes.c_uint32))
    return out


def make_task(kind: int, dt: float = 1e-3, steps_per_run: int = 1, max_episode_steps: int = 5000,
              reward_cart_at_center: bool = True, seed: int = 42, randomize: int = 0,
              mass_range=(-0.2, 0.2), gravity_normal=(-9.8, 0.2), gdir=(0.0, 0.0, 1.0)) -> OrTask:
    t = OrTask()
    t.randomize = randomize
    t.mass_low, t.mass_high = mass_range
    t.gravity_mean, t.gravity_std = gravity_normal
    for k in range(3):
        t.gdir[k] = gdir[k]
    t.kind = kind
    t.dt = dt
    t.steps_per_run = steps_per_run
    t.max_episode_steps = max_episode_steps
    t.reward_cart_at_center = 1 if reward_cart_at_center else 0
    t.seed = seed
    return t


def sample_physics(cm: ChainModel, task: OrTask, world: int, episode: int):
    """(masses [n], gravity z) of one world's episode."""
    m = np.zeros(cm.n)
    gz = ctypes.c_double()
    lib().or_task_sample_physics(ctypes.byref(cm.model), ctypes.byref(task), world, episode, _p(m),
                                 ctypes.byref(gz))
    return m, gz.value


def n_obs(kind: int) -> int:
    return 3 if kind == TASK_PENDULUM_SWINGUP else 4


class VecEnv:
    """fp64 batched env (SoA state) -- the CPU checker of the HIP VecEnv."""

    def __init__(self, cm: ChainModel, task: OrTask, W: int, pgs_iters: int = 50):
        self.cm, self.task, self.W, self.pgs_iters = cm, task, W, pgs_iters
        n = cm.n
        self.q = np.zeros(n * W)
        self.qd = np.zeros(n * W)
        self.episode = np.zeros(W, dtype=np.uint32)
        self.steps = np.zeros(W, dtype=np.uint32)
        no = n_obs(task.kind)
        self.obs = np.zeros(W * no)
        self.reward = np.zeros(W)
        self.done = np.zeros(W, dtype=np.uint8)
        self.terminal_obs = np.zeros(W * no)

    def reset(self):
        lib().or_vec_reset(ctypes.byref(self.cm.model), ctypes.byref(self.task), self.W,
                           _p(self.q), _p(self.qd), _p(self.episode, ctypes.c_uint32),
                           _p(self.steps, ctypes.c_uint32), _p(self.obs))
        return self.obs.reshape(self.W, -1).copy()

    def _actions(self, actions):
        if self.task.kind == TASK_CARTPOLE_DISCRETE:
            return np.ascontiguousarray(actions, dtype=np.int32)
        return np.ascontiguousarray(actions, dtype=np.float64)

    def step(self, actions):
        a = self._actions(actions)
        lib().or_vec_step(ctypes.byref(self.cm.model), ctypes.byref(self.task), self.W,
                          _p(self.q), _p(self.qd), a.ctypes.data_as(ctypes.c_void_p),
                          _p(self.episode, ctypes.c_uint32), _p(self.steps, ctypes.c_uint32),
                          _p(self.obs), _p(self.reward), _p(self.done, ctypes.c_uint8),
                          _p(self.terminal_obs), self.pgs_iters)
        return (self.obs.reshape(self.W, -1).copy(), self.reward.copy(), self.done.astype(bool),
                self.terminal_obs.reshape(self.W, -1).copy())

    def rollout(self, actions):
        """T steps in C (actions [T, W]); used for the CPU baseline timing."""
        a = self._actions(actions)
        T = a.shape[0]
        lib().or_vec_rollout(ctypes.byref(self.cm.model), ctypes.byref(self.task), self.W, T,
                             _p(self.q), _p(self.qd), a.ctypes.data_as(ctypes.c_void_p),
                             _p(self.episode, ctypes.c_uint32), _p(self.steps, ctypes.c_uint32),
                             _p(self.obs), _p(self.reward), _p(self.done, ctypes.c_uint8),
                             _p(self.terminal_obs), self.pgs_iters)
