"""ctypes binding of ``libmwstep.so`` (the C ABI declared in ``include/mwstep.h``).

The library is built in-tree by ``make -C gym-ignition_amd`` (hipcc, gfx950).
There is no CPU fallback: if the shared object is missing, importing the
product raises immediately, and every compute entry point reports HIP errors
as ``RuntimeError``.
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get("MWSTEP_LIB", os.path.join(_PKG_ROOT, "libmwstep.so"))

MW_OK = 0
MW_EINVAL, MW_ESTATE, MW_EPARSE, MW_EHIP, MW_ENOTFOUND, MW_ECAPACITY, MW_EDIVERGED = 1, 2, 3, 4, 5, 6, 7

MODE_INVALID, MODE_IDLE, MODE_FORCE, MODE_VELOCITY = 0, 1, 2, 3
MODE_VELOCITY_FOLLOWER_DART, MODE_POSITION, MODE_POSITION_INTERPOLATED = 4, 5, 6

JOINT_INVALID, JOINT_FIXED, JOINT_REVOLUTE, JOINT_PRISMATIC, JOINT_BALL = 0, 1, 2, 3, 4

LCP_PGS = 0
LCP_EXACT = 1

PARAM_COULOMB_FRICTION = 0
PARAM_VISCOUS_FRICTION = 1
PARAM_MAX_GENERALIZED_FORCE = 2
PARAM_POSITION_LIMIT_MIN = 3
PARAM_POSITION_LIMIT_MAX = 4

TASK_CARTPOLE_DISCRETE = 0
TASK_CARTPOLE_CONTINUOUS_BALANCING = 1
TASK_CARTPOLE_CONTINUOUS_SWINGUP = 2
TASK_PENDULUM_SWINGUP = 3
TASK_PANDA_POSITION_TRACKING = 4
RAND_MASS = 1
RAND_GRAVITY = 2


class MwConfig(ctypes.Structure):
    _fields_ = [
        ("step_size", ctypes.c_double),
        ("rtf", ctypes.c_double),
        ("steps_per_run", ctypes.c_int32),
        ("n_worlds", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("pgs_iters", ctypes.c_int32),
    ]


class MwTaskConfig(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("max_episode_steps", ctypes.c_int32),
        ("reward_cart_at_center", ctypes.c_int32),
        ("world_offset", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("randomize", ctypes.c_int32),
        ("mass_low", ctypes.c_float),
        ("mass_high", ctypes.c_float),
        ("gravity_mean", ctypes.c_float),
        ("gravity_std", ctypes.c_float),
        ("pad_", ctypes.c_int32),
    ]


# (name, restype, argtypes) of every symbol in include/mwstep.h
_P = ctypes.c_void_p
_I = ctypes.c_int32
_D = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int32)
_S = ctypes.c_char_p
SIGNATURES = [
    ("mw_last_error", ctypes.c_char_p, []),
    ("mw_version", ctypes.c_char_p, []),
    ("mw_create", ctypes.c_int, [ctypes.POINTER(MwConfig), ctypes.POINTER(_P)]),
    ("mw_destroy", None, [_P]),
    ("mw_load_model", ctypes.c_int, [_P, _S, _D, _S]),
    ("mw_initialize", ctypes.c_int, [_P]),
    ("mw_initialized", ctypes.c_int, [_P]),
    ("mw_set_stream", ctypes.c_int, [_P, _P]),
    ("mw_run", ctypes.c_int, [_P, ctypes.c_int]),
    ("mw_run_device", ctypes.c_int, [_P, _I]),
    ("mw_time", ctypes.c_int, [_P, _D]),
    ("mw_set_gravity", ctypes.c_int, [_P, _D]),
    ("mw_gravity", ctypes.c_int, [_P, _D]),
    ("mw_n_worlds", ctypes.c_int, [_P, _IP]),
    ("mw_dofs", ctypes.c_int, [_P, _IP]),
    ("mw_joint_name", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_link_name", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_joint_index", ctypes.c_int, [_P, _S, _IP]),
    ("mw_joint_type", ctypes.c_int, [_P, _I, _IP]),
    ("mw_model_name", ctypes.c_int, [_P, ctypes.c_char_p, _I]),
    ("mw_base_frame", ctypes.c_int, [_P, ctypes.c_char_p, _I]),
    ("mw_set_joint_param", ctypes.c_int, [_P, _I, _I, ctypes.c_double]),
    ("mw_joint_param", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_model_export", ctypes.c_int, [_P, _D, _I]),
    ("mw_model_export_base", ctypes.c_int, [_P, _D]),
    ("mw_set_pgs_options", ctypes.c_int, [_P, ctypes.c_double, _I]),
    ("mw_pgs_options", ctypes.c_int, [_P, _D, _IP]),
    ("mw_set_lcp_solver", ctypes.c_int, [_P, _I, _I]),
    ("mw_apply_link_wrench", ctypes.c_int, [_P, _I, _I, _I, _D, ctypes.c_double]),
    ("mw_lcp_solver", ctypes.c_int, [_P, _IP, _IP]),
    ("mw_lcp_unconverged", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    ("mw_model_export_shapes", ctypes.c_int, [_P, _I, _D, _I, _IP]),
    ("mw_compile_collisions", ctypes.c_int, [_S, _D, _D, _I, _IP]),
    ("mw_device_params", ctypes.c_int, [_P, _P, _I]),
    ("mw_device_float_params", ctypes.c_int, [_P, _P, _I]),
    ("mw_baked_model", ctypes.c_int, [_P, _IP]),
    ("mw_get_joint_positions", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_velocities", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_accelerations", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_forces", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_force_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_velocity_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_get_joint_position_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_set_joint_force_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_set_joint_velocity_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_set_joint_position_targets", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_reset_joint_positions", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_reset_joint_velocities", ctypes.c_int, [_P, _I, _I, _IP, _I, _D]),
    ("mw_set_joint_control_mode", ctypes.c_int, [_P, _I, _I, _IP, _I, _I]),
    ("mw_joint_control_mode", ctypes.c_int, [_P, _I, _I, _IP]),
    ("mw_set_joint_pid", ctypes.c_int, [_P, _I, _D]),
    ("mw_joint_pid", ctypes.c_int, [_P, _I, _D]),
    ("mw_set_controller_period", ctypes.c_int, [_P, ctypes.c_double]),
    ("mw_controller_period", ctypes.c_int, [_P, _D]),
    ("mw_is_floating", ctypes.c_int, [_P, _IP]),
    ("mw_get_base_pose", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_get_base_velocity", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_reset_base_pose", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_reset_base_velocity", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_set_ground_plane", ctypes.c_int, [_P, _I, ctypes.c_double]),
    ("mw_enable_contacts", ctypes.c_int, [_P, _I]),
    ("mw_contacts_enabled", ctypes.c_int, [_P, _IP]),
    ("mw_get_contacts", ctypes.c_int, [_P, _I, _D, _I, _IP]),
    ("mw_get_contact_bodies", ctypes.c_int, [_P, _I, _IP, _I, _IP]),
    ("mw_float_kernel", ctypes.c_int, [_P, _IP]),
    ("mw_constraint_overflow", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    ("mw_device_ptr", ctypes.c_int, [_P, _S, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64)]),
    ("mw_copy_state", ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    ("mw_diverged", ctypes.c_int, [_P, _I, _I, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int64)]),
    ("mw_clear_diverged", ctypes.c_int, [_P, _I, _I]),
    ("mw_state_words", ctypes.c_int, [_P, _IP]),
    ("mw_get_state", ctypes.c_int, [_P, _I, _I, ctypes.POINTER(ctypes.c_float)]),
    ("mw_set_state", ctypes.c_int, [_P, _I, _I, ctypes.POINTER(ctypes.c_float)]),
    ("mw_vecenv_create", ctypes.c_int, [_P, ctypes.POINTER(MwTaskConfig), ctypes.POINTER(_P)]),
    ("mw_vecenv_destroy", None, [_P]),
    ("mw_vecenv_obs_dim", ctypes.c_int, [_P, _IP]),
    ("mw_vecenv_reset", ctypes.c_int, [_P, _P]),
    ("mw_vecenv_step", ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    ("mw_vecenv_rollout", ctypes.c_int, [_P, _I, _P, _P, _P, _P, _P]),
    ("mw_vecenv_counters", ctypes.c_int, [_P, _P, _P]),
    ("mw_vecenv_physics", ctypes.c_int, [_P, _P, _P]),
]

# include/mwscene.h
SC_POSITION, SC_VELOCITY, SC_ACCELERATION, SC_FORCE_TARGET = 0, 1, 2, 3
SC_VELOCITY_TARGET, SC_POSITION_TARGET, SC_RESET_POSITION, SC_RESET_VELOCITY, SC_FORCE = 4, 5, 6, 7, 8
# include/mwstep_testhooks.h: test-only entry points (own buffers and stream)
TEST_SIGNATURES = [
    ("mw_debug_lcp_solve", ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                          ctypes.c_uint64, _I, _I, ctypes.POINTER(ctypes.c_float)]),
    ("mw_debug_hull", ctypes.c_int, [_D, _I, _D, _IP, _IP, _IP]),
    ("mw_debug_scene_big_ws", ctypes.c_int, [_P, _I, ctypes.POINTER(ctypes.c_float), ctypes.c_int64, _IP, _IP]),
]

SCENE_SIGNATURES = [
    ("mw_scene_create", ctypes.c_int, [ctypes.POINTER(MwConfig), ctypes.POINTER(_P)]),
    ("mw_scene_destroy", None, [_P]),
    ("mw_scene_set_stream", ctypes.c_int, [_P, _P]),
    ("mw_scene_insert_model", ctypes.c_int, [_P, _S, _D, _S, _I, _I, _IP]),
    ("mw_scene_set_present", ctypes.c_int, [_P, _I, _I, _I, _I]),
    ("mw_scene_present", ctypes.c_int, [_P, _I, _I, _IP]),
    ("mw_scene_replace_model", ctypes.c_int, [_P, _I, _S, _D, _S]),
    ("mw_scene_set_world_ground", ctypes.c_int, [_P, _I, _I, _I]),
    ("mw_scene_n_worlds", ctypes.c_int, [_P, _IP]),
    ("mw_scene_n_models", ctypes.c_int, [_P, _IP]),
    ("mw_scene_model_info", ctypes.c_int, [_P, _I, _IP, _IP, _IP]),
    ("mw_scene_model_name", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_scene_base_frame", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_scene_joint_name", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_scene_link_name", ctypes.c_int, [_P, _I, ctypes.c_char_p, _I]),
    ("mw_scene_joint_type", ctypes.c_int, [_P, _I, _IP]),
    ("mw_scene_model_export", ctypes.c_int, [_P, _I, _D, _I]),
    ("mw_scene_run", ctypes.c_int, [_P, _I]),
    ("mw_scene_run_device", ctypes.c_int, [_P, _I]),
    ("mw_scene_time", ctypes.c_int, [_P, _D]),
    ("mw_scene_set_gravity", ctypes.c_int, [_P, _D]),
    ("mw_scene_gravity", ctypes.c_int, [_P, _D]),
    ("mw_scene_set_ground_plane", ctypes.c_int, [_P, _I, ctypes.c_double]),
    ("mw_scene_set_world_gravity", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_scene_world_gravity", ctypes.c_int, [_P, _I, _D]),
    ("mw_scene_set_world_friction", ctypes.c_int, [_P, _I, _I, ctypes.c_double]),
    ("mw_scene_set_lcp_solver", ctypes.c_int, [_P, _I, _I]),
    ("mw_scene_lcp_solver", ctypes.c_int, [_P, _IP, _IP]),
    ("mw_scene_lcp_unconverged", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    ("mw_scene_get_joints", ctypes.c_int, [_P, _I, _I, _I, _IP, _I, _D]),
    ("mw_scene_set_joints", ctypes.c_int, [_P, _I, _I, _I, _IP, _I, _D]),
    ("mw_scene_set_control_mode", ctypes.c_int, [_P, _I, _I, _IP, _I, _I]),
    ("mw_scene_control_mode", ctypes.c_int, [_P, _I, _I, _IP]),
    ("mw_scene_set_joint_pid", ctypes.c_int, [_P, _I, _D]),
    ("mw_scene_joint_pid", ctypes.c_int, [_P, _I, _D]),
    ("mw_scene_set_joint_param", ctypes.c_int, [_P, _I, _I, ctypes.c_double]),
    ("mw_scene_joint_param", ctypes.c_int, [_P, _I, _I, _D]),
    ("mw_scene_set_controller_period", ctypes.c_int, [_P, _I, ctypes.c_double]),
    ("mw_scene_controller_period", ctypes.c_int, [_P, _I, _D]),
    ("mw_scene_get_base_pose", ctypes.c_int, [_P, _I, _I, _I, _D]),
    ("mw_scene_get_base_velocity", ctypes.c_int, [_P, _I, _I, _I, _D]),
    ("mw_scene_reset_base_pose", ctypes.c_int, [_P, _I, _I, _I, _D]),
    ("mw_scene_reset_base_velocity", ctypes.c_int, [_P, _I, _I, _I, _D]),
    ("mw_scene_get_contacts", ctypes.c_int, [_P, _I, _D, _I, _IP]),
    ("mw_scene_apply_world_wrench", ctypes.c_int, [_P, _I, _I, _I, _I, _D, ctypes.c_double]),
    ("mw_scene_overflow", ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    ("mw_scene_diverged", ctypes.c_int, [_P, _I, _I, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int64)]),
    ("mw_scene_clear_diverged", ctypes.c_int, [_P, _I, _I]),
]

_lib: Optional[ctypes.CDLL] = None


class NativeLibraryMissing(ImportError):
    pass


def lib() -> ctypes.CDLL:
    """Load libmwstep.so (once).  Raises NativeLibraryMissing if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `make -C gym-ignition_amd` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES + SCENE_SIGNATURES + TEST_SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().mw_last_error().decode()


class DivergedError(RuntimeError):
    """MW_EDIVERGED: the run advanced every world, and some world's state
    became non-finite (``Simulator.diverged`` / ``Scene.diverged`` list them)."""


def check(rc: int, what: str = "") -> None:
    if rc != MW_OK:
        msg = f"{what}: {last_error()}" if what else last_error()
        raise DivergedError(msg) if rc == MW_EDIVERGED else RuntimeError(msg)


def dptr(arr) -> ctypes.POINTER(ctypes.c_double):
    return arr.ctypes.data_as(_D)


def iptr(arr) -> ctypes.POINTER(ctypes.c_int32):
    return None if arr is None else arr.ctypes.data_as(_IP)
