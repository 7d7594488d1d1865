"""Pythonic handle over one native ``mw_scene``: several models per world,
many worlds per launch (include/mwscene.h, csrc/scene_kernel.hip).

A scene is what the reference builds with ``World::insertModel`` on every
world of a ``GazeboSimulator`` (``cpp/scenario/gazebo/src/World.cpp:394-420``,
``GazeboSimulator.cpp:435-488``): models collide with the ground plane and
with each other, links take world wrenches (``Link.cpp:484-560``), and one
``run()`` steps every world in one kernel launch.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import native as N


class Scene:
    def __init__(self, n_worlds: int = 1, step_size: float = 1e-3, steps_per_run: int = 1, rtf: float = 1.0,
                 device: int = 0, pgs_iters: int = 50):
        L = N.lib()
        cfg = N.MwConfig(step_size, rtf, steps_per_run, n_worlds, device, pgs_iters)
        h = ctypes.c_void_p()
        N.check(L.mw_scene_create(ctypes.byref(cfg), ctypes.byref(h)), "mw_scene_create")
        self._h = h
        self.n_worlds = n_worlds
        self.step_size = step_size
        self.steps_per_run = steps_per_run
        self.models: List[dict] = []
        self._models_changed()

    def _models_changed(self) -> None:
        # the per-env ScenarI/O path asks for the same selections every step
        self._selcache = {}
        self._touch()
        self._nd = sum(i["dofs"] for i in self.models)

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise RuntimeError("the scene was closed")
        return self._h

    def close(self) -> None:
        if self._h is not None:
            N.lib().mw_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- models
    def insert_model(self, urdf: str, pose: Sequence[float] = (0, 0, 0, 1, 0, 0, 0), name: str = "",
                     worlds: Optional[Sequence[int]] = None) -> int:
        """World::insertModel into worlds [w0, w0 + nw) (default: all); returns the model index."""
        self._touch()
        w0, nw = (0, self.n_worlds) if worlds is None else (worlds[0], worlds[1])
        p = np.ascontiguousarray(pose, dtype=np.float64)
        m = ctypes.c_int32()
        N.check(N.lib().mw_scene_insert_model(self.handle, urdf.encode(), N.dptr(p), name.encode(), w0, nw,
                                              ctypes.byref(m)), "insert_model")
        self.models.append(self._info(m.value))
        self._models_changed()
        return m.value

    def _info(self, m: int) -> dict:
        L = N.lib()
        first, n, fl = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        N.check(L.mw_scene_model_info(self.handle, m, ctypes.byref(first), ctypes.byref(n), ctypes.byref(fl)))
        buf = ctypes.create_string_buffer(256)
        N.check(L.mw_scene_model_name(self.handle, m, buf, 256))
        name = buf.value.decode()
        N.check(L.mw_scene_base_frame(self.handle, m, buf, 256))
        base = buf.value.decode()
        joints, links = [], []
        for d in range(first.value, first.value + n.value):
            N.check(L.mw_scene_joint_name(self.handle, d, buf, 256))
            joints.append(buf.value.decode())
            N.check(L.mw_scene_link_name(self.handle, d, buf, 256))
            links.append(buf.value.decode())
        return dict(first=first.value, dofs=n.value, floating=bool(fl.value), name=name, base_frame=base,
                    joint_names=joints, link_names=links)

    def set_present(self, m: int, present, w0: int = 0, nw: Optional[int] = None) -> None:
        """present: False / 0 remove, True / 1 (re-)insert at the insertion pose, 2 resume with the state kept"""
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_scene_set_present(self.handle, m, w0, nw, int(present)), "set_present")

    def replace_model(self, m: int, urdf: str, pose: Sequence[float] = (0, 0, 0, 1, 0, 0, 0), name: str = "") -> None:
        self._touch()
        p = np.ascontiguousarray(pose, dtype=np.float64)
        N.check(N.lib().mw_scene_replace_model(self.handle, m, urdf.encode(), N.dptr(p), name.encode()),
                "replace_model")
        self.models[m] = self._info(m)
        self._models_changed()

    def set_world_ground(self, enabled: bool, w0: int = 0, nw: Optional[int] = None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_scene_set_world_ground(self.handle, w0, nw, 1 if enabled else 0), "set_world_ground")

    def present(self, m: int, w: int = 0) -> bool:
        v = ctypes.c_int32()
        N.check(N.lib().mw_scene_present(self.handle, m, w, ctypes.byref(v)))
        return bool(v.value)

    def export_model(self, m: int) -> np.ndarray:
        """34 doubles per body, gravity in the base frame (3), base mass and COM (4)"""
        n = self.models[m]["dofs"]
        out = np.zeros(34 * n + 7)
        N.check(N.lib().mw_scene_model_export(self.handle, m, N.dptr(out), out.size))
        return out

    # ----------------------------------------------------------- stepping
    def run(self, paused: bool = False) -> None:
        self._touch()
        N.check(N.lib().mw_scene_run(self.handle, 1 if paused else 0), "run")

    def run_device(self, runs: int = 1) -> None:
        self._touch()
        N.check(N.lib().mw_scene_run_device(self.handle, runs), "run_device")

    def set_stream(self, stream: int) -> None:
        N.check(N.lib().mw_scene_set_stream(self.handle, ctypes.c_void_p(stream)), "set_stream")

    def time(self) -> float:
        t = ctypes.c_double()
        N.check(N.lib().mw_scene_time(self.handle, ctypes.byref(t)))
        return t.value

    def gravity(self) -> List[float]:
        g = np.zeros(3)
        N.check(N.lib().mw_scene_gravity(self.handle, N.dptr(g)))
        return g.tolist()

    def set_gravity(self, g: Sequence[float]) -> None:
        self._touch()
        a = np.ascontiguousarray(g, dtype=np.float64)
        N.check(N.lib().mw_scene_set_gravity(self.handle, N.dptr(a)), "set_gravity")

    def set_world_gravity(self, g: Sequence[float], w0: int = 0, nw: Optional[int] = None) -> None:
        """World::setGravity of worlds [w0, w0 + nw) (each world its own gravity)."""
        self._touch()
        a = np.ascontiguousarray(g, dtype=np.float64)
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_scene_set_world_gravity(self.handle, w0, nw, N.dptr(a)), "set_world_gravity")

    def world_gravity(self, w: int) -> List[float]:
        g = np.zeros(3)
        N.check(N.lib().mw_scene_world_gravity(self.handle, w, N.dptr(g)))
        return g.tolist()

    def set_world_friction(self, mu: float, w0: int = 0, nw: Optional[int] = None) -> None:
        """Ground-plane friction coefficient of worlds [w0, w0 + nw)."""
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_scene_set_world_friction(self.handle, w0, nw, float(mu)), "set_world_friction")

    def set_lcp_solver(self, exact: bool = True, max_solves: int = 48) -> None:
        """mw_scene_set_lcp_solver: exact boxed LCP after the PGS sweeps (default) or the sweeps alone."""
        N.check(N.lib().mw_scene_set_lcp_solver(self.handle, N.LCP_EXACT if exact else N.LCP_PGS, int(max_solves)),
                "set_lcp_solver")

    def lcp_solver(self):
        m, k = ctypes.c_int32(), ctypes.c_int32()
        N.check(N.lib().mw_scene_lcp_solver(self.handle, ctypes.byref(m), ctypes.byref(k)))
        return m.value == N.LCP_EXACT, k.value

    def diverged(self, w0: int = 0, nw: Optional[int] = None):
        """(flags [nw] bool, worlds flagged since initialisation): worlds whose
        stored state became non-finite (mw_scene_diverged)."""
        nw = self.n_worlds - w0 if nw is None else nw
        flags = np.zeros(nw, dtype=np.uint8)
        n = ctypes.c_int64()
        N.check(N.lib().mw_scene_diverged(self.handle, w0, nw, flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                          ctypes.byref(n)), "diverged")
        return flags.astype(bool), n.value

    def clear_diverged(self, w0: int = 0, nw: Optional[int] = None) -> None:
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_scene_clear_diverged(self.handle, w0, nw), "clear_diverged")

    def lcp_unconverged(self) -> int:
        v = ctypes.c_int64()
        N.check(N.lib().mw_scene_lcp_unconverged(self.handle, ctypes.byref(v)))
        return v.value

    def set_ground_plane(self, enabled: bool = True, mu: float = 1.0) -> None:
        self._touch()
        N.check(N.lib().mw_scene_set_ground_plane(self.handle, 1 if enabled else 0, float(mu)), "set_ground_plane")

    # ------------------------------------------------------------- joints
    _FIELDS = {"q": N.SC_POSITION, "qd": N.SC_VELOCITY, "qdd": N.SC_ACCELERATION,
               "force_target": N.SC_FORCE_TARGET, "velocity_target": N.SC_VELOCITY_TARGET,
               "position_target": N.SC_POSITION_TARGET, "reset_q": N.SC_RESET_POSITION,
               "reset_qd": N.SC_RESET_VELOCITY, "force": N.SC_FORCE}

    def _sel(self, m: Optional[int], dofs):
        """global dof indices of model m (local indices `dofs`), or every dof"""
        if m is None:
            return None if dofs is None else np.ascontiguousarray(dofs, dtype=np.int32)
        key = (m, None if dofs is None else tuple(int(d) for d in dofs))
        sel = self._selcache.get(key)
        if sel is None:
            info = self.models[m]
            local = range(info["dofs"]) if dofs is None else key[1]
            sel = self._selcache[key] = np.ascontiguousarray([info["first"] + d for d in local], dtype=np.int32)
        return sel

    # The joint state changes only through runs and the mutators below, so the
    # per-env ScenarI/O path (a handful of getters per env step, each a C call
    # into the host mirror of the last run) reads each state field once per
    # run for small scenes and slices it.
    _STATE = ("q", "qd", "qdd", "force")
    _CACHE_MAX = 4096  # worlds x dofs of a cached field

    def _touch(self) -> None:
        self.__dict__.setdefault("_cache", {}).clear()
        # generation of the joint state: getters above this layer memoise
        # per generation (scenario.gazebo.Model)
        self.gen = self.__dict__.get("gen", 0) + 1

    def _cached(self, what: str) -> Optional[np.ndarray]:
        nd = self._nd
        if what not in self._STATE or nd == 0 or self.n_worlds * nd > self._CACHE_MAX:
            return None
        cache = self.__dict__.setdefault("_cache", {})
        full = cache.get(what)
        if full is None:
            full = np.zeros((self.n_worlds, nd))
            N.check(N.lib().mw_scene_get_joints(self.handle, self._FIELDS[what], 0, self.n_worlds, None, 0,
                                                N.dptr(full)), f"get {what}")
            cache[what] = full
        return full

    def get(self, what: str, m: Optional[int] = None, w0: int = 0, nw: Optional[int] = None, dofs=None) -> np.ndarray:
        nw = self.n_worlds - w0 if nw is None else nw
        sel = self._sel(m, dofs)
        full = self._cached(what)
        if full is not None:
            return full[w0:w0 + nw].copy() if sel is None else full[w0:w0 + nw][:, sel]
        nd = (self._nd if sel is None else len(sel))
        out = np.zeros((nw, nd))
        if nd:
            N.check(N.lib().mw_scene_get_joints(self.handle, self._FIELDS[what], w0, nw, N.iptr(sel),
                                                0 if sel is None else len(sel), N.dptr(out)), f"get {what}")
        return out

    def set(self, what: str, values, m: Optional[int] = None, w0: int = 0, nw: Optional[int] = None,
            dofs=None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        sel = self._sel(m, dofs)
        nd = (self._nd if sel is None else len(sel))
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.float64), (nw, nd)))
        N.check(N.lib().mw_scene_set_joints(self.handle, self._FIELDS[what], w0, nw, N.iptr(sel),
                                            0 if sel is None else len(sel), N.dptr(v)), f"set {what}")

    def set_control_mode(self, mode: int, m: Optional[int] = None, w0: int = 0, nw: Optional[int] = None,
                         dofs=None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        sel = self._sel(m, dofs)
        N.check(N.lib().mw_scene_set_control_mode(self.handle, w0, nw, N.iptr(sel),
                                                  0 if sel is None else len(sel), mode), "set_control_mode")

    def control_mode(self, w: int, dof: int) -> int:
        v = ctypes.c_int32()
        N.check(N.lib().mw_scene_control_mode(self.handle, w, dof, ctypes.byref(v)))
        return v.value

    def set_pid(self, dof: int, gains) -> None:
        self._touch()
        g = np.ascontiguousarray(gains, dtype=np.float64)
        N.check(N.lib().mw_scene_set_joint_pid(self.handle, dof, N.dptr(g)), "set_pid")

    def pid(self, dof: int) -> np.ndarray:
        g = np.zeros(8)
        N.check(N.lib().mw_scene_joint_pid(self.handle, dof, N.dptr(g)))
        return g

    def set_joint_param(self, dof: int, which: int, value: float) -> None:
        self._touch()
        N.check(N.lib().mw_scene_set_joint_param(self.handle, dof, which, float(value)), "set_joint_param")

    def joint_param(self, dof: int, which: int) -> float:
        v = ctypes.c_double()
        N.check(N.lib().mw_scene_joint_param(self.handle, dof, which, ctypes.byref(v)))
        return v.value

    def set_controller_period(self, m: int, period: float) -> None:
        self._touch()
        N.check(N.lib().mw_scene_set_controller_period(self.handle, m, float(period)), "set_controller_period")

    def controller_period(self, m: int) -> float:
        v = ctypes.c_double()
        N.check(N.lib().mw_scene_controller_period(self.handle, m, ctypes.byref(v)))
        return v.value

    # -------------------------------------------------------------- bases
    def base_pose(self, m: int, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        nw = self.n_worlds - w0 if nw is None else nw
        out = np.zeros((nw, 7))
        N.check(N.lib().mw_scene_get_base_pose(self.handle, m, w0, nw, N.dptr(out)), "base_pose")
        return out

    def base_velocity(self, m: int, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        nw = self.n_worlds - w0 if nw is None else nw
        out = np.zeros((nw, 6))
        N.check(N.lib().mw_scene_get_base_velocity(self.handle, m, w0, nw, N.dptr(out)), "base_velocity")
        return out

    def reset_base_pose(self, m: int, pose, w0: int = 0, nw: Optional[int] = None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        p = np.ascontiguousarray(np.broadcast_to(np.asarray(pose, dtype=np.float64), (nw, 7)))
        N.check(N.lib().mw_scene_reset_base_pose(self.handle, m, w0, nw, N.dptr(p)), "reset_base_pose")

    def reset_base_velocity(self, m: int, lin_ang, w0: int = 0, nw: Optional[int] = None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(lin_ang, dtype=np.float64), (nw, 6)))
        N.check(N.lib().mw_scene_reset_base_velocity(self.handle, m, w0, nw, N.dptr(v)), "reset_base_velocity")

    # ---------------------------------------------------- contacts, wrenches
    def contacts(self, w: int = 0) -> np.ndarray:
        """rows: point(3), normal B->A (3), force on A (3), depth, model A, link A, model B, link B"""
        out = np.zeros((128, 14))   # kScBigContacts: the large-contact capacity
        n = ctypes.c_int32()
        N.check(N.lib().mw_scene_get_contacts(self.handle, w, N.dptr(out), len(out), ctypes.byref(n)), "contacts")
        if n.value > len(out):
            out = np.zeros((n.value, 14))
            N.check(N.lib().mw_scene_get_contacts(self.handle, w, N.dptr(out), len(out), ctypes.byref(n)), "contacts")
        return out[:n.value]

    def apply_world_wrench(self, m: int, link: int, wrench, duration: float, w0: int = 0,
                           nw: Optional[int] = None) -> None:
        self._touch()
        nw = self.n_worlds - w0 if nw is None else nw
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(wrench, dtype=np.float64), (nw, 6)))
        N.check(N.lib().mw_scene_apply_world_wrench(self.handle, m, link, w0, nw, N.dptr(v), float(duration)),
                "apply_world_wrench")

    def overflow(self) -> int:
        v = ctypes.c_int64()
        N.check(N.lib().mw_scene_overflow(self.handle, ctypes.byref(v)))
        return v.value


class SceneView:
    """One model of one world of a Scene, with the interface of
    ``mwstep.sim.Simulator`` that the ScenarI/O mirror (``scenario.gazebo``)
    drives: joint getters / setters over local dof indices, base state,
    contacts from this model's side, parameters.  Joint parameters, PID gains
    and the controller period belong to the model slot (shared by the worlds
    that hold the same model); state, commands, targets, control modes,
    resets and wrenches are per world."""

    def __init__(self, scene: Scene, m: int, w: int):
        self.scene, self.m, self.w = scene, m, w
        self._contacts_enabled = False
        self._refresh()

    def _refresh(self) -> None:
        info = self.scene.models[self.m]
        self.first = info["first"]
        self.dofs = info["dofs"]
        self.floating = info["floating"]
        self.joint_names = list(info["joint_names"])
        self.link_names = list(info["link_names"])
        self.base_frame = info["base_frame"]
        self._index = {n: i for i, n in enumerate(self.joint_names)}

    # ---- identity / parameters
    def dof_indices(self, names) -> Optional[np.ndarray]:
        if names is None:
            return None
        try:
            return np.array([self._index[n] for n in names], dtype=np.int32)
        except KeyError as e:
            raise RuntimeError(f"Joint {e} not found") from None

    def joint_type(self, dof: int) -> int:
        v = ctypes.c_int32()
        N.check(N.lib().mw_scene_joint_type(self.scene.handle, self.first + dof, ctypes.byref(v)))
        return v.value

    def control_mode(self, w: int, dof: int) -> int:
        return self.scene.control_mode(self.w, self.first + dof)

    def pid(self, dof: int) -> np.ndarray:
        return self.scene.pid(self.first + dof)

    def set_pid(self, dof: int, gains) -> None:
        self.scene.set_pid(self.first + dof, gains)

    def set_joint_param(self, dof: int, which: int, value: float) -> None:
        self.scene.set_joint_param(self.first + dof, which, value)

    def joint_param(self, dof: int, which: int) -> float:
        return self.scene.joint_param(self.first + dof, which)

    def controller_period(self) -> float:
        return self.scene.controller_period(self.m)

    def set_controller_period(self, period: float) -> None:
        self.scene.set_controller_period(self.m, period)

    def export_model(self) -> np.ndarray:
        return self.scene.export_model(self.m)

    # ---- joints (local dof indices, this world)
    def get(self, what: str, w0: int = 0, nw: Optional[int] = None, dofs=None) -> np.ndarray:
        return self.scene.get(what, self.m, self.w, 1, None if dofs is None else tuple(np.asarray(dofs).tolist()))

    def set(self, what: str, values, w0: int = 0, nw: Optional[int] = None, dofs=None) -> None:
        self.scene.set(what, values, self.m, self.w, 1, None if dofs is None else list(np.asarray(dofs)))

    def set_control_mode(self, mode: int, w0: int = 0, nw: Optional[int] = None, dofs=None) -> None:
        self.scene.set_control_mode(mode, self.m, self.w, 1, None if dofs is None else list(np.asarray(dofs)))

    # ---- base
    def base_pose(self, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        return self.scene.base_pose(self.m, self.w, 1)

    def base_velocity(self, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        return self.scene.base_velocity(self.m, self.w, 1)

    def reset_base_pose(self, pose, w0: int = 0, nw: Optional[int] = None) -> None:
        self.scene.reset_base_pose(self.m, np.asarray(pose, dtype=np.float64).reshape(1, 7), self.w, 1)

    def reset_base_velocity(self, lin_ang, w0: int = 0, nw: Optional[int] = None) -> None:
        self.scene.reset_base_velocity(self.m, np.asarray(lin_ang, dtype=np.float64).reshape(1, 6), self.w, 1)

    # ---- contacts (reporting only: collisions always act) and wrenches
    def contacts_enabled(self) -> bool:
        return self._contacts_enabled

    def enable_contacts(self, enable: bool = True) -> None:
        self._contacts_enabled = bool(enable)

    def contact_rows(self) -> np.ndarray:
        """This model's contacts in world w, rows of 13: point, normal into
        this model's body, force on it, depth, own link, other model (-1:
        ground), other link (Physics.cpp:2498-2529 flips the second body)."""
        rows = self.scene.contacts(self.w)
        out = []
        for r in rows:
            if int(r[10]) == self.m:
                out.append(np.concatenate([r[0:10], [r[11], r[12], r[13]]]))
            elif int(r[12]) == self.m:
                out.append(np.concatenate([r[0:3], -r[3:6], -r[6:9], [r[9], r[13], r[10], r[11]]]))
        return np.array(out).reshape(-1, 13)

    def apply_world_wrench(self, link: int, wrench, duration: float) -> None:
        self.scene.apply_world_wrench(self.m, link, np.asarray(wrench, dtype=np.float64).reshape(1, 6), duration,
                                      self.w, 1)
