"""Pythonic handle over one native ``mw_sim`` (many worlds, one model each)."""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import native as N


class Simulator:
    """N parallel worlds of one articulated model on one GPU.

    Mirrors ``scenario::gazebo::GazeboSimulator`` for the stepping path
    (``/root/reference/cpp/scenario/gazebo/src/GazeboSimulator.cpp:202-251``):
    ``run(paused)`` applies pending resets/commands, steps ``steps_per_run``
    substeps, and refreshes the readback that the getters return.
    """

    def __init__(self, model: str, n_worlds: int = 1, step_size: float = 1e-3,
                 steps_per_run: int = 1, rtf: float = 1.0, device: int = 0,
                 pose: Sequence[float] = (0, 0, 0, 1, 0, 0, 0), name: str = "",
                 pgs_iters: int = 20, gravity: Optional[Sequence[float]] = None,
                 stream: Optional[int] = None, joint_params: Optional[dict] = None,
                 cache_reads: bool = False, lcp_exact: Optional[bool] = None):
        L = N.lib()
        cfg = N.MwConfig(step_size, rtf, steps_per_run, n_worlds, device, pgs_iters)
        h = ctypes.c_void_p()
        N.check(L.mw_create(ctypes.byref(cfg), ctypes.byref(h)), "mw_create")
        self._h = h
        self.n_worlds = n_worlds
        self.step_size = step_size
        self.steps_per_run = steps_per_run
        # cache_reads: joint positions / velocities / accelerations are read
        # back once per run and sliced for every later getter call (the
        # ScenarI/O mirror asks for them several times per env step); any
        # call that can change state drops the cache
        self._cache_reads = cache_reads
        self._cache: dict = {}
        try:
            if lcp_exact is not None:
                # the solver picks the kernel of a floating model at load time:
                # exact (default) -> world-per-wavefront, PGS -> the lane kernels
                N.check(L.mw_set_lcp_solver(h, N.LCP_EXACT if lcp_exact else N.LCP_PGS, 24), "mw_set_lcp_solver")
            p = np.ascontiguousarray(pose, dtype=np.float64)
            N.check(L.mw_load_model(h, model.encode(), N.dptr(p), name.encode()), "mw_load_model")
            if gravity is not None:
                g = np.ascontiguousarray(gravity, dtype=np.float64)
                N.check(L.mw_set_gravity(h, N.dptr(g)), "mw_set_gravity")
            for (dof, which), value in (joint_params or {}).items():
                N.check(L.mw_set_joint_param(h, dof, which, float(value)), "mw_set_joint_param")
            if stream is not None:
                N.check(L.mw_set_stream(h, ctypes.c_void_p(stream)), "mw_set_stream")
            N.check(L.mw_initialize(h), "mw_initialize")
        except Exception:
            L.mw_destroy(h)
            self._h = None
            raise
        n = ctypes.c_int32()
        N.check(L.mw_dofs(h, ctypes.byref(n)))
        self.dofs = n.value
        buf = ctypes.create_string_buffer(256)
        self.joint_names: List[str] = []
        for d in range(self.dofs):
            N.check(L.mw_joint_name(h, d, buf, 256))
            self.joint_names.append(buf.value.decode())
        N.check(L.mw_model_name(h, buf, 256))
        self.model_name = buf.value.decode()
        N.check(L.mw_base_frame(h, buf, 256))
        self.base_frame = buf.value.decode()
        # links moved by the joints, in dof order (the base link is not among them)
        self.link_names: List[str] = []
        for d in range(self.dofs):
            N.check(L.mw_link_name(h, d, buf, 256))
            self.link_names.append(buf.value.decode())
        self._index = {n_: i for i, n_ in enumerate(self.joint_names)}

    # ------------------------------------------------------------------
    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise RuntimeError("the simulator was closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            N.lib().mw_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, paused: bool = False) -> None:
        self._cache.clear()
        N.check(N.lib().mw_run(self.handle, 1 if paused else 0), "run")

    def run_device(self, runs: int = 1) -> None:
        """`runs` runs with the state kept on the device (graph-capturable)."""
        self._cache.clear()
        N.check(N.lib().mw_run_device(self.handle, runs), "run_device")

    def time(self) -> float:
        t = ctypes.c_double()
        N.check(N.lib().mw_time(self.handle, ctypes.byref(t)))
        return t.value

    def gravity(self) -> List[float]:
        g = np.zeros(3)
        N.check(N.lib().mw_gravity(self.handle, N.dptr(g)))
        return g.tolist()

    def set_gravity(self, g: Sequence[float]) -> None:
        self._cache.clear()
        a = np.ascontiguousarray(g, dtype=np.float64)
        N.check(N.lib().mw_set_gravity(self.handle, N.dptr(a)), "set_gravity")

    # ------------------------------------------------------------------
    def dof_indices(self, names: Optional[Sequence[str]]) -> Optional[np.ndarray]:
        if names is None or len(names) == 0:
            return None
        try:
            return np.array([self._index[n] for n in names], dtype=np.int32)
        except KeyError as e:
            raise RuntimeError(f"joint {e.args[0]!r} not found in model {self.model_name!r}") from None

    def _get(self, fn, w0: int, nw: int, dofs: Optional[np.ndarray]) -> np.ndarray:
        m = self.dofs if dofs is None else len(dofs)
        out = np.zeros((nw, m))
        N.check(fn(self.handle, w0, nw, N.iptr(dofs), 0 if dofs is None else len(dofs), N.dptr(out)))
        return out

    def _set(self, fn, w0: int, nw: int, dofs: Optional[np.ndarray], values) -> None:
        m = self.dofs if dofs is None else len(dofs)
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.float64), (nw, m)))
        N.check(fn(self.handle, w0, nw, N.iptr(dofs), 0 if dofs is None else len(dofs), N.dptr(v)))

    def get(self, what: str, w0: int = 0, nw: Optional[int] = None, dofs=None) -> np.ndarray:
        fn = {
            "q": N.lib().mw_get_joint_positions,
            "qd": N.lib().mw_get_joint_velocities,
            "qdd": N.lib().mw_get_joint_accelerations,
            "force": N.lib().mw_get_joint_forces,
            "force_target": N.lib().mw_get_joint_force_targets,
            "velocity_target": N.lib().mw_get_joint_velocity_targets,
            "position_target": N.lib().mw_get_joint_position_targets,
        }[what]
        nw = self.n_worlds - w0 if nw is None else nw
        if self._cache_reads and what in ("q", "qd", "qdd"):
            full = self._cache.get(what)
            if full is None:
                full = self._cache[what] = self._get(fn, 0, self.n_worlds, None)
            out = full[w0:w0 + nw]
            if dofs is not None:
                out = out[:, dofs]
            return out.copy()
        return self._get(fn, w0, nw, dofs)

    def set(self, what: str, values, w0: int = 0, nw: Optional[int] = None, dofs=None) -> None:
        self._cache.clear()
        fn = {
            "force_target": N.lib().mw_set_joint_force_targets,
            "velocity_target": N.lib().mw_set_joint_velocity_targets,
            "position_target": N.lib().mw_set_joint_position_targets,
            "reset_q": N.lib().mw_reset_joint_positions,
            "reset_qd": N.lib().mw_reset_joint_velocities,
        }[what]
        self._set(fn, w0, self.n_worlds - w0 if nw is None else nw, dofs, values)

    def set_control_mode(self, mode: int, w0: int = 0, nw: Optional[int] = None, dofs=None) -> None:
        self._cache.clear()
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_set_joint_control_mode(self.handle, w0, nw, N.iptr(dofs),
                                                  0 if dofs is None else len(dofs), mode))

    def control_mode(self, w: int, dof: int) -> int:
        m = ctypes.c_int32()
        N.check(N.lib().mw_joint_control_mode(self.handle, w, dof, ctypes.byref(m)))
        return m.value

    def joint_type(self, dof: int) -> int:
        t = ctypes.c_int32()
        N.check(N.lib().mw_joint_type(self.handle, dof, ctypes.byref(t)))
        return t.value

    def set_joint_param(self, dof: int, which: int, value: float) -> None:
        self._cache.clear()
        N.check(N.lib().mw_set_joint_param(self.handle, dof, which, float(value)))

    def joint_param(self, dof: int, which: int) -> float:
        v = ctypes.c_double()
        N.check(N.lib().mw_joint_param(self.handle, dof, which, ctypes.byref(v)))
        return v.value

    def set_pid(self, dof: int, gains) -> None:
        """gains = {p, i, d, cmd_min, cmd_max, cmd_offset, i_min, i_max} (all worlds)."""
        self._cache.clear()
        g = np.ascontiguousarray(gains, dtype=np.float64)
        assert g.shape == (8,)
        N.check(N.lib().mw_set_joint_pid(self.handle, dof, N.dptr(g)))

    def pid(self, dof: int) -> np.ndarray:
        g = np.zeros(8)
        N.check(N.lib().mw_joint_pid(self.handle, dof, N.dptr(g)))
        return g

    def set_controller_period(self, period: float) -> None:
        self._cache.clear()
        N.check(N.lib().mw_set_controller_period(self.handle, float(period)))

    def controller_period(self) -> float:
        v = ctypes.c_double()
        N.check(N.lib().mw_controller_period(self.handle, ctypes.byref(v)))
        return v.value

    # -- floating single bodies (mwstep.h: floating bases)
    @property
    def floating(self) -> bool:
        v = ctypes.c_int32()
        N.check(N.lib().mw_is_floating(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def base_pose(self, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        """[nw, 7]: x y z qw qx qy qz."""
        nw = self.n_worlds - w0 if nw is None else nw
        out = np.zeros((nw, 7))
        N.check(N.lib().mw_get_base_pose(self.handle, w0, nw, N.dptr(out)), "base_pose")
        return out

    def base_velocity(self, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        """[nw, 6]: world linear xyz (base origin), world angular xyz."""
        nw = self.n_worlds - w0 if nw is None else nw
        out = np.zeros((nw, 6))
        N.check(N.lib().mw_get_base_velocity(self.handle, w0, nw, N.dptr(out)), "base_velocity")
        return out

    def reset_base_pose(self, pose, w0: int = 0, nw: Optional[int] = None) -> None:
        self._cache.clear()
        nw = self.n_worlds - w0 if nw is None else nw
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(pose, dtype=np.float64), (nw, 7)))
        N.check(N.lib().mw_reset_base_pose(self.handle, w0, nw, N.dptr(v)), "reset_base_pose")

    def reset_base_velocity(self, lin_ang, w0: int = 0, nw: Optional[int] = None) -> None:
        self._cache.clear()
        nw = self.n_worlds - w0 if nw is None else nw
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(lin_ang, dtype=np.float64), (nw, 6)))
        N.check(N.lib().mw_reset_base_velocity(self.handle, w0, nw, N.dptr(v)), "reset_base_velocity")

    def set_ground_plane(self, enabled: bool, mu: float = 1.0) -> None:
        self._cache.clear()
        N.check(N.lib().mw_set_ground_plane(self.handle, 1 if enabled else 0, float(mu)), "set_ground_plane")

    def enable_contacts(self, enable: bool = True) -> None:
        self._cache.clear()
        N.check(N.lib().mw_enable_contacts(self.handle, 1 if enable else 0))

    def contacts_enabled(self) -> bool:
        v = ctypes.c_int32()
        N.check(N.lib().mw_contacts_enabled(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def contacts(self, w: int = 0) -> np.ndarray:
        """[n, 10]: point xyz, normal xyz, force on the body xyz, depth."""
        cap = 64
        out = np.zeros((cap, 10))
        n = ctypes.c_int32()
        N.check(N.lib().mw_get_contacts(self.handle, w, N.dptr(out), cap, ctypes.byref(n)), "contacts")
        return out[:min(n.value, cap)].copy()

    def contact_bodies(self, w: int = 0) -> np.ndarray:
        """Body of every row of contacts(w): -1 = base link, i = the link of joint i."""
        cap = 64
        out = np.zeros(cap, dtype=np.int32)
        n = ctypes.c_int32()
        N.check(N.lib().mw_get_contact_bodies(self.handle, w, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              cap, ctypes.byref(n)), "contact_bodies")
        return out[:min(n.value, cap)].copy()

    def set_pgs_options(self, tol: float = 0.0, warm_start: bool = False) -> None:
        """mw_set_pgs_options: PGS tolerance exit and warm start (world-per-wavefront kernel)."""
        N.check(N.lib().mw_set_pgs_options(self.handle, float(tol), 1 if warm_start else 0), "set_pgs_options")

    def pgs_options(self):
        t, w = ctypes.c_double(), ctypes.c_int32()
        N.check(N.lib().mw_pgs_options(self.handle, ctypes.byref(t), ctypes.byref(w)))
        return t.value, bool(w.value)

    def apply_world_wrench(self, link: int, wrench, duration: float, w0: int = 0, nw: Optional[int] = None) -> None:
        """mw_apply_link_wrench (Link::applyWorldWrench, Link.cpp:484-560): world
        force at the link origin + world torque ([nw, 6] or one row for all),
        from the next step for max(1, ceil(duration / dt)) steps; link -1 = base."""
        nw = self.n_worlds - w0 if nw is None else nw
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(wrench, dtype=np.float64), (nw, 6)))
        N.check(N.lib().mw_apply_link_wrench(self.handle, int(link), int(w0), int(nw), N.dptr(v), float(duration)),
                "apply_world_wrench")

    def set_lcp_solver(self, exact: bool = True, max_solves: int = 48) -> None:
        """mw_set_lcp_solver: exact boxed LCP after the PGS sweeps (default) or the sweeps alone."""
        N.check(N.lib().mw_set_lcp_solver(self.handle, N.LCP_EXACT if exact else N.LCP_PGS, int(max_solves)),
                "set_lcp_solver")

    def lcp_solver(self):
        m, k = ctypes.c_int32(), ctypes.c_int32()
        N.check(N.lib().mw_lcp_solver(self.handle, ctypes.byref(m), ctypes.byref(k)))
        return m.value == N.LCP_EXACT, k.value

    def diverged(self, w0: int = 0, nw: Optional[int] = None):
        """(flags [nw] bool of worlds [w0, w0 + nw), number of worlds flagged
        since initialisation): worlds whose stored state became non-finite
        (mw_diverged)."""
        nw = self.n_worlds - w0 if nw is None else nw
        flags = np.zeros(nw, dtype=np.uint8)
        n = ctypes.c_int64()
        N.check(N.lib().mw_diverged(self.handle, w0, nw, flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                    ctypes.byref(n)), "diverged")
        return flags.astype(bool), n.value

    def clear_diverged(self, w0: int = 0, nw: Optional[int] = None) -> None:
        nw = self.n_worlds - w0 if nw is None else nw
        N.check(N.lib().mw_clear_diverged(self.handle, w0, nw), "clear_diverged")

    def get_state(self, w0: int = 0, nw: Optional[int] = None) -> np.ndarray:
        """mw_get_state: the full per-world record, float32 [nw, words]."""
        nw = self.n_worlds - w0 if nw is None else nw
        k = ctypes.c_int32()
        N.check(N.lib().mw_state_words(self.handle, ctypes.byref(k)), "state_words")
        out = np.zeros((nw, k.value), dtype=np.float32)
        N.check(N.lib().mw_get_state(self.handle, w0, nw, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))),
                "get_state")
        return out

    def set_state(self, state, w0: int = 0) -> None:
        """mw_set_state: write a record of get_state back (bit-exact)."""
        st = np.ascontiguousarray(state, dtype=np.float32)
        N.check(N.lib().mw_set_state(self.handle, w0, st.shape[0], st.ctypes.data_as(ctypes.POINTER(ctypes.c_float))),
                "set_state")

    def lcp_unconverged(self) -> int:
        """World-steps whose exact LCP solve ran out of its budget."""
        v = ctypes.c_int64()
        N.check(N.lib().mw_lcp_unconverged(self.handle, ctypes.byref(v)))
        return v.value

    def float_kernel(self) -> int:
        """0: not an articulated floating model, 1: world-per-lane kernel, 2: world-per-wavefront kernel."""
        v = ctypes.c_int32()
        N.check(N.lib().mw_float_kernel(self.handle, ctypes.byref(v)))
        return v.value

    def constraint_overflow(self) -> int:
        v = ctypes.c_int64()
        N.check(N.lib().mw_constraint_overflow(self.handle, ctypes.byref(v)))
        return v.value

    def export_model(self) -> np.ndarray:
        out = np.zeros(34 * self.dofs + 3)
        N.check(N.lib().mw_model_export(self.handle, N.dptr(out), len(out)))
        return out

    def baked_model(self) -> int:
        """1/2 when the batched env runs the constant-folded cartpole/pendulum kernel."""
        v = ctypes.c_int32()
        N.check(N.lib().mw_baked_model(self.handle, ctypes.byref(v)))
        return v.value

    def device_ptr(self, field: str):
        self._cache.clear()
        p = ctypes.c_void_p()
        stride = ctypes.c_int64()
        N.check(N.lib().mw_device_ptr(self.handle, field.encode(), ctypes.byref(p), ctypes.byref(stride)))
        return p.value, stride.value

    def set_stream(self, stream: int) -> None:
        self._cache.clear()
        N.check(N.lib().mw_set_stream(self.handle, ctypes.c_void_p(stream)))
