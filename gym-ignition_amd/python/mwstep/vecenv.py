"""Batched, device-resident environment over the HIP step kernel.

One ``step()`` advances every world once: the action is applied, the physics
runs ``steps_per_run`` substeps, and the Task logic of the reference
(``/root/reference/python/gym_ignition_environments/tasks/*.py``: observation,
reward, done) plus gym's TimeLimit (``max_episode_steps``,
``gym_ignition_environments/__init__.py:14-52``) and auto-reset of the done
worlds all run inside the same kernel.  Buffers live in HBM as torch tensors;
nothing crosses PCIe per step.

Auto-reset follows the common VecEnv convention: where ``done`` is set, ``obs``
holds the first observation of the next episode and ``info["terminal_obs"]``
the last observation of the finished one.
"""

from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import numpy as np

from . import native as N
from .models import get_model_file
from .sim import Simulator

TASKS = {
    "CartPoleDiscreteBalancing": (N.TASK_CARTPOLE_DISCRETE, "cartpole"),
    "CartPoleContinuousBalancing": (N.TASK_CARTPOLE_CONTINUOUS_BALANCING, "cartpole"),
    "CartPoleContinuousSwingup": (N.TASK_CARTPOLE_CONTINUOUS_SWINGUP, "cartpole"),
    "PendulumSwingUp": (N.TASK_PENDULUM_SWINGUP, "pendulum"),
    # BASELINE config 4: Position-mode PID control of every Panda joint,
    # actions = position targets [n_worlds, 9]
    "PandaPositionTracking": (N.TASK_PANDA_POSITION_TRACKING, "panda"),
}


def _torch():
    import torch  # noqa: WPS433 (plumbing only: device memory + streams)
    return torch


class VecEnv:
    """``n_worlds`` copies of one gym-ignition task stepped together on one GPU."""

    def __init__(self, task: str = "CartPoleDiscreteBalancing", n_worlds: int = 4096,
                 device: int = 0, seed: int = 42, agent_rate: float = 1000.0,
                 physics_rate: float = 1000.0, max_episode_steps: int = 5000,
                 reward_cart_at_center: bool = True, model_file: Optional[str] = None,
                 pgs_iters: int = 20, world_offset: int = 0, randomize: bool = False,
                 mass_range: Tuple[float, float] = (-0.2, 0.2),
                 gravity_normal: Tuple[float, float] = (-9.8, 0.2)):
        """``randomize=True`` resamples every world's physics at each reset as the
        reference's CartPole randomizer does (randomizers/cartpole.py:51-56,
        100-135): body masses + max(U(*mass_range), 0), gravity z ~
        N(*gravity_normal)."""
        torch = _torch()
        if task not in TASKS:
            raise ValueError(f"unknown task {task!r}; known: {sorted(TASKS)}")
        kind, model = TASKS[task]
        steps_per_run = int(physics_rate / agent_rate)
        if steps_per_run <= 0:
            raise ValueError("physics_rate must be >= agent_rate")
        self.task = task
        self.kind = kind
        self.n_worlds = n_worlds
        self.device = torch.device("cuda", device)
        with torch.cuda.device(self.device):
            self._stream = torch.cuda.current_stream(self.device)
            self.sim = Simulator(model_file or get_model_file(model), n_worlds=n_worlds,
                                 step_size=1.0 / physics_rate, steps_per_run=steps_per_run,
                                 device=device, pgs_iters=pgs_iters,
                                 stream=self._stream.cuda_stream)
        if kind == N.TASK_PANDA_POSITION_TRACKING:
            from .models import PANDA_PID_GAINS_1000HZ
            big = float(np.finfo(np.float64).max)
            for d, name in enumerate(self.sim.joint_names):
                p, i, dd = PANDA_PID_GAINS_1000HZ[name]
                self.sim.set_pid(d, [p, i, dd, -big, big, 0.0, -big, big])
        cfg = N.MwTaskConfig(kind, max_episode_steps, 1 if reward_cart_at_center else 0,
                             world_offset, seed & 0xFFFFFFFFFFFFFFFF,
                             (N.RAND_MASS | N.RAND_GRAVITY) if randomize else 0,
                             mass_range[0], mass_range[1], gravity_normal[0], gravity_normal[1], 0)
        self.randomize = randomize
        h = ctypes.c_void_p()
        N.check(N.lib().mw_vecenv_create(self.sim.handle, ctypes.byref(cfg), ctypes.byref(h)),
                "mw_vecenv_create")
        self._h = h
        no = ctypes.c_int32()
        N.check(N.lib().mw_vecenv_obs_dim(h, ctypes.byref(no)))
        self.obs_dim = no.value
        self.discrete = kind == N.TASK_CARTPOLE_DISCRETE
        self.action_dim = self.sim.dofs if kind == N.TASK_PANDA_POSITION_TRACKING else 0
        f32 = dict(dtype=torch.float32, device=self.device)
        self.obs = torch.zeros((n_worlds, self.obs_dim), **f32)
        self.reward = torch.zeros((n_worlds,), **f32)
        self.done = torch.zeros((n_worlds,), dtype=torch.uint8, device=self.device)
        self.terminal_obs = torch.zeros((n_worlds, self.obs_dim), **f32)

    # ------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            N.lib().mw_vecenv_destroy(self._h)
            self._h = None
        if getattr(self, "sim", None) is not None:
            self.sim.close()
            self.sim = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_actions(self, actions, T: int = 0):
        torch = _torch()
        want = torch.int32 if self.discrete else torch.float32
        shape = (self.n_worlds,) if T == 0 else (T, self.n_worlds)
        if self.action_dim:
            shape = shape + (self.action_dim,)
        if not isinstance(actions, torch.Tensor) or actions.device != self.device:
            raise TypeError(f"actions must be a torch tensor on {self.device}")
        if actions.dtype != want or tuple(actions.shape) != shape or not actions.is_contiguous():
            raise TypeError(f"actions must be a contiguous {want} tensor of shape {shape}")

    def reset(self):
        """Reset every world (episode 0); returns obs [n_worlds, obs_dim]."""
        N.check(N.lib().mw_vecenv_reset(self._h, ctypes.c_void_p(self.obs.data_ptr())), "reset")
        return self.obs

    def step(self, actions) -> Tuple[object, object, object, Dict]:
        """Asynchronous on the current stream; returns views of reused buffers."""
        self._check_actions(actions)
        N.check(N.lib().mw_vecenv_step(
            self._h, ctypes.c_void_p(actions.data_ptr()), ctypes.c_void_p(self.obs.data_ptr()),
            ctypes.c_void_p(self.reward.data_ptr()), ctypes.c_void_p(self.done.data_ptr()),
            ctypes.c_void_p(self.terminal_obs.data_ptr())), "step")
        return self.obs, self.reward, self.done, {"terminal_obs": self.terminal_obs}

    def step_raw(self, actions_ptr: int) -> None:
        """Launch one step with a raw device pointer (bench / graph capture)."""
        N.lib().mw_vecenv_step(self._h, ctypes.c_void_p(actions_ptr),
                               ctypes.c_void_p(self.obs.data_ptr()),
                               ctypes.c_void_p(self.reward.data_ptr()),
                               ctypes.c_void_p(self.done.data_ptr()),
                               ctypes.c_void_p(self.terminal_obs.data_ptr()))

    def rollout(self, actions):
        """Open-loop T-step rollout in ONE launch: actions [T, n_worlds].

        Returns (obs [T, W, obs_dim], reward [T, W], done [T, W], terminal_obs)."""
        torch = _torch()
        T = actions.shape[0]
        self._check_actions(actions, T)
        obs = torch.empty((T, self.n_worlds, self.obs_dim), dtype=torch.float32, device=self.device)
        rew = torch.empty((T, self.n_worlds), dtype=torch.float32, device=self.device)
        done = torch.empty((T, self.n_worlds), dtype=torch.uint8, device=self.device)
        term = torch.zeros((T, self.n_worlds, self.obs_dim), dtype=torch.float32, device=self.device)
        N.check(N.lib().mw_vecenv_rollout(
            self._h, T, ctypes.c_void_p(actions.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
            ctypes.c_void_p(rew.data_ptr()), ctypes.c_void_p(done.data_ptr()),
            ctypes.c_void_p(term.data_ptr())), "rollout")
        return obs, rew, done, term

    def counters(self):
        """(episode, steps) per world as int32 tensors (copies of the uint32 counters)."""
        torch = _torch()
        ep = torch.empty((self.n_worlds,), dtype=torch.int32, device=self.device)
        st = torch.empty_like(ep)
        N.check(N.lib().mw_vecenv_counters(self._h, ctypes.c_void_p(ep.data_ptr()),
                                           ctypes.c_void_p(st.data_ptr())), "counters")
        return ep, st

    def physics(self):
        """(masses [dofs, n_worlds], gravity z [n_worlds]) of a randomised env."""
        torch = _torch()
        m = torch.empty((self.sim.dofs, self.n_worlds), dtype=torch.float32, device=self.device)
        gz = torch.empty((self.n_worlds,), dtype=torch.float32, device=self.device)
        N.check(N.lib().mw_vecenv_physics(self._h, ctypes.c_void_p(m.data_ptr()),
                                          ctypes.c_void_p(gz.data_ptr())), "physics")
        return m, gz

    def state(self):
        """(q, qd) float32 [dofs, n_worlds] copies of the device SoA state."""
        torch = _torch()
        q = torch.empty((self.sim.dofs, self.n_worlds), dtype=torch.float32, device=self.device)
        qd = torch.empty_like(q)
        N.check(N.lib().mw_copy_state(self.sim.handle, ctypes.c_void_p(q.data_ptr()),
                                      ctypes.c_void_p(qd.data_ptr()), 0), "state")
        return q, qd

    def set_state(self, q, qd) -> None:
        """Overwrite the device state (teacher forcing in parity tests)."""
        torch = _torch()
        q = q.to(device=self.device, dtype=torch.float32).contiguous()
        qd = qd.to(device=self.device, dtype=torch.float32).contiguous()
        assert tuple(q.shape) == (self.sim.dofs, self.n_worlds) == tuple(qd.shape)
        N.check(N.lib().mw_copy_state(self.sim.handle, ctypes.c_void_p(q.data_ptr()),
                                      ctypes.c_void_p(qd.data_ptr()), 1), "set_state")
        self._keep = (q, qd)  # alive until the async copy has run
