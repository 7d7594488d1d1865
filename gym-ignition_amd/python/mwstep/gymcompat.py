"""Minimal stand-in for the parts of OpenAI ``gym`` the reference's hot path uses.

``gym`` is a declared dependency of the reference (``python/gym_ignition/base/
runtime.py:5``, ``base/task.py:6``) but it is not installed in this image.  The
host-side mirror imports the real ``gym`` when it is available and falls back to
this module otherwise.  What is restated (gym 0.17/0.18 behaviour):

  * ``spaces.Box`` / ``spaces.Discrete``: ``contains``, ``sample``, ``seed``
    (float32 bounds, uniform sampling from the space's own RandomState);
  * ``utils.seeding.np_random``: sha512-hashed seed -> ``RandomState``, so the
    task RNG streams are the ones the reference sees for the same seed;
  * ``Env``, ``Wrapper``, ``envs.registration.register`` / ``make`` with the
    ``TimeLimit`` wrapper (``max_episode_steps``).
"""

from __future__ import annotations

import hashlib
import os
import struct
import types
from typing import Any, Dict, Optional

import numpy as np


# ------------------------------------------------------------------ seeding
def _bigint_from_bytes(data: bytes) -> int:
    pad = (4 - len(data) % 4) % 4 or 4
    data = data + b"\0" * pad
    words = struct.unpack(f"{len(data) // 4}I", data)
    return sum(w << (32 * i) for i, w in enumerate(words))


def _int_list_from_bigint(v: int):
    if v < 0:
        raise ValueError("seed must be non-negative")
    if v == 0:
        return [0]
    out = []
    while v > 0:
        v, mod = divmod(v, 2 ** 32)
        out.append(mod)
    return out


def _create_seed(a: Optional[int] = None, max_bytes: int = 8) -> int:
    if a is None:
        return _bigint_from_bytes(os.urandom(max_bytes))
    if isinstance(a, str):
        a = a.encode("utf8")
        a += hashlib.sha512(a).digest()
        return _bigint_from_bytes(a[:max_bytes])
    return int(a) % 2 ** (8 * max_bytes)


def _hash_seed(seed: Optional[int] = None, max_bytes: int = 8) -> int:
    if seed is None:
        seed = _create_seed(max_bytes=max_bytes)
    digest = hashlib.sha512(str(seed).encode("utf8")).digest()
    return _bigint_from_bytes(digest[:max_bytes])


def np_random(seed: Optional[int] = None):
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a non-negative integer or omitted, not {seed!r}")
    seed = _create_seed(seed)
    rng = np.random.RandomState()
    rng.seed(_int_list_from_bigint(_hash_seed(seed)))
    return rng, seed


utils = types.SimpleNamespace(seeding=types.SimpleNamespace(np_random=np_random))


# ------------------------------------------------------------------- spaces
class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random, _ = np_random()

    def seed(self, seed: Optional[int] = None):
        self.np_random, seed = np_random(seed)
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.shape(low) else np.shape(high)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
        super().__init__(shape, dtype)

    def sample(self):
        high = self.high if self.dtype.kind == "f" else self.high.astype("int64") + 1
        return self.np_random.uniform(low=self.low, high=high, size=self.shape).astype(self.dtype)

    def contains(self, x) -> bool:
        if isinstance(x, list):
            x = np.array(x)
        x = np.asarray(x)
        if x.shape != self.shape:
            return False
        if x.size <= 16:
            # the per-env path checks a handful of values per step: Python
            # floats beat two numpy reductions (NaN fails either way)
            return all(lo <= v <= hi for v, lo, hi in
                       zip(x.ravel().tolist(), self.low.ravel().tolist(), self.high.ravel().tolist()))
        return bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


class Discrete(Space):
    def __init__(self, n: int):
        self.n = int(n)
        super().__init__((), np.int64)

    def sample(self):
        return int(self.np_random.randint(self.n))

    def contains(self, x) -> bool:
        if isinstance(x, (int, np.integer)):
            v = int(x)
        elif isinstance(x, np.ndarray) and x.shape == () and x.dtype.kind in "iu":
            v = int(x)
        else:
            return False
        return 0 <= v < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


spaces = types.SimpleNamespace(Space=Space, Box=Box, Discrete=Discrete)


# ---------------------------------------------------------------- Env / make
class Env:
    metadata: Dict[str, Any] = {"render.modes": []}
    action_space = None
    observation_space = None
    spec = None

    @property
    def unwrapped(self):
        return self

    def close(self):
        pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.action_space = env.action_space
        self.observation_space = env.observation_space

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def seed(self, seed=None):
        return self.env.seed(seed)

    def render(self, mode="human", **kwargs):
        return self.env.render(mode, **kwargs)

    def close(self):
        return self.env.close()


class TimeLimit(Wrapper):
    def __init__(self, env, max_episode_steps: int):
        super().__init__(env)
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = None

    def step(self, action):
        assert self._elapsed_steps is not None, "Cannot call env.step() before calling reset()"
        obs, reward, done, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            info["TimeLimit.truncated"] = not done
            done = True
        return obs, reward, done, info

    def reset(self, **kwargs):
        self._elapsed_steps = 0
        return self.env.reset(**kwargs)


class EnvSpec:
    def __init__(self, id: str, entry_point: str, max_episode_steps: Optional[int] = None,
                 kwargs: Optional[dict] = None):
        self.id = id
        self.entry_point = entry_point
        self.max_episode_steps = max_episode_steps
        self._kwargs = dict(kwargs or {})

    def make(self, **kwargs):
        mod_name, cls_name = self.entry_point.split(":")
        import importlib
        cls = getattr(importlib.import_module(mod_name), cls_name)
        kw = dict(self._kwargs)
        kw.update(kwargs)
        env = cls(**kw)
        env.spec = self
        return env


class _Registry:
    def __init__(self):
        self.env_specs: Dict[str, EnvSpec] = {}

    def register(self, id: str, **kwargs):
        if id in self.env_specs:
            raise ValueError(f"Cannot re-register id: {id}")
        self.env_specs[id] = EnvSpec(id, **kwargs)

    def make(self, id: str, **kwargs):
        spec = self.env_specs[id]
        env = spec.make(**kwargs)
        if spec.max_episode_steps is not None:
            env = TimeLimit(env, spec.max_episode_steps)
        return env

    def all(self):
        return self.env_specs.values()


registry = _Registry()


def register(id: str, **kwargs):
    registry.register(id, **kwargs)


def make(id: str, **kwargs):
    return registry.make(id, **kwargs)


envs = types.SimpleNamespace(registration=types.SimpleNamespace(register=register),
                             registry=registry)


class _Logger:
    DEBUG, INFO, WARN, ERROR, DISABLED = 10, 20, 30, 40, 50

    def __init__(self):
        self.level = self.WARN

    def set_level(self, level: int):
        self.level = level

    def _log(self, lvl, tag, msg, *args):
        if self.level <= lvl:
            print(f"{tag}: {msg % args if args else msg}")

    def debug(self, msg, *a): self._log(self.DEBUG, "DEBUG", msg, *a)
    def info(self, msg, *a): self._log(self.INFO, "INFO", msg, *a)
    def warn(self, msg, *a): self._log(self.WARN, "WARN", msg, *a)
    def error(self, msg, *a): self._log(self.ERROR, "ERROR", msg, *a)


logger = _Logger()
