"""A/B timing of libmwstep build variants on the config-4 Panda env, in ONE
process (interleaved rounds): a hipGraph of 100 PandaPositionTracking step
launches (C4 sinusoid targets), HIP events on the launch stream.

    python scripts/ab_panda.py [--worlds 1024] lib1.so lib2.so ..."""

import argparse
import ctypes
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mwstep import native as N  # noqa: E402
from mwstep.models import PANDA_PID_GAINS_1000HZ, get_model_file  # noqa: E402


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, res, args in N.SIGNATURES:
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


class Env:
    def __init__(self, L, W, stream):
        self.L, self.W = L, W
        cfg = N.MwConfig(1e-3, 1.0, 1, W, 0, 20)
        self.h = ctypes.c_void_p()
        assert L.mw_create(ctypes.byref(cfg), ctypes.byref(self.h)) == 0
        p = (ctypes.c_double * 7)(0, 0, 0, 1, 0, 0, 0)
        assert L.mw_load_model(self.h, get_model_file("panda").encode(), p, b"") == 0, L.mw_last_error()
        assert L.mw_set_stream(self.h, ctypes.c_void_p(stream.cuda_stream)) == 0
        assert L.mw_initialize(self.h) == 0, L.mw_last_error()
        big = float(np.finfo(np.float64).max)
        buf = ctypes.create_string_buffer(64)
        for d in range(9):
            L.mw_joint_name(self.h, d, buf, 64)
            pp, ii, dd = PANDA_PID_GAINS_1000HZ[buf.value.decode()]
            g = (ctypes.c_double * 8)(pp, ii, dd, -big, big, 0.0, -big, big)
            assert L.mw_set_joint_pid(self.h, d, g) == 0
        t = N.MwTaskConfig(N.TASK_PANDA_POSITION_TRACKING, 5000, 1, 0, 42)
        self.e = ctypes.c_void_p()
        assert L.mw_vecenv_create(self.h, ctypes.byref(t), ctypes.byref(self.e)) == 0, L.mw_last_error()
        f = dict(dtype=torch.float32, device="cuda")
        self.obs = torch.zeros((W, 18), **f)
        self.rew = torch.zeros((W,), **f)
        self.done = torch.zeros((W,), dtype=torch.uint8, device="cuda")
        self.term = torch.zeros((W, 18), **f)
        assert L.mw_vecenv_reset(self.e, ctypes.c_void_p(self.obs.data_ptr())) == 0

    def step(self, a):
        self.L.mw_vecenv_step(self.e, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(self.obs.data_ptr()),
                              ctypes.c_void_p(self.rew.data_ptr()), ctypes.c_void_p(self.done.data_ptr()),
                              ctypes.c_void_p(self.term.data_ptr()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    W, G = a.worlds, 100
    stream = torch.cuda.Stream()
    envs, graphs, tg = [], [], []
    with torch.cuda.stream(stream):
        for path in a.libs:
            env = Env(load(path), W, stream)
            q0 = env.obs[:, :9].clone()
            t = torch.arange(G, device="cuda", dtype=torch.float32) * 1e-3
            s = torch.sin(2 * math.pi * 0.33 * t)[:, None]
            targets = q0[None].repeat(G, 1, 1)
            targets[:, :, 0] += 0.9 * 2.8973 * s
            targets[:, :, 5] += 0.9 * 1.885 * s
            targets = targets.contiguous()
            for g in range(G):
                env.step(targets[g])
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for g in range(G):
                    env.step(targets[g])
            graph.replay()
            envs.append(env)
            graphs.append(graph)
            tg.append(targets)
    stream.synchronize()
    times = [[] for _ in a.libs]
    for _ in range(a.rounds):
        for i, graph in enumerate(graphs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                graph.replay()
                e1.record(stream)
            stream.synchronize()
            times[i].append(e0.elapsed_time(e1) * 1e3 / G)
    for path, t in zip(a.libs, times):
        us = statistics.median(t)
        print(f"{os.path.basename(path):28s} W={W}: {us:8.3f} us/step  {W / (us * 1e-6):14.1f} env-steps/s")


if __name__ == "__main__":
    main()
