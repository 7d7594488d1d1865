"""A/B timing of libmwstep build variants in ONE process (interleaved rounds).

    python scripts/ab_variants.py lib1.so lib2.so ...

Per variant and round: (1) a fused 500-step rollout launch (HIP events on
the launch stream): per-step compute of vecenv_step_kernel without launch
gaps; (2) a hipGraph of 100 per-step launches: the closed-loop path of
bench.py.  4096 CartPole worlds.  Prints the median over rounds."""

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import torch  # noqa: E402

from mwstep import native as N  # noqa: E402  (structs + signatures only)
from mwstep.models import get_model_file  # noqa: E402


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
        assert L.mw_load_model(self.h, get_model_file("cartpole").encode(), p, b"") == 0
        assert L.mw_set_stream(self.h, ctypes.c_void_p(stream.cuda_stream)) == 0
        assert L.mw_initialize(self.h) == 0, L.mw_last_error()
        t = N.MwTaskConfig(0, 5000, 1, 0, 42)
        self.e = ctypes.c_void_p()
        assert L.mw_vecenv_create(self.h, ctypes.byref(t), ctypes.byref(self.e)) == 0
        f = dict(dtype=torch.float32, device="cuda")
        self.obs = torch.zeros((W, 4), **f)
        self.rew = torch.zeros((W,), **f)
        self.done = torch.zeros((W,), dtype=torch.uint8, device="cuda")
        self.term = torch.zeros((W, 4), **f)
        assert L.mw_vecenv_reset(self.e, ctypes.c_void_p(self.obs.data_ptr())) == 0

    def step(self, a):
        self.L.mw_vecenv_step(self.e, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(self.obs.data_ptr()),
                              ctypes.c_void_p(self.rew.data_ptr()), ctypes.c_void_p(self.done.data_ptr()),
                              ctypes.c_void_p(self.term.data_ptr()))

    def rollout(self, acts, o, r, d, t):
        T = acts.shape[0]
        assert self.L.mw_vecenv_rollout(self.e, T, ctypes.c_void_p(acts.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                                        ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                                        ctypes.c_void_p(t.data_ptr())) == 0


def main():
    libs = sys.argv[1:]
    W, T, G, rounds = 4096, 500, 100, 7
    stream = torch.cuda.Stream()
    acts = torch.randint(0, 2, (T, W), device="cuda", dtype=torch.int32)
    o = torch.empty((T, W, 4), device="cuda")
    r = torch.empty((T, W), device="cuda")
    d = torch.empty((T, W), dtype=torch.uint8, device="cuda")
    t = torch.zeros((T, W, 4), device="cuda")
    envs, graphs = [], []
    for path in libs:
        env = Env(load(path), W, stream)
        with torch.cuda.stream(stream):
            for k in range(20):
                env.step(acts[k])
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for k in range(G):
                    env.step(acts[k])
        envs.append(env)
        graphs.append(g)
    res = {p: {"rollout_us_per_step": [], "graph_us_per_step": []} for p in libs}
    for _ in range(rounds):
        for p, env, g in zip(libs, envs, graphs):
            with torch.cuda.stream(stream):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(stream)
                env.rollout(acts, o, r, d, t)
                e1.record(stream)
                g.replay()
                e2.record(stream)
            stream.synchronize()
            res[p]["rollout_us_per_step"].append(e0.elapsed_time(e1) * 1e3 / T)
            res[p]["graph_us_per_step"].append(e1.elapsed_time(e2) * 1e3 / G)
    out = {os.path.basename(p): {k: round(statistics.median(v), 4) for k, v in d_.items()}
           for p, d_ in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
