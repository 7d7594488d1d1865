"""Where does the time of a SHORT timed region go (the driver runs bench.py
--steps 20 --warmup 5)?  CartPole, 4096 worlds, one 20-step hipGraph.

Times, each over many repetitions (min / median, microseconds):
  sync_only   : synchronize; t0; synchronize; t1             (timer + sync floor)
  torch_replay: synchronize; t0; graph.replay(); synchronize  (bench.py today)
  hip_launch  : the same graph exec launched with hipGraphLaunch through ctypes
  events      : HIP-event time of the replayed graph (GPU side only)
"""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import torch  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402


def stats(xs):
    xs = sorted(xs)
    return {"min": round(xs[0] * 1e6, 2), "med": round(statistics.median(xs) * 1e6, 2)}


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    env = VecEnv("CartPoleDiscreteBalancing", n_worlds=4096, device=0, seed=42)
    st = torch.cuda.Stream(device=dev)
    env.sim.set_stream(st.cuda_stream)
    acts = torch.randint(0, 2, (K + 5, 4096), device=dev, dtype=torch.int32)
    with torch.cuda.stream(st):
        env.reset()
        for t in range(5):
            env.step_raw(acts[t].data_ptr())
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for t in range(5, 5 + K):
                env.step_raw(acts[t].data_ptr())
        g.replay()
    st.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    exe = g.raw_cuda_graph_exec()
    sp = st.cuda_stream
    R = 200
    out = {}
    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t0)
    out["sync_only"] = stats(xs)
    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            g.replay()
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t0)
    out["torch_replay"] = stats(xs)
    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        hip.hipGraphLaunch(exe, sp)
        hip.hipStreamSynchronize(sp)
        xs.append(time.perf_counter() - t0)
    out["hip_launch_streamsync"] = stats(xs)
    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        hip.hipGraphLaunch(exe, sp)
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t0)
    out["hip_launch_devsync"] = stats(xs)
    xs = []
    for _ in range(R):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(st)
        hip.hipGraphLaunch(exe, sp)
        e1.record(st)
        torch.cuda.synchronize(dev)
        xs.append(e0.elapsed_time(e1) * 1e-3)
    out["events"] = stats(xs)
    # eager launches (no graph): K step_raw calls
    xs = []
    for _ in range(R):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for t in range(5, 5 + K):
            env.step_raw(acts[t].data_ptr())
        torch.cuda.synchronize(dev)
        xs.append(time.perf_counter() - t0)
    out["eager"] = stats(xs)
    out["K"] = K
    print(out, flush=True)
    env.close()


if __name__ == "__main__":
    main()
