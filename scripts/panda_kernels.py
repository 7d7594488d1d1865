"""Config-4 Panda env: the one-world-per-lane kernel (kernels.hip:
vecenv_pid_step_kernel) against the one-world-per-16-lane-row kernel
(group_kernel.hip), in one process (the library reads MWSTEP_PANDA_KERNEL at
every launch).  Per world count: us per step from a hipGraph of 100 step
launches (HIP events on the launch stream), and the obs difference of the two
kernels after 300 tracking steps from the same reset.

    python scripts/panda_kernels.py [W ...]
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

import torch  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402


def targets(q0, T):
    t = torch.arange(T, device=q0.device, dtype=torch.float32) * 1e-3
    s = torch.sin(2 * math.pi * 0.33 * t)[:, None]
    tg = q0[None].repeat(T, 1, 1)
    tg[:, :, 0] += 0.9 * 2.8973 * s
    tg[:, :, 5] += 0.9 * 1.885 * s
    return tg.contiguous()


def time_kernel(kind, W, G=100, reps=5, **kw):
    os.environ["MWSTEP_PANDA_KERNEL"] = kind
    env = VecEnv("PandaPositionTracking", n_worlds=W, seed=1, max_episode_steps=5000, **kw)
    st = torch.cuda.Stream()
    env.sim.set_stream(st.cuda_stream)
    with torch.cuda.stream(st):
        q0 = env.reset()[:, :9].clone()
        tg = targets(q0, G)
        for t in range(G):
            env.step_raw(tg[t].data_ptr())
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for t in range(G):
                env.step_raw(tg[t].data_ptr())
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.replay()
        e1.record(st)
    st.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (G * reps)
    env.close()
    return us


def compare(W, H=300):
    outs = {}
    for kind in ("lane", "group"):
        os.environ["MWSTEP_PANDA_KERNEL"] = kind
        env = VecEnv("PandaPositionTracking", n_worlds=W, seed=4, max_episode_steps=5000)
        q0 = env.reset()[:, :9].clone()
        tg = targets(q0, H)
        rs = []
        for k in range(H):
            o, r, d, _ = env.step(tg[k])
            rs.append(r.clone())
        outs[kind] = (o.clone(), torch.stack(rs))
        env.close()
    do = float((outs["lane"][0] - outs["group"][0]).abs().max())
    dr = float(((outs["lane"][1] - outs["group"][1]).abs() / (1 + outs["lane"][1].abs())).max())
    return do, dr


def main():
    Ws = [int(a) for a in sys.argv[1:]] or [128, 1024, 4096]
    do, dr = compare(256)
    print(f"lane vs group after 300 steps, 256 worlds: max|obs diff| {do:.2e}, reward rel {dr:.2e}", flush=True)
    for W in Ws:
        a = time_kernel("lane", W)
        b = time_kernel("group", W)
        print(f"W={W}: lane {a:.2f} us/step, group {b:.2f} us/step ({a / b:.2f}x)", flush=True)
    if os.environ.get("PANDA_VARIANTS"):
        # cost structure of the group kernel at 1024 worlds: PGS sweeps, and
        # the marginal cost of a second substep per launch
        for label, kw in (("pgs 0", dict(pgs_iters=0)), ("pgs 1", dict(pgs_iters=1)),
                          ("2 substeps", dict(physics_rate=2000.0)), ("4 substeps", dict(physics_rate=4000.0))):
            print(f"  group W=1024 {label}: {time_kernel('group', 1024, **kw):.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
