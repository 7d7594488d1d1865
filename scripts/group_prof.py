"""Phase breakdown of the one-world-per-16-lane-row Panda kernel
(group_kernel.hip) on BASELINE config 4's workload (PandaPositionTracking,
C4 sinusoid targets).

Needs the debug build with shader-clock phase counters:
    make -C gym-ignition_amd BUILD=build_prof LIB=libmwstep_prof.so EXTRA=-DMW_GROUP_PROF
    MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so python scripts/group_prof.py [W]
Prints shader-clock cycles per world-step of every phase (lane 0 of each world)."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import torch  # noqa: E402

from mwstep import native as N  # noqa: E402
from mwstep.vecenv import VecEnv  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
T = 50
PHASES = ["prologue (params, state loads)", "PID + poses (pointer jumping)", "inertias, composites, M rows",
          "RNEA bias", "Cholesky + solve", "LCP rows + M^-1 columns", "PGS", "epilogue (reward, reset, stores)",
          "whole kernel"]
env = VecEnv("PandaPositionTracking", n_worlds=W, seed=42)
q0 = env.reset()[:, :9].clone()
t = torch.arange(T + 20, device="cuda", dtype=torch.float32) * 1e-3
s = torch.sin(2 * math.pi * 0.33 * t)[:, None]
tg = q0[None].repeat(T + 20, 1, 1)
tg[:, :, 0] += 0.9 * 2.8973 * s
tg[:, :, 5] += 0.9 * 1.885 * s
tg = tg.contiguous()
L = N.lib()
fn = L.mw_debug_group_prof
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 10)()
for k in range(20):
    env.step(tg[k])
torch.cuda.synchronize()
fn(buf)  # clear
for k in range(20, 20 + T):
    env.step(tg[k])
torch.cuda.synchronize()
fn(buf)
print(f"{W} worlds, {T} steps")
for k, name in enumerate(PHASES):
    print(f"  {name:36s} {buf[k] / W / T:10.0f} cycles/world-step")
print(f"  PGS sweeps {buf[9] / W / T:.2f} per world-step")
env.close()
