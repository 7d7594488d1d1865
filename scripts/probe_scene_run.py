"""Where the time of one synchronous ScenarI/O run() goes on the scene
backend (1 CartPole world, BASELINE config 1's shape): the full mw_scene_run
(command upload, launch, readback copies, one synchronisation) vs the launch +
synchronisation alone vs an empty synchronisation, and the chain kernel's
mw_run for the same model.  python scripts/probe_scene_run.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mwstep import get_model_file  # noqa: E402
from mwstep import native as N  # noqa: E402
from mwstep.scene import Scene  # noqa: E402
from mwstep.sim import Simulator  # noqa: E402

T = 3000
stream = torch.cuda.Stream()
sc = Scene(n_worlds=1)
sc.set_stream(stream.cuda_stream)
sc.insert_model(get_model_file("cartpole"), (0, 0, 0, 1, 0, 0, 0), "cartpole")
sc.set_control_mode(N.MODE_FORCE, m=0)
sc.run()


def timeit(fn, n=T):
    for _ in range(100):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


f = np.array([[1.0, 0.0]])
print(f"mw_scene_run (no commands)          {timeit(lambda: sc.run()):7.1f} us")
print(f"mw_scene_run + force command         {timeit(lambda: (sc.set('force_target', f, m=0), sc.run())):7.1f} us")
print(f"mw_scene_run_device(1) + stream sync {timeit(lambda: (sc.run_device(1), stream.synchronize())):7.1f} us")
print(f"stream sync alone                    {timeit(lambda: stream.synchronize()):7.1f} us")
buf = torch.empty(64, device="cuda")
hbuf = torch.empty(64, pin_memory=True)
print(f"64-float D2H copy + sync             {timeit(lambda: (hbuf.copy_(buf, non_blocking=True), torch.cuda.synchronize())):7.1f} us")
sim = Simulator(get_model_file("cartpole"), n_worlds=1)
sim.set_control_mode(N.MODE_FORCE)
print(f"mw_run (chain kernel) + force        {timeit(lambda: (sim.set('force_target', f), sim.run())):7.1f} us")
