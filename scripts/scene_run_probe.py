"""Time mw_scene_run on the per-env path's scene (one CartPole world, steps
per run 1, ground plane) in a tight loop: unpaused, paused (launch + sync
floor) and with the PGS / exact-LCP variants, to split the per-env step.
    python scripts/scene_run_probe.py [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402

from mwstep import get_model_file  # noqa: E402
from mwstep.scene import Scene  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
if os.environ.get("SPIN"):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin | yield)", hip.hipSetDeviceFlags(int(os.environ["SPIN"])))


def make(exact=True):
    sc = Scene(n_worlds=1, step_size=1e-3, steps_per_run=1)
    sc.set_ground_plane(True, 1.0) if hasattr(sc, "set_ground_plane") else None
    sc.insert_model(get_model_file("cartpole"))
    if not exact:
        sc.set_lcp_solver(False)
    sc.run(paused=True)
    return sc


def timeit(fn, n):
    for _ in range(200):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


sc = make()
f = np.zeros((1, sc._nd))
print(f"scene: {sc._nd} dofs, contacts {len(sc.contacts(0)) if hasattr(sc, 'contacts') else '?'}")
print(f"run(paused)            {timeit(lambda: sc.run(paused=True), iters):7.1f} us")
print(f"run()                  {timeit(lambda: sc.run(), iters):7.1f} us")


def cmd_run():
    sc.set("reset_qd", f, m=0)
    sc.run()


print(f"set qd + run()         {timeit(cmd_run, iters):7.1f} us")
sc.close()
sc = make(exact=False)
print(f"run() PGS only         {timeit(lambda: sc.run(), iters):7.1f} us")
sc.close()
