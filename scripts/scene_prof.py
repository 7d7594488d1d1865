"""Scene kernel timings for rocprofv3: (a) one CartPole world (the ScenarI/O
runtime path), (b) 4096 three-cube worlds (the bench scene leg)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402
from mwstep import get_model_file  # noqa: E402
from mwstep import native as N  # noqa: E402
from mwstep.scene import Scene  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
if which in ("cartpole", "both"):
    sc = Scene(n_worlds=1, pgs_iters=50)
    sc.set_ground_plane(True, 1.0)
    sc.insert_model(get_model_file("cartpole"), (0, 0, 0, 1, 0, 0, 0), "cartpole")
    sc.run(paused=True)
    sc.set_control_mode(N.MODE_FORCE, m=0, dofs=[0])
    t0 = time.perf_counter()
    for k in range(300):
        sc.set("force_target", [[20.0 if k % 2 else -20.0]], m=0, dofs=[0])
        sc.run()
        sc.get("q", 0)
    print(f"cartpole scene W=1: {(time.perf_counter() - t0) / 300 * 1e6:.1f} us per run (host loop)")
    sc.close()
if which in ("cubes", "both"):
    W = int(os.environ.get("SCENE_W", "4096"))
    sc = Scene(n_worlds=W, pgs_iters=50)
    sc.set_ground_plane(True, 1.0)
    for k, p in enumerate([(0, -0.15, 0.101), (0, 0.15, 0.101), (0, 0, 0.301)]):
        sc.insert_model(get_model_file("cube"), tuple(p) + (1, 0, 0, 0), f"cube{k + 1}")
    sc.run(paused=True)
    sc.run_device(60)
    sc.run()
    print(f"three cubes x{W}: contacts world 0 {len(sc.contacts(0))}")
    sc.close()
