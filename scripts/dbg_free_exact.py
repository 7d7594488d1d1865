"""Debug probe (r04): the free-body parity states of tests/test_gpu_free_body.py
on the wave kernel's exact LCP -- per world the GPU-oracle velocity error,
contact count and the per-contact force differences of the worst worlds.

    python scripts/dbg_free_exact.py [cube|double|cylinder|rock]
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in ("oracle", "tests", "gym-ignition_amd/python"):
    sys.path.insert(0, os.path.join(ROOT, p))
import pyoracle as oracle  # noqa: E402
from test_cylinder_oracle import cylinder_urdf  # noqa: E402
from test_free_body_oracle import cube_urdf  # noqa: E402
from test_gpu_free_body import _quat_to_R, _rock_body_urdf  # noqa: E402
from mwstep.sim import Simulator  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "double"
text = {"cube": cube_urdf, "double": lambda: cube_urdf(True),
        "cylinder": lambda: cylinder_urdf(rpy="0.2 0 0"), "rock": _rock_body_urdf}[name]()
W = 256
rng = np.random.default_rng(5)
sim = Simulator(text, n_worlds=W, pgs_iters=50, lcp_exact=True)
sim.set_ground_plane(True, 0.8)
sim.enable_contacts(True)
q = rng.normal(size=(W, 4))
q /= np.linalg.norm(q, axis=1, keepdims=True)
zr = (0.0, 0.09) if name == "rock" else (0.05, 0.2)
pos = np.column_stack([rng.uniform(-1, 1, W), rng.uniform(-1, 1, W), rng.uniform(*zr, W)])
lin = rng.uniform(-0.5, 0.5, (W, 3))
ang = rng.uniform(-2, 2, (W, 3))
sim.reset_base_pose(np.column_stack([pos, q]).astype(np.float32).astype(np.float64))
sim.reset_base_velocity(np.column_stack([lin, ang]).astype(np.float32).astype(np.float64))
sim.run(paused=True)
p0, v0 = sim.base_pose(), sim.base_velocity()
sim.run()
v1 = sim.base_velocity()
print(f"{name}: GPU unconverged {sim.lcp_unconverged()}/{W}, overflow {sim.constraint_overflow()}")
cm = oracle.load_urdf(text)
errs = []
for w in range(W):
    R0 = _quat_to_R(p0[w, 3:])
    ow = oracle.FreeWorld(cm, ground=True, mu=0.8, pgs_iters=oracle.PGS_CONVERGED)
    ow.set_pose(p0[w, :3], R0)
    ow.set_twist(R0.T @ v0[w, 3:], R0.T @ v0[w, :3])
    ow.step()
    wv = np.concatenate([ow.R @ ow.twist[1], ow.R @ ow.twist[0]])
    errs.append((float(np.abs(v1[w] - wv).max()), w, ow))
errs.sort(key=lambda e: -e[0])
print("worst velocity errors:", [(w, f"{e:.2e}", len(ow.contacts)) for e, w, ow in errs[:12]])
print("worlds with error > 1e-3:", sum(e > 1e-3 for e, _, _ in errs), "of", W)
for e, w, ow in errs[:3]:
    gc = sim.contacts(w)
    print(f"world {w}: err {e:.3e}, {len(gc)} contacts")
    for row, (p, n, f, d) in zip(gc, ow.contacts):
        print("   p", np.round(row[0:3], 4), "gpu f", np.round(row[6:9], 4), "oracle f", np.round(f, 4), "depth", round(d, 5))
