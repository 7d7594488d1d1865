"""Debug the scene one-step parity: per failing world, which model differs
and the contact set (GPU vs oracle)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as oracle  # noqa: E402
from test_gpu_scene import _oracle_from_gpu, _rand_quat, _scene  # noqa: E402
from scene_models import cube_urdf, sphere_urdf  # noqa: E402
from test_float_tree_oracle import chain_urdf  # noqa: E402
from mwstep import native as N  # noqa: E402

W, pgs, mu = 256, 50, 0.8
rng = np.random.default_rng(7)
texts = [cube_urdf(), cube_urdf(double_collision=True, mass=2.0, edge=0.15), sphere_urdf(1.0, 0.08), chain_urdf(3)]
names = ["cube1", "cube2", "ball", "chain"]
base_z = [0.1, 0.28, 0.45, 0.6]
cms = [oracle.load_urdf(t, pose_xyz=(0, 0, z)) for t, z in zip(texts, base_z)]
sc = _scene([(t, (0, 0, z, 1, 0, 0, 0), nm) for t, z, nm in zip(texts, base_z, names)], W, pgs, mu)
for m, z in enumerate(base_z):
    poses = np.array([np.concatenate([rng.uniform(-0.06, 0.06, 2), [z + rng.uniform(-0.03, 0.02)],
                                      _rand_quat(rng, 0.4)]) for _ in range(W)])
    sc.reset_base_pose(m, poses)
    sc.reset_base_velocity(m, np.column_stack([rng.uniform(-0.5, 0.5, (W, 3)), rng.uniform(-1, 1, (W, 3))]))
nj = cms[3].n
sc.set("reset_q", rng.uniform(-1, 1, (W, nj)), m=3)
sc.set("reset_qd", rng.uniform(-2, 2, (W, nj)), m=3)
sc.run(paused=True)
sc.set_control_mode(N.MODE_FORCE, m=3)
tau = rng.uniform(-5, 5, (W, nj)).astype(np.float32).astype(np.float64)
sc.set("force_target", tau, m=3)
mode = sys.argv[1] if len(sys.argv) > 1 else "full"
orcs = [_oracle_from_gpu(oracle, cms, sc, w, pgs, mu) for w in range(W)]
start_pose = [sc.base_pose(m) for m in range(4)]
start_vel = [sc.base_velocity(m) for m in range(4)]
start_q = sc.get("q", 3)
start_qd = sc.get("qd", 3)
sc.run()
np.set_printoptions(precision=4, suppress=True, linewidth=160)
nbad = 0
for w in range(W):
    ow = orcs[w]
    ow.mode[3, :nj] = oracle.FORCE
    ow.cmd[3, :nj] = tau[w]
    ow.step()
    errs = []
    for m in range(4):
        R = ow.R(m)
        v = sc.base_velocity(m, w, 1)[0]
        errs.append(float(np.abs(v - np.concatenate([R @ ow.V(m)[3:], R @ ow.V(m)[:3]])).max()))
    eq = float(np.abs(sc.get("qd", 3, w, 1)[0] - ow.qd(3)).max())
    gc = sc.contacts(w)
    if max(errs) > 2e-3 or eq > 2e-3:
        nbad += 1
        if nbad <= 3 or w == 9:
            print(f"world {w}: vel err per model {np.array(errs)}, chain qd err {eq:.3e}, contacts gpu {len(gc)} oracle {len(ow.contacts)}")
            for row, (oc, who) in zip(gc, ow.contacts):
                print("   gpu", row[:3], row[3:6], row[6:9], f"{row[9]:.4f}", row[10:14].astype(int))
                print("   orc", oc[:3], oc[3:6], oc[6:9], f"{oc[9]:.4f}", who)
print("bad worlds", nbad, "of", W, "overflow", sc.overflow())

# ---- world 9 alone: same start state in a 1-world scene
from mwstep.scene import Scene  # noqa: E402
wdbg = int(os.environ.get("WDBG", "9"))
ow = orcs[wdbg]
# the oracle object was stepped above; rebuild the start state from a fresh snapshot of the inputs
start = _oracle_from_gpu(oracle, cms, sc, wdbg, pgs, mu)  # post-step GPU state (for reference only)
print("post-step GPU vs oracle V per model:")
for m in range(4):
    R = ow.R(m)
    print(m, sc.base_velocity(m, wdbg, 1)[0], np.concatenate([R @ ow.V(m)[3:], R @ ow.V(m)[:3]]))
s1 = _scene([(t, (0, 0, z, 1, 0, 0, 0), nm) for t, z, nm in zip(texts, base_z, names)], 1, pgs, mu)
for m in range(4):
    s1.reset_base_pose(m, start_pose[m][wdbg:wdbg + 1])
    s1.reset_base_velocity(m, start_vel[m][wdbg:wdbg + 1])
s1.set("reset_q", start_q[wdbg:wdbg + 1], m=3)
s1.set("reset_qd", start_qd[wdbg:wdbg + 1], m=3)
s1.run(paused=True)
s1.set_control_mode(N.MODE_FORCE, m=3)
print("alone pre-step pose diff", max(float(np.abs(s1.base_pose(m)[0] - start_pose[m][wdbg]).max()) for m in range(4)),
      "vel diff", max(float(np.abs(s1.base_velocity(m)[0] - start_vel[m][wdbg]).max()) for m in range(4)))
s1.set("force_target", tau[wdbg:wdbg + 1], m=3)
s1.run()
print("alone post-step V per model vs batched:")
for m in range(4):
    print(m, s1.base_velocity(m)[0], sc.base_velocity(m, wdbg, 1)[0])
oc = _oracle_from_gpu(oracle, cms, s1, 0, -1, mu)
np.savez(os.path.join(ROOT, "gpurun_out", f"scene_w{wdbg}.npz"),
         pose=np.array([start_pose[m][wdbg] for m in range(4)]), vel=np.array([start_vel[m][wdbg] for m in range(4)]),
         q=start_q[wdbg], qd=start_qd[wdbg], tau=tau[wdbg],
         post_pose=np.array([s1.base_pose(m)[0] for m in range(4)]),
         post_vel=np.array([s1.base_velocity(m)[0] for m in range(4)]),
         post_q=s1.get("q", 3)[0], post_qd=s1.get("qd", 3)[0], contacts=s1.contacts(0))
