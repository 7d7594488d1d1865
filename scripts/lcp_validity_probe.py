"""GPU probe behind tests/test_gpu_float_tree.py::test_one_step_exact_lcp_random_states:
runs the same adversarial one-step setup (W worlds, seed 11) and, for every
world whose GPU impulses are NOT a solution of the oracle's fp64 two-stage
LCP within the kernel's tolerance (tests/lcp_validity.py), saves the
problem, the GPU's warm records and both answers to
gpurun_out/validity_<model>_<world>.npz for offline replay.

    python scripts/lcp_validity_probe.py [model] [W]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gym-ignition_amd", "python")]

import pyoracle as oracle  # noqa: E402
from lcp_validity import validity, stage_boxes  # noqa: E402
from test_gpu_float_tree import _model, _quat_to_R, _random_states  # noqa: E402


def main():
    from mwstep import native as N
    from mwstep.sim import Simulator
    name = sys.argv[1] if len(sys.argv) > 1 else "icub"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    budget = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    os.environ["MWSTEP_WAVE_TREE"] = "1"
    text = _model(name)
    mu = 0.8
    rng = np.random.default_rng(11)
    cm = oracle.load_urdf(text)
    q, qd, pose, vel, tau = _random_states(cm, W, rng)
    sim = Simulator(text, n_worlds=W, pgs_iters=50)
    sim.set_lcp_solver(True, budget)
    sim.set_ground_plane(True, mu)
    sim.enable_contacts(True)
    sim.set("reset_q", q)
    sim.set("reset_qd", qd)
    sim.reset_base_pose(pose)
    sim.reset_base_velocity(vel)
    sim.run(paused=True)
    p0, v0 = sim.base_pose(), sim.base_velocity()
    gq0, gqd0 = sim.get("q"), sim.get("qd")
    sim.set_control_mode(N.MODE_FORCE)
    sim.set("force_target", tau)
    sim.run()
    gqd1 = sim.get("qd")
    state = sim.get_state()
    mode = np.full(cm.n, oracle.FORCE, np.int32)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    print(f"{name}: budget {budget}, GPU unconverged {sim.lcp_unconverged()}")
    for w in range(W):
        R0 = _quat_to_R(p0[w, 3:])
        ow = oracle.FloatWorld(cm, ground=True, mu=mu, pgs_iters=oracle.PGS_CONVERGED)
        ow.set_pose(p0[w, :3], R0)
        ow.set_twist(R0.T @ v0[w, 3:], R0.T @ v0[w, :3])
        ow.set_joints(gq0[w], gqd0[w])
        ow.step(mode, tau[w])
        p = oracle.lcp_last()
        if p is None:
            continue
        v = validity(p, state[w])
        if v["ratio"] <= 1.0:
            continue
        (L1, U1), (L2, U2) = stage_boxes(p, v["x1"])
        S = p["kind"] != 1
        e1, e2 = v["e1"], v["e2"]
        r1 = e1 / v["tol1"]
        r2 = e2 / v["tol2"]
        k1 = int(np.argmax(r1)) if S.any() else -1
        k2 = int(np.argmax(r2))
        e_qd = float(np.abs(gqd1[w] - ow.qd).max())
        gc = sim.contacts(w)
        print(f"world {w}: GPU contacts {len(gc)} oracle {len(ow.contacts)}, |dqd| {e_qd:.2e} rows {len(p['b'])} ratio1 {v['ratio1']:.2f} (row {np.flatnonzero(S)[k1] if k1 >= 0 else -1}"
              f" e {e1[k1] if k1 >= 0 else 0:.2e}) ratio2 {v['ratio2']:.2f} (row {k2} kind {p['kind'][k2]} e {e2[k2]:.2e}"
              f" x_gpu {v['x'][k2]:.4e} x_or {p['x'][k2]:.4e} L {L2[k2]:.3e} U {U2[k2]:.3e})")
        np.savez(os.path.join(out, f"validity_{name}_{w}_b{budget}.npz"), gpu_contacts=np.asarray(gc), **{k: np.asarray(val) for k, val in p.items()},
                 gpu_x=v["x"], gpu_x1=v["x1"], gpu_state=state[w], e1=e1, e2=e2,
                 gqd0=gqd0[w], gqd1=gqd1[w], oqd1=ow.qd, tau=tau[w])
    sim.close()


if __name__ == "__main__":
    main()
