"""The oracle's conditioning probe (oracle.c or_set_lcp_perturbation, test
infrastructure): off, the exact LCP solve is untouched (bit-identical steps);
on, every solve sees its Delassus matrix with symmetric relative errors of
the given size, and the step moves by a bounded amount (a standing
humanoid: ~1e-6 in qd at 1e-6 relative; the parity tests' random impacts
move by up to 0.2, tests/test_gpu_float_tree.py)."""

import numpy as np


def _humanoid_stand(oracle, steps):
    from mwstep import get_model_file
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    cm = oracle.load_urdf(get_model_file("icub"), pose_xyz=ICUB_POSE[:3], pose_wxyz=ICUB_POSE[3:])
    ow = oracle.FloatWorld(cm, ground=True, mu=1.0, pgs_iters=oracle.PGS_CONVERGED)
    n = cm.n
    post = np.array(icub_posture(cm.joint_names))
    ow.set_joints(post, np.zeros(n))
    mode = np.full(n, oracle.FORCE, np.int32)
    kp = np.array([p for p, _ in icub_pid_gains(cm.joint_names)])
    for _ in range(steps):
        ow.step(mode, np.clip(-kp * (ow.q - post) - 0.01 * kp * ow.qd, -80, 80))
    return cm, ow


def test_probe_off_is_bit_identical_and_on_moves_redundant_contacts(oracle):
    cm, ow = _humanoid_stand(oracle, 60)
    state = (ow.p.copy(), ow.R.copy(), ow.V.copy(), ow.q.copy(), ow.qd.copy())
    mode = np.full(cm.n, oracle.FORCE, np.int32)
    tau = np.zeros(cm.n)

    def step(eps, seed):
        oracle.set_lcp_perturbation(eps, seed)
        try:
            w = oracle.FloatWorld(cm, ground=True, mu=1.0, pgs_iters=oracle.PGS_CONVERGED)
            w.set_pose(state[0], state[1])
            w.set_twist(state[2][:3], state[2][3:])
            w.set_joints(state[3], state[4])
            w.step(mode, tau)
            return w.qd.copy(), len(w.contacts)
        finally:
            oracle.set_lcp_perturbation(0.0)

    base, nc = step(0.0, 0)
    assert nc >= 4
    assert np.array_equal(step(0.0, 7)[0], base)
    moved = max(float(np.abs(step(1e-6, k + 1)[0] - base).max()) for k in range(4))
    assert 0.0 < moved < 1.0
    print(f"standing humanoid, {nc} contacts: qd moves {moved:.2e} under 1e-6 relative errors in A")
