"""The oracle's C rollouts used by bench.py's CPU baselines of BASELINE
configs 4 and 5 (or_pid_rollout, or_float_pid_rollout): they equal the
step-by-step Python composition of the same oracle calls, and they are
thread-safe (the oracle's scratch buffers are thread-local), so the baseline
may run one world set per host core."""

import threading

import numpy as np
import pytest


def _panda(oracle):
    from mwstep import get_model_file
    return oracle.load_urdf(get_model_file("panda"))


def test_pid_rollout_equals_python_loop(oracle):
    cm = _panda(oracle)
    n, W, T = cm.n, 3, 40
    rng = np.random.default_rng(0)
    lo, hi = np.array(cm.model.lower[:n]), np.array(cm.model.upper[:n])
    q0 = (lo + hi) / 2 + rng.uniform(-0.1, 0.1, (W, n)) * (hi - lo) / 2
    amp = np.zeros(n)
    amp[0], amp[5] = 0.5, 0.3
    gains = [oracle.pid_gains(100.0, 1.0, 5.0, cmdmax=80.0, cmdmin=-80.0) for _ in range(n)]
    q, qd = q0.copy(), np.zeros((W, n))
    oracle.pid_rollout(cm, q, qd, q0, amp, 0.33, gains, T, pgs_iters=20)
    mode = np.full(n, oracle.FORCE, np.int32)
    for w in range(W):
        pq, pqd = q0[w].copy(), np.zeros(n)
        st = [oracle.OrPidState() for _ in range(n)]
        for t in range(T):
            s = np.sin(2 * np.pi * 0.33 * (t + 1) * 1e-3)
            tau = np.array([oracle.pid_update(gains[i], st[i], pq[i] - (q0[w, i] + amp[i] * s), 1e-3)
                            for i in range(n)])
            pq, pqd, *_ = oracle.step(cm, 1e-3, pq, pqd, mode, tau, 20)
        assert np.abs(pq - q[w]).max() <= 1e-12 and np.abs(pqd - qd[w]).max() <= 1e-12


def test_float_rollout_threads_match_sequential(oracle):
    from mwstep import get_model_file
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    cm = oracle.load_urdf(get_model_file("icub"), pose_xyz=ICUB_POSE[:3], pose_wxyz=ICUB_POSE[3:])
    n = cm.n
    gains = [oracle.pid_gains(p, 0.0, d, cmdmax=80.0, cmdmin=-80.0) for p, d in icub_pid_gains(cm.joint_names)]
    post = np.array(icub_posture(cm.joint_names))
    rng = np.random.default_rng(1)
    starts = [post + rng.uniform(-0.05, 0.05, n) for _ in range(4)]

    def world(q0):
        fw = oracle.FloatWorld(cm, pgs_iters=oracle.PGS_CONVERGED)
        fw.set_joints(q0, np.zeros(n))
        return fw

    seq = []
    for q0 in starts:
        fw = world(q0)
        oracle.float_pid_rollout(fw, post, gains, 60)
        seq.append((fw.q, fw.p))
    par = [world(q0) for q0 in starts]
    th = [threading.Thread(target=oracle.float_pid_rollout, args=(fw, post, gains, 60)) for fw in par]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for (q, p), fw in zip(seq, par):
        assert np.array_equal(q, fw.q) and np.array_equal(p, fw.p)
    # the humanoid lands on its feet and stays up
    assert par[0].p[2] == pytest.approx(0.565, abs=0.02)
