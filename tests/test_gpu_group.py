"""The one-world-per-16-lane-row Panda env kernel (group_kernel.hip: base-frame
CRBA + RNEA + row Cholesky, DPP exchanges) against the one-world-per-lane
kernel (kernels.hip: vecenv_pid_step_kernel) and against the fp64 oracle.

Both kernels restate the same DART step (ABA with implicit damping == the
joint-space solve with M + dt D; limit rows by PGS over M^-1 columns), so
their observations agree to float32 rounding carried by the PID feedback.
World counts that are not a multiple of 4 exercise the padding rows of the
last wave (they compute a copy of the last world and store nothing)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _targets(q0, k):
    tgt = q0.clone()
    tgt[:, 0] += 0.9 * 2.8973 * math.sin(2 * math.pi * 0.33 * k * 1e-3)
    tgt[:, 5] += 0.9 * 1.885 * math.sin(2 * math.pi * 0.33 * k * 1e-3)
    return tgt


@pytest.mark.parametrize("W", [1, 6, 257])
def test_group_matches_lane_kernel(require_gpu, monkeypatch, W):
    from mwstep.vecenv import VecEnv
    H = 300
    monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "group")
    a = VecEnv("PandaPositionTracking", n_worlds=W, seed=11, max_episode_steps=120)
    monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "lane")
    b = VecEnv("PandaPositionTracking", n_worlds=W, seed=11, max_episode_steps=120)
    qa = a.reset()[:, :9].clone()
    qb = b.reset()[:, :9].clone()
    assert float((qa - qb).abs().max()) == 0.0
    worst = worst_r = 0.0
    for k in range(H):
        tgt = _targets(qa, k)
        monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "group")
        oa, ra, da, ia = a.step(tgt)
        monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "lane")
        ob, rb, db, ib = b.step(tgt)
        # TimeLimit resets at step 120 and 240: same done flags, same reset states
        assert bool((da == db).all())
        worst = max(worst, float((oa - ob).abs().max()))
        worst_r = max(worst_r, float(((ra - rb).abs() / (1 + rb.abs())).max()))
        if bool(da.any()):
            assert float((ia["terminal_obs"] - ib["terminal_obs"]).abs().max()) <= 1e-4
    print(f"group vs lane kernel, W={W}, H={H}: max|obs diff| {worst:.2e}, reward rel {worst_r:.2e}")
    assert worst <= 1e-4 and worst_r <= 1e-4
    a.close()
    b.close()


def test_group_one_step_vs_oracle(require_gpu, oracle, panda_file, monkeypatch):
    """Teacher-forced single steps from random states (about a fifth of the
    joints 2 mrad beyond a limit, so limit rows are active) against the
    oracle's ScenarioWorld with a fresh JointController: the batched env's
    q within 1e-5, qd within the north star's 1e-4."""
    import torch
    from mwstep.vecenv import VecEnv
    from test_gpu_panda import GAINS
    monkeypatch.setenv("MWSTEP_PANDA_KERNEL", "group")
    W = 64
    rng = np.random.default_rng(5)
    cm = oracle.load_urdf(panda_file)
    for i in range(cm.n):
        cm.model.lower[i] = float(np.float32(cm.model.lower[i]))
        cm.model.upper[i] = float(np.float32(cm.model.upper[i]))
    lo = np.array([cm.model.lower[i] for i in range(cm.n)])
    hi = np.array([cm.model.upper[i] for i in range(cm.n)])
    env = VecEnv("PandaPositionTracking", n_worlds=W, seed=2, max_episode_steps=10_000)
    worst_q = worst_qd = 0.0
    for _ in range(4):
        env.reset()   # PID state, low words of q and counters back to zero
        q = rng.uniform(lo, hi, size=(W, cm.n))
        at = rng.uniform(size=q.shape) < 0.2
        q[at] = np.where(rng.uniform(size=q.shape) < 0.5, lo - 2e-3, hi + 2e-3)[at]
        qd = rng.uniform(-0.5, 0.5, size=q.shape)
        q, qd = q.astype(np.float32), qd.astype(np.float32)
        tgt = np.clip(q + rng.uniform(-0.05, 0.05, size=q.shape), lo, hi).astype(np.float32)
        env.set_state(torch.from_numpy(q.T.copy()), torch.from_numpy(qd.T.copy()))
        o = env.step(torch.from_numpy(tgt).cuda())[0].cpu().numpy()
        for w in range(W):
            ow = oracle.ScenarioWorld(cm, 1e-3, 1, 20)
            ow.q, ow.qd = q[w].astype(float), qd[w].astype(float)
            ow.period_ns = 1_000_000
            for d, name in enumerate(cm.joint_names):
                ow.set_pid(d, *GAINS[name])
                ow.set_mode(d, oracle.POSITION)
            ow.ptgt[:] = tgt[w]
            ow.run()
            worst_q = max(worst_q, float(np.abs(o[w, :9] - ow.q).max()))
            worst_qd = max(worst_qd, float(np.abs(o[w, 9:] - ow.qd).max()))
    print(f"group kernel one-step vs oracle: max|dq| {worst_q:.2e}, max|dqd| {worst_qd:.2e}")
    assert worst_q <= 1e-5 and worst_qd <= 1e-4
    env.close()
