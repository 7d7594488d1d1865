"""GPU parity of the batched env kernel against the fp64 oracle.

Tolerances (stated per SURVEY.md §8d; fp32 kernel vs fp64 oracle):
  * one-step, teacher-forced observation error      <= 1e-4 (north-star bound)
  * free-running observation error over H = 100     <= 1e-3 (chaotic systems;
    the growth curve is printed)
  * reset observations (Philox-sampled)             <= 1e-6
  * reward: same tolerance as the observation it is computed from (x 10)
Done flags must agree except within float32 rounding of a threshold: at most
0.2 % of the (world, step) pairs may differ, and such worlds are excluded
from then on (their episode counters diverge).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TASKS = [
    ("CartPoleDiscreteBalancing", 0, "cartpole"),
    ("CartPoleContinuousBalancing", 1, "cartpole"),
    ("CartPoleContinuousSwingup", 2, "cartpole"),
    ("PendulumSwingUp", 3, "pendulum"),
]
ACTION_RANGE = {1: 50.0, 2: 200.0, 3: 50.0}


def _actions(kind, T, W, seed):
    rng = np.random.default_rng(seed)
    if kind == 0:
        return rng.integers(0, 2, size=(T, W)).astype(np.int32)
    a = ACTION_RANGE[kind]
    return rng.uniform(-a, a, size=(T, W)).astype(np.float32)


def _pair(oracle, task, kind, model, W, seed=42, physics_rate=1000.0, max_steps=5000):
    import torch
    from mwstep.vecenv import VecEnv
    from mwstep.models import get_model_file
    gpu = VecEnv(task, n_worlds=W, seed=seed, physics_rate=physics_rate, max_episode_steps=max_steps)
    cm = oracle.load_urdf(get_model_file(model))
    spr = int(physics_rate / 1000.0)
    ref = oracle.VecEnv(cm, oracle.make_task(kind, dt=1.0 / physics_rate, steps_per_run=spr,
                                             max_episode_steps=max_steps, seed=seed), W)
    return torch, gpu, ref


@pytest.mark.parametrize("task,kind,model", TASKS)
def test_reset_obs(require_gpu, oracle, task, kind, model):
    torch, gpu, ref = _pair(oracle, task, kind, model, W=1000)
    og = gpu.reset().cpu().numpy()
    orf = ref.reset()
    assert np.abs(og - orf).max() <= 1e-6
    gpu.close()


@pytest.mark.parametrize("task,kind,model", TASKS)
def test_one_step_teacher_forced(require_gpu, oracle, task, kind, model):
    W, T = 512, 300
    torch, gpu, ref = _pair(oracle, task, kind, model, W)
    gpu.reset()
    ref.reset()
    acts = _actions(kind, T, W, seed=7)
    alive = np.ones(W, dtype=bool)
    worst_obs = worst_rew = 0.0
    mism = 0
    n = ref.cm.n
    for t in range(T):
        # teacher forcing: the GPU starts every step from the oracle state
        gpu.set_state(torch.from_numpy(ref.q.reshape(n, W)), torch.from_numpy(ref.qd.reshape(n, W)))
        a = acts[t]
        og, rg, dg, info = gpu.step(torch.from_numpy(a).cuda())
        og, rg, dg = og.cpu().numpy(), rg.cpu().numpy(), dg.cpu().numpy().astype(bool)
        orf, rrf, drf, _ = ref.step(a.astype(np.float64) if kind else a)
        same = (dg == drf)
        mism += int(np.sum(~same & alive))
        alive &= same
        m = alive & ~drf
        if m.any():
            worst_obs = max(worst_obs, float(np.abs(og[m] - orf[m]).max()))
            worst_rew = max(worst_rew, float(np.abs(rg[m] - rrf[m]).max()))
    print(f"{task}: one-step max|obs err| {worst_obs:.3e}, max|reward err| {worst_rew:.3e}, "
          f"done mismatches {mism}")
    assert worst_obs <= 1e-4
    assert worst_rew <= 1e-3
    assert mism <= 0.002 * W * T
    gpu.close()


@pytest.mark.parametrize("task,kind,model", TASKS)
def test_free_running_horizon(require_gpu, oracle, task, kind, model):
    W, H = 512, 100
    torch, gpu, ref = _pair(oracle, task, kind, model, W)
    gpu.reset()
    ref.reset()
    acts = _actions(kind, H, W, seed=11)
    alive = np.ones(W, dtype=bool)
    curve = []
    for t in range(H):
        og, rg, dg, _ = gpu.step(torch.from_numpy(acts[t]).cuda())
        og, dg = og.cpu().numpy(), dg.cpu().numpy().astype(bool)
        orf, rrf, drf, _ = ref.step(acts[t].astype(np.float64) if kind else acts[t])
        alive &= (dg == drf)
        curve.append(float(np.abs(og[alive] - orf[alive]).max()) if alive.any() else 0.0)
    print(f"{task}: free-running max|obs err| at t=1,10,50,100: "
          f"{curve[0]:.2e} {curve[9]:.2e} {curve[49]:.2e} {curve[-1]:.2e}")
    assert max(curve) <= 1e-3
    assert alive.mean() >= 0.99
    gpu.close()


def test_rollout_kernel_equals_stepping(require_gpu, oracle):
    W, T = 700, 64
    torch, a, _ = _pair(oracle, "CartPoleDiscreteBalancing", 0, "cartpole", W, seed=5)
    _, b, _ = _pair(oracle, "CartPoleDiscreteBalancing", 0, "cartpole", W, seed=5)
    a.reset()
    b.reset()
    acts = torch.from_numpy(_actions(0, T, W, seed=3)).cuda()
    obs_r, rew_r, done_r, _ = a.rollout(acts)
    for t in range(T):
        o, r, d, _ = b.step(acts[t].contiguous())
        assert torch.equal(o, obs_r[t]) and torch.equal(r, rew_r[t]) and torch.equal(d, done_r[t])
    a.close()
    b.close()


def test_steps_per_run_force_consumed_by_first_substep(require_gpu, oracle):
    """physics_rate = 4 x agent_rate: the force acts on the first substep only
    (Physics.cpp:2250-2254; tests/.python/test_joint_force.py:48-81)."""
    W, T = 256, 100
    torch, gpu, ref = _pair(oracle, "CartPoleContinuousBalancing", 1, "cartpole", W,
                            physics_rate=4000.0)
    gpu.reset()
    ref.reset()
    acts = _actions(1, T, W, seed=2)
    worst = 0.0
    alive = np.ones(W, dtype=bool)
    for t in range(T):
        og, _, dg, _ = gpu.step(torch.from_numpy(acts[t]).cuda())
        orf, _, drf, _ = ref.step(acts[t].astype(np.float64))
        alive &= dg.cpu().numpy().astype(bool) == drf
        worst = max(worst, float(np.abs(og.cpu().numpy()[alive] - orf[alive]).max()))
    assert worst <= 1e-3
    gpu.close()


def test_c2_config_properties(require_gpu):
    """4096 CartPole worlds (BASELINE config 2): determinism, finiteness,
    auto-reset draws from the reset distribution, TimeLimit respected."""
    import torch
    from mwstep.vecenv import VecEnv
    W, T = 4096, 400
    envs = [VecEnv("CartPoleDiscreteBalancing", n_worlds=W, seed=42, max_episode_steps=100)
            for _ in range(2)]
    for e in envs:
        e.reset()
    g = torch.Generator(device="cuda").manual_seed(43)
    outs = [[], []]
    for t in range(T):
        a = torch.randint(0, 2, (W,), generator=g, device="cuda", dtype=torch.int32)
        for i, e in enumerate(envs):
            o, r, d, info = e.step(a)
            outs[i].append((o.clone(), r.clone(), d.clone(), info["terminal_obs"].clone()))
    for (o1, r1, d1, _), (o2, r2, d2, _) in zip(*outs):
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2)
    obs = torch.stack([x[0] for x in outs[0]])
    done = torch.stack([x[2] for x in outs[0]]).bool()
    assert torch.isfinite(obs).all()
    # where done, obs is the first observation of the next episode: |.| <= 0.05
    assert (obs[done].abs() <= 0.05 + 1e-6).all()
    ep, st = envs[0].counters()
    assert int(st.max()) < 100          # TimeLimit(100) always fires
    assert int(ep.min()) >= T // 100    # every world finished >= 4 episodes
    for e in envs:
        e.close()


@pytest.mark.parametrize("task,kind,model", [TASKS[0], TASKS[3]])
def test_baked_kernel_matches_generic(require_gpu, oracle, task, kind, model, monkeypatch):
    """The constant-folded kernel of a shipped model against the generic kernel
    on the same inputs (rounding may differ: <= 1e-5 after 200 steps)."""
    import torch
    W, T = 1024, 200
    _, a, _ = _pair(oracle, task, kind, model, W, seed=9)
    _, b, _ = _pair(oracle, task, kind, model, W, seed=9)
    assert a.sim.baked_model() in (1, 2)
    a.reset()
    b.reset()
    acts = _actions(kind, T, W, seed=4)
    worst = 0.0
    for t in range(T):
        x = torch.from_numpy(acts[t]).cuda()
        monkeypatch.delenv("MWSTEP_DISABLE_BAKED", raising=False)
        oa, _, da, _ = a.step(x)
        monkeypatch.setenv("MWSTEP_DISABLE_BAKED", "1")
        ob, _, db, _ = b.step(x)
        same = (da == db)
        worst = max(worst, float((oa[same] - ob[same]).abs().max()))
    monkeypatch.delenv("MWSTEP_DISABLE_BAKED", raising=False)
    assert worst <= 1e-5
    a.close()
    b.close()


def test_pendulum_2048_worlds(require_gpu, oracle):
    """BASELINE config 3 at its size: 2048 PendulumSwingUp worlds (continuous
    torque U(-50, 50)).  One-step teacher-forced observation error <= 1e-4 over
    50 steps, free-running error <= 1e-3 over 100 steps, reset observations
    <= 1e-6, done flags equal."""
    W = 2048
    torch, gpu, ref = _pair(oracle, "PendulumSwingUp", 3, "pendulum", W)
    og = gpu.reset().cpu().numpy()
    assert np.abs(og - ref.reset()).max() <= 1e-6
    acts = _actions(3, 150, W, seed=11)
    n = ref.cm.n
    worst = 0.0
    for t in range(50):
        gpu.set_state(torch.from_numpy(ref.q.reshape(n, W)), torch.from_numpy(ref.qd.reshape(n, W)))
        o, _, d, _ = gpu.step(torch.from_numpy(acts[t]).cuda())
        orf, _, drf, _ = ref.step(acts[t].astype(np.float64))
        assert np.array_equal(d.cpu().numpy().astype(bool), drf)
        worst = max(worst, float(np.abs(o.cpu().numpy() - orf).max()))
    free = 0.0
    for t in range(50, 150):
        o, _, d, _ = gpu.step(torch.from_numpy(acts[t]).cuda())
        orf, _, drf, _ = ref.step(acts[t].astype(np.float64))
        m = ~(d.cpu().numpy().astype(bool) | drf)
        free = max(free, float(np.abs(o.cpu().numpy()[m] - orf[m]).max()))
    print(f"pendulum x{W}: one-step {worst:.2e}, free-running 100 steps {free:.2e}")
    assert worst <= 1e-4 and free <= 1e-3
    gpu.close()
