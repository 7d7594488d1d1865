"""Per-world physics randomisation, restating the
reference's CartPole randomizer: every reset draws new link masses
m + max(U(-0.2, 0.2), 0) -- SDFRandomizer.sample clips the additive SAMPLE at 0
when force_positive is set (python/gym_ignition/randomizers/model/sdf.py:294-295,
cartpole.py:100-135) -- and a new gravity (0, 0, N(-9.8, 0.2))
(randomizers/cartpole.py:51-56).

CPU: the oracle's sampler against the distributions it restates and against a
numpy restatement from the raw Philox4x32-10 stream.  GPU: the batched env's
per-world physics and trajectories against the randomised oracle env.
"""

import math

import numpy as np
import pytest


def test_sampler_distributions(oracle, cartpole_file):
    cm = oracle.load_urdf(cartpole_file)
    t = oracle.make_task(0, seed=11, randomize=3)
    n = 20000
    dm = np.zeros((n, cm.n))
    gz = np.zeros(n)
    for w in range(n):
        m, g = oracle.sample_physics(cm, t, w, w % 7)
        dm[w] = m - np.array([cm.model.mass[i] for i in range(cm.n)])
        gz[w] = g
    assert dm.min() == 0.0 and dm.max() <= 0.2
    zero = np.mean(dm == 0.0)
    assert abs(zero - 0.5) < 0.02                       # half of U(-0.2, 0.2) clips to 0
    assert abs(dm[dm > 0].mean() - 0.1) < 0.005         # the rest is U(0, 0.2)
    assert abs(gz.mean() + 9.8) < 4 * 0.2 / math.sqrt(n)
    assert abs(gz.std() - 0.2) < 0.01
    # no randomisation: the nominal model
    m0, g0 = oracle.sample_physics(cm, oracle.make_task(0), 3, 0)
    assert np.all(m0 == [cm.model.mass[i] for i in range(cm.n)]) and g0 == 0.0


def test_sampler_matches_numpy_restatement(oracle, cartpole_file):
    cm = oracle.load_urdf(cartpole_file)
    seed = 0x1234_5678_9ABC
    t = oracle.make_task(1, seed=seed, randomize=3, mass_range=(-0.3, 0.25), gravity_normal=(-9.81, 0.5))
    key = [seed & 0xFFFFFFFF, seed >> 32]
    for w, ep in [(0, 0), (5, 3), (1000, 17)]:
        m, g = oracle.sample_physics(cm, t, w, ep)
        r = oracle.philox_raw([w, ep, 1, 0], key)
        u = (r >> 8).astype(np.float64) / 16777216.0
        exp_m = np.array([cm.model.mass[i] for i in range(cm.n)]) + np.maximum(-0.3 + 0.55 * u[:cm.n], 0.0)
        np.testing.assert_allclose(m, exp_m, rtol=0, atol=1e-15)
        r8 = oracle.philox_raw([w, ep, 8, 0], key)
        u1 = ((int(r8[0]) >> 8) + 1) / 16777216.0
        u2 = (int(r8[1]) >> 8) / 16777216.0
        assert g == pytest.approx(-9.81 + 0.5 * math.sqrt(-2 * math.log(u1)) * math.cos(2 * math.pi * u2), abs=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("task,kind,model", [("CartPoleContinuousBalancing", 1, "cartpole"),
                                             ("PendulumSwingUp", 3, "pendulum")])
def test_randomised_env_vs_oracle(require_gpu, oracle, task, kind, model):
    import torch
    from mwstep import get_model_file
    from mwstep.vecenv import VecEnv
    W, H, T_LIM = 512, 250, 100
    gpu = VecEnv(task, n_worlds=W, seed=21, randomize=True, max_episode_steps=T_LIM)
    cm = oracle.load_urdf(get_model_file(model))
    ref = oracle.VecEnv(cm, oracle.make_task(kind, seed=21, randomize=3, max_episode_steps=T_LIM), W)
    og = gpu.reset().cpu().numpy()
    orf = ref.reset()
    assert np.abs(og - orf).max() <= 1e-6
    # per-world physics of episode 0
    m, gz = (x.cpu().numpy() for x in gpu.physics())
    for w in range(0, W, 37):
        mr, gr = oracle.sample_physics(cm, ref.task, w, 0)
        assert np.abs(m[:, w] - mr).max() <= 1e-6 and abs(gz[w] - gr) <= 2e-5
    assert np.unique(gz).size > W // 2                   # every world has its own gravity
    rng = np.random.default_rng(4)
    a = 50.0
    alive = np.ones(W, dtype=bool)
    worst = 0.0
    for t in range(H):
        act = rng.uniform(-a, a, W).astype(np.float32)
        o, _, d, _ = gpu.step(torch.from_numpy(act).cuda())
        o, d = o.cpu().numpy(), d.cpu().numpy().astype(bool)
        orf, _, drf, _ = ref.step(act.astype(np.float64))
        alive &= (d == drf)
        worst = max(worst, float(np.abs(o[alive] - orf[alive]).max()))
    print(f"{task} randomised: free-running max|obs err| {worst:.2e}, alive {alive.mean():.3f}")
    assert worst <= 1e-3 and alive.mean() >= 0.99
    # after the TimeLimit resets the worlds carry their episode-2 physics
    ep, _ = gpu.counters()
    m, gz = (x.cpu().numpy() for x in gpu.physics())
    for w in range(0, W, 41):
        mr, gr = oracle.sample_physics(cm, ref.task, w, int(ep[w]))
        assert np.abs(m[:, w] - mr).max() <= 1e-6 and abs(gz[w] - gr) <= 2e-5
    gpu.close()


@pytest.mark.gpu
def test_randomisation_changes_dynamics(require_gpu):
    """Same seed, same actions: the randomised env diverges from the nominal one
    and two randomised envs with different seeds diverge from each other."""
    import torch
    from mwstep.vecenv import VecEnv
    W = 256
    envs = [VecEnv("CartPoleContinuousBalancing", n_worlds=W, seed=s, randomize=r)
            for s, r in [(1, False), (1, True), (2, True)]]
    for e in envs:
        e.reset()
    a = torch.full((W,), 10.0, device="cuda")
    for _ in range(50):
        outs = [e.step(a)[0].clone() for e in envs]
    assert not torch.equal(outs[0], outs[1])
    for e in envs:
        e.close()
