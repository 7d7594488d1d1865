"""Multi-rank path on CPU (gloo, world_size 2): shard layout and the final
observation all-gather used by bench.py (RCCL on the GPU box)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, ws, port, n_global, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gym-ignition_amd", "python"))
    from mwstep.shard import gather_obs, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    b, e = shard_range(n_global, rank, ws)
    obs = torch.arange(b, e, dtype=torch.float32).repeat_interleave(4).reshape(-1, 4)
    g = gather_obs(obs, n_global=n_global)
    g2 = gather_obs(obs)  # slab sizes gathered first
    assert torch.equal(g, g2)
    q.put((rank, b, e, g.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,n", [(2, 10), (3, 1024), (2, 7)])
def test_gather_obs_world_order(ws, n):
    """Equal and unequal slabs (1024 worlds over 3 ranks: 342 / 341 / 341)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, n, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res.sort()
    from mwstep.shard import shard_range
    assert [(b, e) for _, b, e, _ in res] == [shard_range(n, r, ws) for r in range(ws)]
    expect = [[float(w)] * 4 for w in range(n)]
    for _, _, _, g in res:
        assert g == expect


def _env_worker(rank, ws, port, n_global, T, q):
    import sys
    import numpy as np
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(here, "gym-ignition_amd", "python"))
    sys.path.insert(0, os.path.join(here, "oracle"))
    import pyoracle
    from mwstep import get_model_file
    from mwstep.shard import gather_obs, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    b, e = shard_range(n_global, rank, ws)
    task = pyoracle.make_task(pyoracle.TASK_CARTPOLE_DISCRETE, seed=42, max_episode_steps=40)
    task.world0 = b  # this rank's Philox streams: the global world indices
    env = pyoracle.VecEnv(pyoracle.load_urdf(get_model_file("cartpole")), task, e - b)
    env.reset()
    acts = np.random.default_rng(7).integers(0, 2, size=(T, n_global)).astype(np.int32)
    for t in range(T):
        obs, _, _, _ = env.step(acts[t, b:e])
    g = gather_obs(torch.from_numpy(obs))
    q.put((rank, g.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,n", [(2, 64), (3, 50)])
def test_gather_real_env_slabs(ws, n):
    """The gathered observations of a sharded batched env (each rank steps
    its block of worlds, Philox resets keyed by the global world index, 100
    steps with TimeLimit resets every 40) equal the observations of one env
    over all worlds, bit for bit -- the property bench.py's final all-gather
    relies on."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle
    from mwstep import get_model_file
    T = 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_env_worker, args=(r, ws, port, n, T, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    task = pyoracle.make_task(pyoracle.TASK_CARTPOLE_DISCRETE, seed=42, max_episode_steps=40)
    env = pyoracle.VecEnv(pyoracle.load_urdf(get_model_file("cartpole")), task, n)
    env.reset()
    acts = np.random.default_rng(7).integers(0, 2, size=(T, n)).astype(np.int32)
    for t in range(T):
        ref, _, _, _ = env.step(acts[t])
    for _, g in res:
        assert g.shape == ref.shape and np.array_equal(g, ref)


@pytest.mark.parametrize("n,ws", [(4096, 8), (1024, 3), (5, 8)])
def test_shard_range_partitions(n, ws):
    import sys
    from mwstep.shard import shard_range
    spans = [shard_range(n, r, ws) for r in range(ws)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[i][1] == spans[i + 1][0] for i in range(ws - 1))
    assert max(e - b for b, e in spans) - min(e - b for b, e in spans) <= 1
