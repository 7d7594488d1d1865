"""The bench's multi-rank path as the driver launches it (torch.distributed.run,
one process per rank), rehearsed on the one-GPU box: two ranks share the
device, gloo carries the collectives (MWSTEP_DIST_BACKEND=gloo; RCCL refuses
two ranks on one device).  Checks the headline's world sharding and final
observation all-gather, and the strong splits of BASELINE configs 4 (1024
Panda worlds) and 5 (512 humanoids) over the ranks."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bench(n_ranks, worlds):
    env = dict(os.environ, MWSTEP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n_ranks), "--steps", "20", "--warmup", "5",
            "--worlds", str(worlds), "--no-rollout", "--no-sweep", "--no-rand-leg", "--no-pendulum",
            "--no-runtime-leg", "--no-scene-leg", "--no-cpu-baseline", "--no-free-legs", "--no-pgs-leg",
            "--no-share-proj"]
    if n_ranks > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n_ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints one JSON line
    return json.loads(lines[0])


def test_two_rank_bench(require_gpu):
    """Two ranks of 1024 CartPole worlds each vs one rank of 2048: the
    gathered final observations (global world order) are bit-identical to
    the one-rank run's, and so are the final states of the strong splits of
    configs 4 (1024 Panda worlds) and 5 (512 humanoids) gathered over the
    ranks (per-world actions, Philox resets and initial states are keyed by
    the global world index)."""
    out = _bench(2, 1024)
    one = _bench(1, 2048)
    print(json.dumps({k: out[k] for k in ("value", "ms_per_step", "n_gpus")}),
          json.dumps({k: out[k]["worlds_per_gpu"] for k in ("panda_c4", "humanoid_c5")}))
    assert out["n_gpus"] == 2 and out["config"]["global_worlds"] == 2048
    assert out["value"] > 0 and out["scaling"] == "weak"
    assert out["gathered_obs_shape"] == [2048, 4]
    p, h = out["panda_c4"], out["humanoid_c5"]
    assert p["scaling"] == "strong" and p["worlds_per_gpu"] == 512 and p["value"] > 0
    assert h["scaling"] == "strong" and h["worlds_per_gpu"] == 256 and h["value"] > 0
    assert h["constraint_overflow"] == 0
    assert one["n_gpus"] == 1 and one["config"]["global_worlds"] == 2048
    assert out["final_obs_sha256"] == one["final_obs_sha256"]
    assert p["final_state_sha256"] == one["panda_c4"]["final_state_sha256"]
    assert h["final_state_sha256"] == one["humanoid_c5"]["final_state_sha256"]
