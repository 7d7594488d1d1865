"""The driver's exact bench command (`python bench.py --gpus 1 --steps 20
--warmup 5`) in a fresh process: one JSON line with the contract's fields,
`roofline`, `cpu_baseline` and the parity figure (the r01 bench
crashed on exactly this command because a leg was sized from --steps)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_driver_bench_command(require_gpu):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5"],
                       cwd=ROOT, capture_output=True, text=True, timeout=560, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["steps"] == 20 and out["warmup"] == 5 and out["n_gpus"] == 1
    assert out["value"] > 1e6
    assert "configs[1]" in out["config"]["workload"]
    rl = out["roofline"]
    assert rl["bound"] == "hbm" and 0 < rl["frac"] < 1 and rl["peak"] == 8000.0
    cpu = out["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0 and "dart_probe" in cpu
    assert out["obs_max_abs_err_vs_oracle"]["value"] <= 1e-4
    assert out["rollout_fused"]["steps_per_launch"] == 1000
    assert out["panda_c4"]["worlds_per_gpu"] == 1024
    assert out["humanoid_c5"]["worlds_per_gpu"] == 512
    # every BASELINE config leg carries its roofline and a CPU baseline
    pend = out["pendulum_c3"]
    assert "configs[2]" in pend["workload"] and pend["value"] > 1e6 and pend["kernel_us_per_launch"] > 0
    for leg in ("pendulum_c3", "panda_c4", "humanoid_c5"):
        rl_, cb = out[leg]["roofline"], out[leg]["cpu_baseline"]
        assert rl_["peak"] > 0 and rl_["bound"] in ("hbm", "valu-issue"), leg
        assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0, leg
    assert out["pendulum_c3"]["roofline"]["frac"] > 0 and out["panda_c4"]["roofline"]["frac"] > 0
    # PMC traffic of the config-3 and config-4 kernels (committed FETCH / WRITE passes)
    assert out["pendulum_c3"]["roofline"]["traffic"] and out["panda_c4"]["roofline"]["traffic"]
    # the headline roofline is timed on the driver clock (one launch per step)
    assert rl["time_us_per_launch"] == pytest.approx(out["ms_per_step"] * 1e3, rel=1e-3)
    h = out["humanoid_c5"]
    assert h["constraint_overflow"] == 0 and h["lcp_unconverged_world_steps"] is not None
    assert "boxed LCP solved as DART does" in h["workload"] and "PGS" in out["humanoid_c5_pgs_only"]["workload"]
    # configs 4 / 5: the 8-GPU strong split projected from the 8 rank shares timed alone
    for leg, wg in (("panda_c4", 1024), ("humanoid_c5", 512)):
        ps = out[leg]["projected_split"]
        assert ps["n_gpus"] == 8 and ps["worlds_per_gpu"] == wg // 8 and len(ps["share_ms_per_step"]) == 8, leg
        assert ps["ms_per_step"] == max(ps["share_ms_per_step"]) and ps["speedup_vs_1gpu"] > 0, leg
