"""the exact boxed LCP converges on the bench's contact
workloads.  Runs bench.py's `contacts_floating` leg (4,096 cubes dropped from
random poses, 1,300 steps) and `scene_multi_model` leg (4,096 worlds of the
reference's three-cube contact scene, tests/test_scenario/test_contacts.py:
125-236, 600 steps) exactly as the bench does and asserts that no world-step
ran out of its linear-solve budget or hit the fp32 floor unconverged
(wave_lcp.hpp wave_boxqp; before round 5's frozen-row rule the legs counted
507 and 2,715 such world-steps, profiles/r05q)."""
import os
import sys
import types

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


@pytest.fixture(scope="module")
def bench_mod(require_gpu):
    sys.path.insert(0, ROOT)
    import bench
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bench.hip_runtime()
    args = types.SimpleNamespace(seed=42, groups=1, graph_chunk=100, no_cpu_baseline=True, cpu_leg_seconds=0.0)
    return bench, args, dev, torch


@pytest.mark.gpu
def test_contacts_leg_converges(bench_mod):
    bench, args, dev, torch = bench_mod
    out = bench.contact_leg(args, dev, torch)
    print(f"contacts_floating: {out['ms_per_step']} ms/step, unconverged {out['lcp_unconverged_world_steps']}")
    assert out["lcp_unconverged_world_steps"] == 0


@pytest.mark.gpu
def test_scene_leg_converges(bench_mod):
    bench, args, dev, torch = bench_mod
    out = bench.scene_leg(args, dev, torch)
    print(f"scene_multi_model: {out['ms_per_step']} ms/step, unconverged {out['lcp_unconverged_world_steps']}, "
          f"dropped rows {out['dropped_rows']}, cube3 support {out['cube3_support_N_world0']} N")
    assert out["dropped_rows"] == 0
    assert out["lcp_unconverged_world_steps"] == 0


@pytest.mark.gpu
def test_humanoid_leg_converges(bench_mod):
    """config 5's bench leg (512 humanoids standing, exact LCP): before round
    5's residual-scaled stall test 8 world-steps stopped at the fp32 floor on a
    joint-limit row."""
    bench, args, dev, torch = bench_mod
    out = bench.humanoid_leg(args, dev, torch)
    print(f"humanoid_c5: {out['ms_per_step']} ms/step, unconverged {out['lcp_unconverged_world_steps']}")
    assert out["constraint_overflow"] == 0
    assert out["lcp_unconverged_world_steps"] == 0
