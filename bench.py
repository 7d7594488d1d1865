"""Benchmark: env.steps/s of batched CartPole worlds on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--worlds 4096]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

One "step" = one gym step of EVERY world of a rank: the action is applied, the
physics runs (ABA + semi-implicit Euler, dt = 1 ms), and observation, reward,
done, TimeLimit and auto-reset are computed -- all inside one HIP kernel
launch per step (vecenv_step_kernel).  The K timed steps are replayed from
HIP graphs of `--graph-chunk` launches each; per-step actions are written into
the graph's action buffer before each replay (as a policy would), so the path
is the closed-loop one.  Worlds shard across ranks with no data-path
collective (weak scaling); the final observation tensor is all-gathered once
over RCCL, as the north star asks.

Printed JSON (rank 0): value = total env.steps/s over all ranks; roofline of
the dominant kernel from per-launch HIP-event timing on its own stream;
cpu_baseline = the fp64 C oracle on a bounded sample (rank 0, N = 1 only).
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))

METRIC = "env·steps/sec (whole node) at N parallel worlds; obs max-abs-err vs DART"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def algorithmic_bytes_per_env_step(n_dofs: int, n_obs: int) -> int:
    """Compulsory HBM bytes of one env step of one world:
    read q, qd (4 B each per dof), action (4 B), steps + episode counters (8 B);
    write q, qd, obs (4 B per element), reward (4 B), done (1 B), steps (4 B)."""
    reads = 4 * 2 * n_dofs + 4 + 8
    writes = 4 * 2 * n_dofs + 4 * n_obs + 4 + 1 + 4
    return reads + writes


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--worlds", type=int, default=4096, help="worlds per GPU")
    p.add_argument("--task", default="CartPoleDiscreteBalancing")
    p.add_argument("--graph-chunk", type=int, default=100)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    p.add_argument("--cpu-leg-seconds", type=float, default=4.0, help="CPU baseline budget of the other configs")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-rollout", action="store_true")
    p.add_argument("--no-sweep", action="store_true")
    p.add_argument("--no-panda", action="store_true", help="skip the config-4 Panda leg")
    p.add_argument("--no-rand-leg", action="store_true", help="skip the randomised-physics leg")
    p.add_argument("--no-pendulum", action="store_true", help="skip the config-3 Pendulum leg")
    p.add_argument("--no-contact-leg", action="store_true", help="skip the floating-body contact leg")
    p.add_argument("--no-runtime-leg", action="store_true", help="skip the config-1 GazeboRuntime leg")
    p.add_argument("--no-scene-leg", action="store_true", help="skip the multi-model scene leg")
    p.add_argument("--no-free-legs", action="store_true",
                   help="skip the floating-cube and quadruped legs (configs 4 / 5 still run)")
    p.add_argument("--no-pgs-leg", action="store_true", help="skip the config-5 PGS-only leg")
    p.add_argument("--no-share-proj", action="store_true",
                   help="skip the projected 8-GPU strong split of configs 4 / 5 (their rank shares timed alone)")
    p.add_argument("--groups", type=int, default=1,
                   help="world groups per GPU, each on its own stream / hardware queue")
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    # one process per GPU; the modulo only matters when rehearsing several
    # ranks on fewer GPUs (the driver launches one rank per GPU)
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    if world_size > 1:
        # RCCL ("nccl") is the product path; MWSTEP_DIST_BACKEND=gloo rehearses
        # several ranks on one GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("MWSTEP_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from mwstep.vecenv import VecEnv

    W = args.worlds
    envs = make_groups(args.task, W, args.groups, dev, args.seed, rank * W)
    env = envs[0]
    K = args.steps
    # actions of the GLOBAL worlds, this rank's block sliced out: every world
    # sees the same action sequence at any rank count
    actions = make_actions(envs, args.warmup + K, dev, torch, 0, offset=rank * W, n_global=world_size * W)
    timed = time_steps(envs, actions, args.warmup, K, args.graph_chunk, dev, torch, dist, world_size,
                       gather=(world_size > 1))
    elapsed, kernel_us = timed["elapsed"], timed["kernel_us"]
    value = world_size * W * K / elapsed
    G = timed["G"]

    # per-launch time of the step kernel: HIP events recorded on the launch
    # stream around the timed graph replays (K launches), see time_steps()
    if env.action_dim:
        bpe = panda_bytes_per_env_step(env.sim.dofs)
        kname = "vecenv_pid_group_kernel<9,false,true> (one world per 16-lane row)"
    else:
        bpe = algorithmic_bytes_per_env_step(env.sim.dofs, env.obs_dim)
        kname = (f"vecenv_step_kernel<{env.sim.dofs},{env.kind},false,true,false,{env.sim.baked_model()}>"
                 + (" (model constant-folded)" if env.sim.baked_model() else ""))
    # the roofline's time is the driver-clock step time of the timed region
    # (K steps / wall time, per GPU): the figure the committed kernel trace of
    # the same command reproduces (profiles/r04a/trace_summary.json: timed
    # dispatch mean); the HIP-event launch period is reported beside it
    step_us = elapsed / K * 1e6
    achieved_gbs = bpe * W / (step_us * 1e-6) / 1e9
    event_gbs = bpe * W / (kernel_us * 1e-6) / 1e9
    traffic = pmc_traffic(args.task, W)
    floor_us = launch_floor(dev, torch) if rank == 0 else None

    # ------------------------------------------- fused open-loop rollout figure
    rollout = None
    if not args.no_rollout and not env.action_dim:
        # its own T-step action tensor: independent of --steps / --warmup
        T = 1000
        ractions = make_actions(envs, T, dev, torch, rank + 1000)[:, :env.n_worlds].contiguous()
        stream = timed["stream"]
        with torch.cuda.stream(stream):
            env.rollout(ractions)   # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.rollout(ractions)
            e1.record(stream)
        stream.synchronize()
        r_ms = e0.elapsed_time(e1)
        Wr = env.n_worlds
        assert ractions.shape[0] == T
        rollout = {"steps_per_launch": T, "worlds": Wr, "ms_per_launch": round(r_ms, 4),
                   "env_steps_per_s_per_gpu": round(Wr * T / (r_ms * 1e-3), 1),
                   "note": "open-loop (actions known ahead); not the headline value"}

    # ---------------- world-count sweep (same kernel, graph mode): where the
    # latency regime ends and the HBM / VALU bound takes over
    sweep = None
    if not args.no_sweep and world_size == 1 and not env.action_dim:
        sweep = world_sweep(args, dev, torch)

    # ---------------- BASELINE config 3: 2048 Pendulum worlds (continuous torque)
    pend = None
    if not args.no_pendulum and rank == 0 and world_size == 1 and args.task == "CartPoleDiscreteBalancing":
        penvs = make_groups("PendulumSwingUp", 2048, 1, dev, args.seed, 0)
        pacts = make_actions(penvs, args.warmup + K, dev, torch, 0)
        r = time_steps(penvs, pacts, args.warmup, K, args.graph_chunk, dev, torch, dist, 1)
        pb = algorithmic_bytes_per_env_step(1, 3)
        pend = {"workload": "PendulumSwingUp: 2048 worlds, tau ~ U(-50, 50), dt = 1 ms (BASELINE.json configs[2])",
                "value": round(2048 * K / r["elapsed"], 1), "unit": "env·steps/s",
                "ms_per_step": round(r["elapsed"] / K * 1e3, 6),
                "kernel_us_per_launch": round(r["kernel_us"], 3), "bytes_per_env_step": pb,
                "kernel": f"vecenv_step_kernel<1,3,false,false,false,{penvs[0].sim.baked_model()}>",
                "roofline": hbm_roofline(pb * 2048, r["elapsed"] / K * 1e6, pmc_traffic("PendulumSwingUp", 2048),
                                         "vecenv_step_kernel (Pendulum)", r["kernel_us"])}
        if not args.no_cpu_baseline:
            pend["cpu_baseline"] = cpu_vec_baseline("PendulumSwingUp", args.seed, args.cpu_leg_seconds)
        for e in penvs:
            e.close()

    # ---------------- the same workload with per-world physics randomisation
    # (masses + gravity resampled at every reset, randomizers/cartpole.py)
    rand = None
    if not args.no_rand_leg and rank == 0 and world_size == 1 and not env.action_dim:
        renvs = make_groups(args.task, W, 1, dev, args.seed, 0, randomize=True)
        r = time_steps(renvs, actions, args.warmup, K, args.graph_chunk, dev, torch, dist, 1)
        rand = {"value": round(W * K / r["elapsed"], 1), "unit": "env·steps/s",
                "ms_per_step": round(r["elapsed"] / K * 1e3, 6),
                "kernel_us_per_launch": round(r["kernel_us"], 3),
                "extra_bytes_per_env_step": 4 * (env.sim.dofs + 1),
                "note": "per-world masses + gravity read every step, resampled at every reset"}
        for e in renvs:
            e.close()

    # ---------------- BASELINE config 4 (1024 Panda worlds, PID position
    # tracking) measured in the same run when the headline is config 2
    # every rank takes part (strong split of the 1024 global worlds, barrier +
    # max over ranks like the headline)
    panda = None
    if not args.no_panda and args.task != "PandaPositionTracking":
        panda = panda_leg(args, dev, torch, dist, world_size, rank)
    contacts = quadruped = humanoid = humanoid_pgs = None
    if not args.no_contact_leg:
        if rank == 0 and world_size == 1 and not args.no_free_legs:
            contacts = contact_leg(args, dev, torch)
            quadruped = quadruped_leg(args, dev, torch)
        # BASELINE config 5: 512 global humanoid worlds split over the ranks
        humanoid = humanoid_leg(args, dev, torch, dist, world_size, rank)
        # the same workload on the PGS sweeps alone (the round-2 default): the exact solve's cost
        if not args.no_pgs_leg:
            humanoid_pgs = humanoid_leg(args, dev, torch, dist, world_size, rank, exact=False)
    # the 8-GPU strong split of configs 4 / 5, projected on this one GPU: every
    # rank's share run alone, one after another (the worlds are independent,
    # no data-path collective); the slowest share is the split's step time
    if world_size == 1 and not args.no_share_proj:
        if panda is not None:
            panda["projected_split"] = share_projection(
                lambda r: panda_leg(args, dev, torch, _NoDist, SHARE_N, r), panda["ms_per_step"], 1024)
        if humanoid is not None:
            humanoid["projected_split"] = share_projection(
                lambda r: humanoid_leg(args, dev, torch, _NoDist, SHARE_N, r), humanoid["ms_per_step"], 512)
    runtime = None
    if rank == 0 and world_size == 1 and not args.no_runtime_leg:
        runtime = runtime_leg(args, dev)
    scene = None
    if rank == 0 and world_size == 1 and not args.no_scene_leg:
        scene = scene_leg(args, dev, torch)

    # ------------------------------------------------------ CPU baseline (rank 0, N=1)
    cpu = None
    parity = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline and not env.action_dim:
        cpu, parity = cpu_baseline_and_parity(args, env, np, torch)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env·steps/s",
            "n_gpus": world_size,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox resets, uniform random actions, seed 42/43)",
            "config": {
                "workload": f"{args.task}: {W} worlds per GPU, dt=1ms, 1 physics step per env step "
                            + ("(BASELINE.json configs[3])" if env.action_dim else "(BASELINE.json configs[1])"),
                "task": args.task,
                "worlds_per_gpu": W,
                "global_worlds": W * world_size,
                "dt": 1e-3,
                "launch": (f"hipGraph of {G} per-step kernels" if args.groups == 1 else
                           f"{args.groups} world groups of {W // args.groups}, each on its own stream "
                           f"(hardware queue) replaying a hipGraph of {G} per-step kernels"),
                "parallelism": f"worlds sharded over {world_size} GPU(s)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "kernel": kname,
                "time_us_per_launch": round(step_us, 3),
                "timing": "driver clock: the timed region's wall time / K (one launch per step); the committed "
                          "rocprofv3 trace of the same command gives the timed dispatches' mean "
                          "(profiles/r04a/trace_summary.json)",
                "kernel_us_per_launch": round(kernel_us, 3),
                "achieved_by_launch_period": round(event_gbs, 3),
                "launch_period_timing": "HIP events on the launch stream over the K timed launches (excludes the "
                                        "host graph launch and the final synchronisation)",
                "bytes_per_env_step": bpe,
                "algorithmic_bytes_per_launch": bpe * W,
                "traffic_source": traffic["source"] if traffic else None,
                "launch_floor_us": round(floor_us, 3) if floor_us else None,
                "launch_floor_note": "per-node time of a hipGraph of 1-element kernels, same replay pattern: "
                                     "the dispatch floor of a one-kernel-per-step closed loop",
                "regime": "launch/latency-bound: the kernel sits within ~1 us of the launch floor at this "
                          "world count; 'bound' names the roofline axis, the HBM roof is reached only at "
                          "~1M worlds (world_sweep)",
            },
            "gathered_obs_shape": timed["gathered_obs_shape"],
            "final_obs_sha256": timed["final_obs_sha256"],
            "world_sweep": sweep,
            "cpu_baseline": cpu,
            "obs_max_abs_err_vs_oracle": parity,
            "rollout_fused": rollout,
            "panda_c4": panda,
            "pendulum_c3": pend,
            "randomized": rand,
            "contacts_floating": contacts,
            "quadruped_floating": quadruped,
            "humanoid_c5": humanoid,
            "humanoid_c5_pgs_only": humanoid_pgs,
            "runtime_c1": runtime,
            "scene_multi_model": scene,
        }
        print(json.dumps(out))
    for e in envs:
        e.close()
    if world_size > 1:
        dist.destroy_process_group()


SHARE_N = 8


class _NoDist:
    """torch.distributed stand-in for one rank's share run alone on one GPU:
    the legs' barriers and max-over-ranks become no-ops"""
    class ReduceOp:
        MAX = None

    @staticmethod
    def barrier():
        pass

    @staticmethod
    def all_reduce(t, op=None):
        pass


def share_projection(run_share, ms_1gpu, W_global, n=SHARE_N):
    """Time every rank's share of an n-GPU strong split on this GPU, one after
    another; the split's step time is the slowest share's (each GPU steps its
    own worlds, no collective in the step).  Reports the projected whole-job
    rate and its speedup over the measured one-GPU step."""
    shares = []
    for r in range(n):
        o = run_share(r)
        shares.append(o["ms_per_step"])
    worst = max(shares)
    return {"n_gpus": n, "worlds_per_gpu": W_global // n, "share_ms_per_step": [round(x, 6) for x in shares],
            "ms_per_step": round(worst, 6), "value": round(W_global / (worst * 1e-3), 1),
            "speedup_vs_1gpu": round(ms_1gpu / worst, 3),
            "method": f"each of the {n} rank shares timed alone on this GPU (same leg code, no collective in the "
                      "step); the split's step time is the slowest share's; projection, not an 8-GPU measurement"}


def panda_targets(q0, T, dt, torch):
    """BASELINE config 4 targets: q0 + 0.9 (range/2) sin(2 pi 0.33 t) on joints 1
    and 6 (tests/test_scenario/test_pid_controllers.py:91-99), the other joints
    hold q0.  q0 [W, 9] is each world's reset pose; returns [T, W, 9]."""
    import math
    t = torch.arange(T, device=q0.device, dtype=torch.float32) * dt
    s = torch.sin(2 * math.pi * 0.33 * t)[:, None]
    tg = q0[None].repeat(T, 1, 1)
    tg[:, :, 0] += 0.9 * (2 * 2.8973) / 2 * s
    tg[:, :, 5] += 0.9 * (3.7525 + 0.0175) / 2 * s
    return tg.contiguous()


def make_actions(envs, total, dev, torch, tag, offset=0, n_global=None):
    """[total, W] actions of the envs' worlds: columns offset .. offset + W of
    one [total, n_global] draw (seed 43 + tag), so a world's actions do not
    depend on how the worlds are split over ranks."""
    gen = torch.Generator(device=dev).manual_seed(43 + tag)
    env = envs[0]
    W = sum(e.n_worlds for e in envs)
    n_global = W if n_global is None else n_global
    if env.action_dim:
        q0 = torch.cat([e.reset()[:, :e.action_dim].clone() for e in envs])
        return panda_targets(q0, total, 1e-3, torch)
    if env.discrete:
        a = torch.randint(0, 2, (total, n_global), generator=gen, device=dev, dtype=torch.int32)
    else:
        a = (torch.rand((total, n_global), generator=gen, device=dev) * 2 - 1) * 50.0
    return a[:, offset:offset + W].contiguous() if (offset or n_global != W) else a


def state_digest(t, dist, world_size, n_global):
    """sha256 of a final per-world state [W_local, k] gathered over the ranks
    into global world order (mwstep.shard.gather_obs; the slab itself at one
    rank): equal digests at different rank counts = the sharded run and its
    gather reproduce the one-GPU result bit for bit (tests/test_gpu_multirank.py)."""
    import hashlib
    if world_size > 1:
        if dist is _NoDist:
            return None
        from mwstep.shard import gather_obs
        t = gather_obs(t.contiguous(), n_global=n_global)
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def make_groups(task, W, S, dev, seed, offset, **kw):
    """S VecEnvs covering worlds [offset, offset + W) in contiguous slices.
    Resets are keyed by the global world index (world_offset), so a grouped
    run is bit-identical to one VecEnv of W worlds (tests/test_gpu_shard.py)."""
    from mwstep.vecenv import VecEnv
    if W % S:
        raise SystemExit(f"--worlds {W} is not divisible by --groups {S}")
    Wg = W // S
    return [VecEnv(task, n_worlds=Wg, device=dev.index, seed=seed, world_offset=offset + g * Wg, **kw)
            for g in range(S)]


def time_steps(envs, actions, warmup, K, chunk, dev, torch, dist, world_size, gather=False):
    n_global = sum(e.n_worlds for e in envs) * world_size  # equal slabs per rank (--worlds per GPU)
    """W untimed warmup steps, then EXACTLY K steps replayed from hipGraphs of
    `chunk` step launches, bracketed by barrier + synchronize; max over ranks.
    Every step reads its action slice where the policy wrote it (the device
    action tensor [T, W]): each chunk's graph is captured with the pointers of
    its own steps, so a replay is the K-step closed loop with nothing but the
    step kernels inside (no per-chunk copy into a staging buffer).

    With several world groups (envs), each group has its own stream (its own
    hardware queue) and graphs; a step = every group advanced once.  The
    groups' kernels overlap each other's launch gaps."""
    from mwstep.shard import gather_obs
    S = len(envs)
    Wg = envs[0].n_worlds
    G = max(1, min(chunk, K))
    n_chunks = (K + G - 1) // G
    groups = []
    keep = []  # the CUDAGraph objects own the executables launched below
    hip_runtime()
    for g, env in enumerate(envs):
        st = torch.cuda.Stream(device=dev)
        env.sim.set_stream(st.cuda_stream)
        acts = actions[:, g * Wg:(g + 1) * Wg].contiguous()
        graphs = []
        with torch.cuda.stream(st):
            env.reset()
            for t in range(warmup):
                env.step_raw(acts[t].data_ptr())
            st.synchronize()
            for c in range(n_chunks):
                t0_ = warmup + c * G
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=st):
                    for t in range(t0_, min(warmup + K, t0_ + G)):
                        env.step_raw(acts[t].data_ptr())
                graphs.append(graph)
            # one untimed replay of every graph: the first launch of an
            # instantiated graph uploads it (more warmup steps, same actions)
            for graph in graphs:
                graph.replay()
        st.synchronize()
        groups.append((env, st, acts, [g.raw_cuda_graph_exec() for g in graphs]))
        keep.extend(graphs)

    if gather:
        # the first RCCL collective sets up its channels (milliseconds): do it
        # once here so the timed region holds only the steady-state all-gather
        st0 = groups[0][1]
        with torch.cuda.stream(st0):
            obs = torch.cat([g[0].obs for g in groups]) if S > 1 else groups[0][0].obs
            gather_obs(obs, n_global=n_global)
        torch.cuda.synchronize(dev)
    ev_start, ev_end = hip_event(), hip_event()
    ev_join = [hip_event() for _ in range(S - 1)]
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # HIP events on group 0's launch stream bracket the timed region (raw
    # hipEventRecord: torch's Event.record costs several us of host time per
    # call); the other groups join it through one event wait at the start and
    # one at the end
    st0 = groups[0][1]
    hip = hip_runtime()
    hip.hipEventRecord(ev_start, st0.cuda_stream)
    for env, st, acts, graphs in groups[1:]:
        hip.hipStreamWaitEvent(st.cuda_stream, ev_start, 0)
    for c in range(n_chunks):
        for env, st, acts, graphs in groups:
            launch_graph(graphs[c], st)
    for (env, st, acts, graphs), ev in zip(groups[1:], ev_join):
        hip.hipEventRecord(ev, st.cuda_stream)
        hip.hipStreamWaitEvent(st0.cuda_stream, ev, 0)
    hip.hipEventRecord(ev_end, st0.cuda_stream)
    if gather:
        with torch.cuda.stream(st0):
            obs = torch.cat([g[0].obs for g in groups]) if S > 1 else groups[0][0].obs
            gathered = gather_obs(obs, n_global=n_global)  # final observation tensor, RCCL over xGMI
    torch.cuda.synchronize(dev)
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    del keep
    kernel_us = hip_elapsed_ms(ev_start, ev_end) * 1e3 / K
    for ev in [ev_start, ev_end] + ev_join:
        hip_runtime().hipEventDestroy(ev)
    final = gathered if gather else (torch.cat([g[0].obs for g in groups]) if S > 1 else groups[0][0].obs)
    import hashlib
    return {"elapsed": elapsed, "kernel_us": kernel_us, "G": G,
            "stream": groups[0][1], "groups": S,
            "gathered_obs_shape": list(gathered.shape) if gather else None,
            "final_obs_sha256": hashlib.sha256(final.detach().cpu().contiguous().numpy().tobytes()).hexdigest(),
            "final_obs": torch.cat([g[0].obs for g in groups]) if S > 1 else groups[0][0].obs}


_HIP = None


def hip_runtime():
    """The HIP runtime library (loaded once, before any timed region)."""
    global _HIP
    import ctypes
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _HIP.hipGraphLaunch.restype = ctypes.c_int
        _HIP.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _HIP.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        _HIP.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        _HIP.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return _HIP


def hip_event():
    """A timing hipEvent_t (raw handle)."""
    import ctypes
    ev = ctypes.c_void_p()
    if hip_runtime().hipEventCreate(ctypes.byref(ev)) != 0:
        raise RuntimeError("hipEventCreate failed")
    return ev


def hip_elapsed_ms(a, b):
    import ctypes
    ms = ctypes.c_float()
    if hip_runtime().hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
        raise RuntimeError("hipEventElapsedTime failed")
    return ms.value


def launch_graph(exe, stream):
    """hipGraphLaunch of a captured graph's executable (`raw_cuda_graph_exec()`,
    fetched before the timed region) on `stream` through the HIP runtime
    directly: torch's CUDAGraph.replay adds ~8 us of host work per call
    (scripts/probe_short_run.py: a 20-step region 75.7 -> 67.9 us)."""
    rc = _HIP.hipGraphLaunch(exe, stream.cuda_stream)
    if rc != 0:
        raise RuntimeError(f"hipGraphLaunch failed: {rc}")


def launch_floor(dev, torch, K=2000, G=100):
    """Per-node time of a hipGraph of G back-to-back 1-element kernels (a
    torch add on one float), replayed like the step graphs: the dispatch /
    completion floor any one-kernel-per-step closed loop pays on this GPU."""
    st = torch.cuda.Stream(device=dev)
    x = torch.zeros(1, device=dev)
    with torch.cuda.stream(st):
        for _ in range(10):
            x.add_(1.0)
        st.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=st):
            for _ in range(G):
                x.add_(1.0)
        graph.replay()
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record(st)
        for _ in range(K // G):
            graph.replay()
        e1.record(st)
    st.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (K // G * G)


def panda_bytes_per_env_step(n=9):
    """Compulsory HBM bytes of one PandaPositionTracking step of one world:
    read q, qlo, qd, targets (4 B x 4n), PID state e/i/u (12n), counters (8 B);
    write q, qlo, qd (12n), PID state (12n), obs 2n floats (8n), reward 4, done 1,
    steps 4.  qlo: low word of the compensated joint positions (kernels.hpp)."""
    return (16 * n + 12 * n + 8) + (12 * n + 12 * n + 8 * n + 9)


def panda_leg(args, dev, torch, dist, world_size=1, rank=0, W_global=1024):
    """BASELINE config 4: 1024 Panda worlds in total, split over the ranks in
    contiguous blocks (strong scaling, "1->8 MI355X shard"); resets are keyed
    by the global world index, so every world's trajectory is the same at any
    rank count (tests/test_gpu_shard.py)."""
    from mwstep.shard import shard_range
    b, e = shard_range(W_global, rank, world_size)
    W = e - b
    K, warm = 1000, 100
    envs = make_groups("PandaPositionTracking", W, args.groups, dev, args.seed, b, max_episode_steps=5000)
    env = envs[0]
    actions = make_actions(envs, warm + K, dev, torch, 0)
    r = time_steps(envs, actions, warm, K, args.graph_chunk, dev, torch, dist, world_size)
    bpe = panda_bytes_per_env_step(env.sim.dofs)
    gbs = bpe * W / (r["kernel_us"] * 1e-6) / 1e9
    out = {"workload": f"PandaPositionTracking: {W_global} worlds (9-dof tree) split over {world_size} GPU(s) "
                       f"({W} per GPU), Position-mode PID every 1 ms step, sinusoidal targets on joints 1 "
                       "and 6 (BASELINE.json configs[3])",
           "value": round(W_global * K / r["elapsed"], 1), "unit": "env·steps/s", "steps": K, "warmup": warm,
           "scaling": "strong", "worlds_per_gpu": W,
           "ms_per_step": round(r["elapsed"] / K * 1e3, 6),
           "kernel_us_per_launch": round(r["kernel_us"], 3),
           "bytes_per_env_step": bpe, "achieved_GBs": round(gbs, 3),
           "hbm_frac": round(gbs / HBM_PEAK_GBS, 6), "groups": args.groups,
           "kernel": "vecenv_pid_group_kernel<9,false,true> (one world per 16-lane row)"}
    out["final_state_sha256"] = state_digest(r["final_obs"], dist, world_size, W_global)
    tr = pmc_traffic("PandaPositionTracking", W)
    out["traffic"] = tr["bytes_per_launch"] if tr else None
    out["algorithmic_bytes_per_launch"] = bpe * W
    out["roofline"] = hbm_roofline(bpe * W, r["elapsed"] / K * 1e6, tr, out["kernel"], r["kernel_us"])
    for e_ in envs:
        e_.close()
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_panda_baseline(args.cpu_leg_seconds)
    return out


def quadruped_leg(args, dev, torch, W=16384, pgs=20, ground=True, exact=True):
    """Articulated floating base with contacts (BASELINE
    config 5's machinery on the authored 8-dof quadruped): W quadrupeds
    standing on the ground plane under the JointController PID (Position
    mode, period = dt), foot / trunk contacts enabled, PGS 20 iterations,
    one physics step per run, replayed from hipGraphs of mw_run_device."""
    import numpy as np
    stand = np.array([0.6, -1.2] * 4)
    rng = np.random.default_rng(args.seed)
    q0 = stand + rng.uniform(-0.1, 0.1, (W, 8))
    out = float_tree_leg(args, dev, torch, "quadruped", W, pgs, 0.45, [(400.0, 10.0, 60.0)] * 8,
                         q0, np.tile(stand, (W, 1)), rng.uniform(-5, 5, (W, 2)), exact=exact)
    solve = ("the boxed LCP solved as DART does (wave_lcp.hpp: two exact box-QP stages, each the primal "
             f"active-set method from the previous step's working set after at most {min(pgs, 4)} PGS sweeps)"
             if exact else f"PGS {pgs} iterations")
    out["workload"] = (f"{W} quadrupeds (16 kg, 8 dofs, floating base) standing on a ground plane under "
                       f"JointController PID hold, sphere-foot / box-trunk contacts, {solve}, dt = 1 ms")
    return out


def humanoid_leg(args, dev, torch, dist=None, world_size=1, rank=0, W_global=512, pgs=50, pgs_opts=(0.0, False),
                 exact=True):
    """BASELINE config 5: 512 iCub-class humanoids in total (models/icub.urdf:
    the reference iCub wrapper's 32 joints and 39 links, 30.7 kg, floating
    base, box feet) split over the ranks, inserted as the wrapper inserts
    them -- base at (0, 0, 0.572), wxyz (0, 0, 0, 1), joints at its
    initial_positions (python/gym_ignition_environments/models/icub.py:19-40,
    :86) -- standing on the ground plane under the JointController PID hold
    of that posture (stiff legs / torso, soft arms), contacts enabled, one
    physics step per run; the one-world-per-wavefront kernel (wave_tree.hpp).
    Worlds sit on an xy grid (no interaction); the state is independent of
    the rank count."""
    import numpy as np
    from mwstep import get_model_file
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    from mwstep.shard import shard_range
    from mwstep.sim import Simulator
    probe = Simulator(get_model_file("icub"), n_worlds=1)
    names = probe.joint_names
    probe.close()
    gains = [(p, d, 80.0) for p, d in icub_pid_gains(names)]
    b, e = shard_range(W_global, rank, world_size)
    q0 = np.tile(icub_posture(names), (W_global, 1))
    rng = np.random.default_rng(args.seed)
    xy = rng.uniform(-5, 5, (W_global, 2))
    out = float_tree_leg(args, dev, torch, "icub", e - b, pgs, ICUB_POSE[2], gains,
                         q0[b:e], q0[b:e], xy[b:e], K=200, G=20, warm=40, wxyz=ICUB_POSE[3:],
                         dist=dist, world_size=world_size, pgs_opts=pgs_opts, exact=exact, W_global=W_global)
    out["value"] = round(W_global * out["steps"] / out["elapsed_s"], 1)
    out["scaling"] = "strong"
    out["worlds_per_gpu"] = e - b
    solve = ("the boxed LCP solved as DART does (wave_lcp.hpp: a frictionless stage, then friction boxed by its "
             "normals; each stage the primal active-set method from the previous step's working set after at most "
             "4 PGS sweeps, <= 48 linear solves per world-step)" if exact
             else f"PGS {pgs} iterations only (mw_set_lcp_solver PGS)")
    out["workload"] = (f"{W_global} iCub-class humanoids (models/icub.urdf: the reference iCub wrapper's 32 joints "
                       f"and 39 links, 30.7 kg, floating base, box feet) split over {world_size} GPU(s), inserted at "
                       f"(0, 0, 0.572) wxyz (0, 0, 0, 1) with the wrapper's initial posture (icub.py:19-40, :86), "
                       f"standing on a ground plane under a JointController PID hold of that posture, "
                       f"{solve}, dt = 1 ms (BASELINE.json configs[4])")
    out["roofline"] = valu_roofline(out["kernel_us_per_launch"], e - b, exact)
    if exact and rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_humanoid_baseline(args.cpu_leg_seconds)
    if pgs_opts[0] > 0.0 or pgs_opts[1]:
        out["workload"] = out["workload"].replace(
            f"PGS {pgs} iterations", f"PGS warm-started from the previous step's impulses, ending when a sweep "
            f"changes no constraint velocity by more than {pgs_opts[0]:g} m/s (at most {pgs} sweeps; "
            f"mw_set_pgs_options)")
        out["accuracy"] = ("closer to the exact boxed-LCP step (DART's Dantzig result) than the cold PGS-50 "
                           "step: tests/test_gpu_float_tree.py::test_humanoid_warm_started_pgs")
    return out


def float_tree_leg(args, dev, torch, model, W, pgs, z0, gains, q0, targets, xy, K=500, G=50, warm=100,
                   dist=None, world_size=1, pgs_opts=(0.0, False), exact=True, W_global=None, wxyz=(1, 0, 0, 0)):
    """Time W floating-base worlds of `model` under a PID hold, one physics
    step per run, replayed from hipGraphs of mw_run_device; with several ranks
    the timed region is bracketed by barriers and the max over ranks is kept."""
    import numpy as np
    from mwstep import get_model_file
    from mwstep import native as N
    from mwstep.sim import Simulator
    stream = torch.cuda.Stream(device=dev)
    sim = Simulator(get_model_file(model), n_worlds=W, device=dev.index, pgs_iters=pgs,
                    stream=stream.cuda_stream, pose=(0, 0, z0, *wxyz))
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    if pgs_opts[0] > 0.0 or pgs_opts[1]:
        sim.set_pgs_options(*pgs_opts)
    if not exact:
        sim.set_lcp_solver(False)
    sim.set("reset_q", q0)
    pose = np.column_stack([xy, np.full(W, z0), np.tile(np.asarray(wxyz, dtype=float), (W, 1))])
    sim.reset_base_pose(pose)
    sim.run(paused=True)
    sim.set_controller_period(1e-3)
    for d, (p, dd, lim) in enumerate(gains):
        sim.set_pid(d, [p, 0.0, dd, -lim, lim, 0.0, 0.0, -1.0])
    sim.set_control_mode(N.MODE_POSITION)
    sim.set("position_target", targets)
    with torch.cuda.stream(stream):
        sim.run_device(warm)
        stream.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            sim.run_device(G)
        graph.replay()
    stream.synchronize()
    n_rep = K // G
    torch.cuda.synchronize(dev)
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        for _ in range(n_rep):
            graph.replay()
        e1.record(stream)
    torch.cuda.synchronize(dev)
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    steps = n_rep * G
    sample = range(0, W, max(1, W // 64))
    pts = [len(sim.contacts(w)) for w in sample]
    z = sim.base_pose()[:, 2]
    out = {"value": round(W * steps / elapsed, 1), "unit": "env·steps/s", "steps": steps,
           "elapsed_s": elapsed,
           "ms_per_step": round(elapsed / steps * 1e3, 6),
           "kernel_us_per_launch": round(e0.elapsed_time(e1) * 1e3 / steps, 3),
           "float_kernel": {1: "world per lane (float_tree.hpp)", 2: "world per wavefront (wave_tree.hpp)"}.get(sim.float_kernel()),
           "contact_points_sampled": f"{sum(pts)} in {len(pts)} worlds",
           "base_z_range_after": [round(float(z.min()), 4), round(float(z.max()), 4)],
           "constraint_overflow": int(sim.constraint_overflow()),
           "lcp_unconverged_world_steps": int(sim.lcp_unconverged()) if sim.float_kernel() == 2 else None}
    if W_global is not None:
        st = torch.from_numpy(np.concatenate([sim.get("q"), sim.get("qd"), sim.base_pose(), sim.base_velocity()],
                                             axis=1)).to(dev)
        out["final_state_sha256"] = state_digest(st, dist, world_size, W_global)
    sim.close()
    return out


def runtime_leg(args, dev, steps=3000):
    """BASELINE config 1's shape on the GPU backend: ONE CartPoleDiscreteBalancing
    world through the unchanged-surface gym stack (gym.make -> GazeboRuntime ->
    Task -> ScenarI/O mirror -> C-ABI mw_run, one kernel + one H2D / D2H copy
    per env step), random actions, seed 42, episodes reset as they end.  This
    is the drop-in plumbing path (per-env Python and getters), not the
    throughput path."""
    import gym_ignition_environments  # noqa: F401
    from gym_ignition_environments import randomizers
    from mwstep import gym_module
    gym = gym_module()
    os.environ.setdefault("MWSTEP_DEVICE", str(dev.index))
    env = randomizers.cartpole_no_rand.CartpoleEnvNoRandomizations(
        env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))
    env.seed(args.seed)
    env.reset()
    for _ in range(200):
        if env.step(env.action_space.sample())[2]:
            env.reset()
    resets = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        if env.step(env.action_space.sample())[2]:
            env.reset()
            resets += 1
    elapsed = time.perf_counter() - t0
    env.close()
    return {"workload": "1 CartPoleDiscreteBalancing world through gym.make / GazeboRuntime / ScenarI/O "
                        "(BASELINE.json configs[0] shape, GPU backend), random actions, seed 42",
            "value": round(steps / elapsed, 1), "unit": "env·steps/s", "steps": steps,
            "ms_per_step": round(elapsed / steps * 1e3, 4), "episode_resets": resets}


def scene_leg(args, dev, torch, W=4096, K=500, warm=100, G=50):
    """Multi-model worlds on the scene kernel (include/mwscene.h): every world
    holds the reference's three-cube contact scene (tests/test_scenario/
    test_contacts.py:125-236: two cubes on the ground, a third across their
    gap, box-box + box-plane contacts) with per-world random offsets, PGS 50,
    one physics step per run, replayed from hipGraphs of mw_scene_run_device."""
    import numpy as np
    from mwstep import get_model_file
    from mwstep.scene import Scene
    stream = torch.cuda.Stream(device=dev)
    sc = Scene(n_worlds=W, device=dev.index, pgs_iters=50)
    sc.set_stream(stream.cuda_stream)
    sc.set_ground_plane(True, 1.0)
    rng = np.random.default_rng(args.seed)
    for k, p in enumerate([(0, -0.15, 0.101), (0, 0.15, 0.101), (0, 0, 0.301)]):
        sc.insert_model(get_model_file("cube"), tuple(p) + (1, 0, 0, 0), f"cube{k + 1}")
        pose = np.column_stack([np.full(W, p[0]) + rng.uniform(-0.01, 0.01, W), np.full(W, p[1]),
                                np.full(W, p[2]) + rng.uniform(0, 0.02, W), np.ones(W), np.zeros((W, 3))])
        sc.reset_base_pose(k, pose)
    sc.run(paused=True)
    with torch.cuda.stream(stream):
        sc.run_device(warm)
        stream.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            sc.run_device(G)
        graph.replay()
    stream.synchronize()
    n_rep = K // G
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        for _ in range(n_rep):
            graph.replay()
        e1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    steps = n_rep * G
    rows = sc.contacts(0)
    fz3 = float(sum(r[8] for r in rows if int(r[12]) == 2)) * -1.0
    out = {"workload": f"{W} worlds x 3 cubes (the three-cube contact KAT scene), box-box + box-plane "
                       "contacts, the boxed LCP solved as DART does (two exact stages, each after at most 4 PGS "
                       "sweeps), dt = 1 ms, scene kernel (one world per wavefront)",
           "value": round(W * steps / elapsed, 1), "unit": "env·steps/s", "steps": steps,
           "ms_per_step": round(elapsed / steps * 1e3, 6),
           "kernel_us_per_launch": round(e0.elapsed_time(e1) * 1e3 / steps, 3),
           "contacts_world0": len(rows), "cube3_support_N_world0": round(fz3, 2),
           "dropped_rows": sc.overflow(), "lcp_unconverged_world_steps": sc.lcp_unconverged()}
    sc.close()
    return out


def contact_leg(args, dev, torch):
    """Floating bodies with ground contacts (SURVEY §8f row 1 slice): 4096 cubes
    (the reference's contact-test cube) dropped from random poses onto the
    ground plane, contacts enabled (read back on the device), one physics step
    per run, replayed from hipGraphs of device-resident runs (mw_run_device)."""
    import numpy as np
    from mwstep import get_model_file
    from mwstep.sim import Simulator
    W, K, warm, G = 4096, 1000, 200, 100
    stream = torch.cuda.Stream(device=dev)
    sim = Simulator(get_model_file("cube"), n_worlds=W, device=dev.index, pgs_iters=20,
                    stream=stream.cuda_stream)
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    rng = np.random.default_rng(args.seed)
    q = rng.normal(size=(W, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    pose = np.column_stack([rng.uniform(-5, 5, (W, 2)), rng.uniform(0.2, 0.6, W), q])
    sim.reset_base_pose(pose)
    sim.reset_base_velocity(np.column_stack([rng.uniform(-1, 1, (W, 3)), rng.uniform(-3, 3, (W, 3))]))
    sim.run(paused=True)
    with torch.cuda.stream(stream):
        sim.run_device(warm)
        stream.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            sim.run_device(G)
        graph.replay()
    stream.synchronize()
    n_rep = K // G
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        for _ in range(n_rep):
            graph.replay()
        e1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    steps = n_rep * G
    in_contact = int(sum(len(sim.contacts(w)) > 0 for w in range(0, W, 16)))
    exact = sim.lcp_solver()[0]
    solve = ("the boxed LCP solved as DART does (wave_lcp.hpp: two exact box-QP stages, each the primal "
             "active-set method from the previous step's working set after at most 4 PGS sweeps)"
             if exact else "PGS 20 iterations")
    out = {"workload": f"{W} floating cubes (5 kg, 0.2 m) on a ground plane, box-plane contacts, "
                       f"normal + 2 friction rows per point, {solve}, dt = 1 ms",
           "kernel": {0: "free_run_kernel (free_body.hpp, PGS only)", 2: "wave_run_kernel (world per wavefront)"}.get(
               sim.float_kernel()),
           "lcp_unconverged_world_steps": int(sim.lcp_unconverged()) if sim.float_kernel() == 2 else None,
           "value": round(W * steps / elapsed, 1), "unit": "env·steps/s", "steps": steps,
           "ms_per_step": round(elapsed / steps * 1e3, 6),
           "kernel_us_per_launch": round(e0.elapsed_time(e1) * 1e3 / steps, 3),
           "worlds_in_contact_sampled": f"{in_contact}/{W // 16}"}
    sim.close()
    return out


VALU_PEAK_PER_S = 1024 * 2.4e9 / 2  # wave-instructions/s: 1,024 SIMDs, one wave64 VALU op per 2 cycles (MI355X_MICROARCH.md)


def hbm_roofline(bytes_per_launch, step_us, traffic, kernel, kernel_us=None):
    """HBM roofline of one launch: algorithmic bytes / the driver-clock time
    per launch (one launch per step); the HIP-event launch period beside it."""
    gbs = bytes_per_launch / (step_us * 1e-6) / 1e9
    out = {"bound": "hbm", "achieved": round(gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 6), "traffic": traffic["bytes_per_launch"] if traffic else None,
           "traffic_source": traffic["source"] if traffic else None,
           "algorithmic_bytes_per_launch": int(bytes_per_launch), "kernel": kernel,
           "time_us_per_launch": round(step_us, 3), "timing": "driver clock (timed wall time / K)",
           "regime": "launch/latency (one dependent chain per world; far below the HBM roof)"}
    if kernel_us is not None:
        out["kernel_us_per_launch"] = round(kernel_us, 3)
        out["achieved_by_launch_period"] = round(bytes_per_launch / (kernel_us * 1e-6) / 1e9, 3)
    return out


def valu_roofline(kernel_us, W, exact):
    """VALU-issue roofline of the world-per-wavefront kernel (config 5): the
    SQ_INSTS_VALU count per launch from the committed rocprofv3 PMC pass
    (profiles/pmc_summary_wave.json, scripts/pmc_summary.py) over this
    launch's measured time, against the chip's VALU issue rate."""
    path = os.path.join(ROOT, "profiles", "pmc_summary_wave.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = None
    d = next((e for e in (d or {}).get("entries", []) if e.get("worlds") == W and e.get("exact_lcp") == exact), None)
    if not d:
        return {"bound": "valu-issue", "achieved": None, "peak": VALU_PEAK_PER_S, "unit": "wave-instr/s",
                "frac": None, "kernel_us_per_launch": kernel_us,
                "note": f"no PMC summary for {W} worlds (exact_lcp={exact}) in profiles/pmc_summary_wave.json"}
    rate = d["valu_insts_per_launch"] / (kernel_us * 1e-6)
    return {"bound": "valu-issue", "achieved": round(rate, 1), "peak": VALU_PEAK_PER_S, "unit": "wave-instr/s",
            "frac": round(rate / VALU_PEAK_PER_S, 6), "valu_insts_per_launch": d["valu_insts_per_launch"],
            "valu_insts_per_wave_step": round(d["valu_insts_per_launch"] / W, 1),
            "lone_wave_ceiling_frac": round(W / 1024 * 0.5, 4),
            "kernel_us_per_launch": kernel_us, "source": os.path.relpath(path, ROOT),
            "regime": "latency: one world per wavefront, <= 1 wave per SIMD, a lone wave issues one VALU op "
                      "per 4 cycles at best"}


def host_threads():
    """Host cores this process may use, at most 16 (the GPU box's CPU share)."""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        return ""


def _threaded(make, run, seconds, probe_units):
    """Size a per-thread sample to ~`seconds` from a one-thread probe of
    `probe_units`, then run it on every host thread at once (the oracle's C
    calls release the GIL).  make() -> per-thread state; run(state, units)."""
    from concurrent.futures import ThreadPoolExecutor
    st = make()
    t0 = time.perf_counter()
    run(st, probe_units)
    per_unit = (time.perf_counter() - t0) / probe_units
    units = int(max(probe_units, seconds / max(per_unit, 1e-9)))
    threads = host_threads()
    states = [make() for _ in range(threads)]
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.perf_counter()
        list(pool.map(lambda x: run(x, units), states))
        wall = time.perf_counter() - t0
    return threads, units, wall


def cpu_vec_baseline(task, seed, seconds, Wc=2048):
    """fp64 C oracle VecEnv of `task` (the same env the GPU runs) on every host thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from mwstep import get_model_file
    from mwstep.vecenv import TASKS
    kind, model = TASKS[task]
    cm = pyoracle.load_urdf(get_model_file(model))
    acts = np.random.default_rng(43).uniform(-50.0, 50.0, (64, Wc))

    def make():
        e = pyoracle.VecEnv(cm, pyoracle.make_task(kind, seed=seed), Wc)
        e.reset()
        return e

    def run(e, T):
        for t0 in range(0, T, 64):
            e.rollout(acts[:min(64, T - t0)])

    threads, T, wall = _threaded(make, run, seconds, 10)
    return {"value": round(threads * Wc * T / wall, 1), "unit": "env·steps/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {Wc} worlds x {T} env steps of {task}, fp64 C oracle "
                      f"({wall:.1f} s wall; {cpu_model_name()})"}


def cpu_panda_baseline(seconds, Wc=64):
    """BASELINE config 4 on the host: the fp64 oracle's Panda (9-dof tree,
    joint-limit LCP, PGS 20) under the JointController PID, sinusoidal targets
    on joints 1 and 6 (or_pid_rollout), Wc worlds per thread, every host thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from mwstep import get_model_file
    cm = pyoracle.load_urdf(get_model_file("panda"))
    n = cm.n
    lo, hi = np.array(cm.model.lower[:n]), np.array(cm.model.upper[:n])
    q0 = np.tile((lo + hi) / 2, (Wc, 1))
    amp = np.zeros(n)
    amp[0], amp[5] = 0.9 * (2 * 2.8973) / 2, 0.9 * (3.7525 + 0.0175) / 2
    from mwstep.models import PANDA_PID_GAINS_1000HZ
    # ScenarI/O's setPID clamps the command to +-effort (Joint.cpp:504-513)
    gains = [pyoracle.pid_gains(*PANDA_PID_GAINS_1000HZ[nm], cmdmax=cm.model.effort[i], cmdmin=-cm.model.effort[i])
             for i, nm in enumerate(cm.joint_names)]

    def make():
        return [q0.copy(), np.zeros((Wc, n)), None]

    def run(st, T):
        st[2] = pyoracle.pid_rollout(cm, st[0], st[1], q0, amp, 0.33, gains, T, pgs_iters=20, states=st[2])

    threads, T, wall = _threaded(make, run, seconds, 20)
    return {"value": round(threads * Wc * T / wall, 1), "unit": "env·steps/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {Wc} Panda worlds x {T} PID-tracking steps (physics + PID, no task "
                      f"I/O), fp64 C oracle ({wall:.1f} s wall; {cpu_model_name()})"}


def cpu_humanoid_baseline(seconds):
    """BASELINE config 5 on the host: one fp64 oracle iCub-class humanoid
    (dense CRBA + contact LCP solved exactly, PGS_CONVERGED -- the GPU
    default's problem) from the wrapper's posture and pose under the PID hold
    per thread (or_float_pid_rollout), every host thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from mwstep import get_model_file
    from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture
    cm = pyoracle.load_urdf(get_model_file("icub"), pose_xyz=ICUB_POSE[:3], pose_wxyz=ICUB_POSE[3:])
    n = cm.n
    q0 = np.array(icub_posture(cm.joint_names))
    gains = [pyoracle.pid_gains(p, 0.0, d, cmdmax=80.0, cmdmin=-80.0) for p, d in icub_pid_gains(cm.joint_names)]

    def make():
        fw = pyoracle.FloatWorld(cm, pgs_iters=pyoracle.PGS_CONVERGED)
        fw.set_joints(q0, np.zeros(n))
        return [fw, None]

    def run(st, T):
        st[1] = pyoracle.float_pid_rollout(st[0], q0, gains, T, states=st[1])

    threads, T, wall = _threaded(make, run, seconds, 5)
    return {"value": round(threads * T / wall, 1), "unit": "env·steps/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x 1 iCub-class humanoid x {T} steps standing under the PID hold, exact contact "
                      f"LCP, fp64 C oracle ({wall:.1f} s wall; {cpu_model_name()})"}


def pmc_traffic(task, W):
    """HBM bytes per launch of the step kernel from the committed PMC summary
    (profiles/pmc_summary.json, or pmc_summary_panda.json for config 4;
    produced by scripts/pmc_summary.py from rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of scripts/profile_step.py / profile_panda.py)."""
    name = {"PandaPositionTracking": "pmc_summary_panda.json",
            "PendulumSwingUp": "pmc_summary_pendulum.json"}.get(task, "pmc_summary.json")
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("task") != task or d.get("worlds") != W:
        return None
    return {"bytes_per_launch": d["bytes_per_launch"], "source": os.path.relpath(path, ROOT)}


def world_sweep(args, dev, torch):
    from mwstep.vecenv import VecEnv
    out = []
    for W in (16384, 65536, 262144, 1048576):
        env = VecEnv(args.task, n_worlds=W, device=dev.index, seed=args.seed)
        stream = torch.cuda.Stream(device=dev)
        env.sim.set_stream(stream.cuda_stream)
        G, reps = 20, 5
        acts = torch.randint(0, 2, (G, W), device=dev, dtype=torch.int32) if env.discrete else \
            (torch.rand((G, W), device=dev) * 2 - 1) * 50.0
        with torch.cuda.stream(stream):
            env.reset()
            for g in range(G):
                env.step_raw(acts[g].data_ptr())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for g in range(G):
                    env.step_raw(acts[g].data_ptr())
            graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                graph.replay()
            e1.record(stream)
        stream.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (G * reps)
        bpe = algorithmic_bytes_per_env_step(env.sim.dofs, env.obs_dim)
        out.append({"worlds": W, "us_per_step": round(us, 3), "env_steps_per_s": round(W / (us * 1e-6), 1),
                    "achieved_GBs": round(bpe * W / (us * 1e-6) / 1e9, 1),
                    "hbm_frac": round(bpe * W / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)})
        env.close()
        del acts, graph
    return out


def dart_probe():
    """is a DART (the reference's physics engine) runtime on
    this host?  `ldconfig -p` lines naming dart; nothing is installed or run."""
    import subprocess
    try:
        out = subprocess.run(["ldconfig", "-p"], capture_output=True, text=True, timeout=20).stdout
    except (OSError, subprocess.SubprocessError) as e:
        return {"found": False, "probe": f"ldconfig -p failed: {e}"}
    libs = sorted({ln.split()[0] for ln in out.splitlines() if "dart" in ln.lower() and ln.strip()})
    return {"found": bool(libs), "libs": libs[:8],
            "probe": "ldconfig -p | grep -i dart",
            "note": ("DART libraries present, but not ign-gazebo/ign-physics: the reference path is still "
                     "not runnable" if libs else "no DART on this host: the reference CPU path cannot run")}


def cpu_baseline_and_parity(args, env, np, torch):
    """fp64 C oracle (oracle/, test infrastructure) on a bounded sample of the
    same workload (its own actions: PCG64(43) Bernoulli(0.5) for the discrete
    task, U(-50, 50) otherwise -- SURVEY §8d), on every host core this process
    may use; plus a teacher-forced one-step parity check of the GPU kernel
    against it on 256 worlds x 100 steps.  Nothing here depends on --steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from mwstep import get_model_file
    from mwstep.vecenv import TASKS

    kind, model = TASKS[args.task]
    cm = pyoracle.load_urdf(get_model_file(model))
    Wc, T_max = 4096, 4000
    rng = np.random.default_rng(43)
    if kind == 0:
        acts = rng.integers(0, 2, (T_max, Wc)).astype(np.int32)
    else:
        acts = rng.uniform(-50.0, 50.0, (T_max, Wc))
    ref = pyoracle.VecEnv(cm, pyoracle.make_task(kind, seed=args.seed), Wc)
    ref.reset()
    t0 = time.perf_counter()
    ref.rollout(acts[:20])
    probe = time.perf_counter() - t0
    T = int(max(20, min(T_max, args.cpu_seconds / max(probe / 20, 1e-9))))
    ref.reset()
    t0 = time.perf_counter()
    ref.rollout(acts[:T])
    cpu_s = time.perf_counter() - t0
    single = Wc * T / cpu_s
    # the same sample on every host core this process may use (at most 16,
    # the box's CPU share): one oracle VecEnv of Wc worlds per thread, the C
    # rollout releases the GIL (ctypes), worlds are independent
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    envs = [pyoracle.VecEnv(cm, pyoracle.make_task(kind, seed=args.seed + k), Wc) for k in range(threads)]
    for e in envs:
        e.reset()
    a_T = np.ascontiguousarray(acts[:T])
    with ThreadPoolExecutor(threads) as pool:
        t0 = time.perf_counter()
        list(pool.map(lambda e: e.rollout(a_T), envs))
        mt_s = time.perf_counter() - t0
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    dart = dart_probe()
    cpu = {"value": round(threads * Wc * T / mt_s, 1), "unit": "env·steps/s", "cores": threads, "kind": "port",
           "sample": f"{threads} threads x {Wc} worlds x {T} env steps of {args.task}, fp64 C oracle "
                     f"({mt_s:.1f} s wall; {cpu_model}); the reference's ign-gazebo+DART path is not buildable here",
           "single_thread_value": round(single, 1),
           "single_thread_sample": f"{Wc} worlds x {T} env steps, 1 thread ({cpu_s:.1f} s)",
           "dart_probe": dart}

    # teacher-forced one-step parity on 256 worlds x 100 steps
    from mwstep.vecenv import VecEnv
    Wp, Tp = 256, 100
    gpu = VecEnv(args.task, n_worlds=Wp, device=env.device.index, seed=args.seed)
    orc = pyoracle.VecEnv(cm, pyoracle.make_task(kind, seed=args.seed), Wp)
    gpu.reset()
    orc.reset()
    worst = 0.0
    n = cm.n
    for t in range(Tp):
        gpu.set_state(torch.from_numpy(orc.q.reshape(n, Wp)), torch.from_numpy(orc.qd.reshape(n, Wp)))
        a = acts[t, :Wp]
        o, _, d, _ = gpu.step(torch.from_numpy(np.ascontiguousarray(a).astype(
            np.int32 if kind == 0 else np.float32)).to(gpu.device))
        o, d = o.cpu().numpy(), d.cpu().numpy().astype(bool)
        orf, _, drf, _ = orc.step(a)
        m = ~(d | drf)
        if m.any():
            worst = max(worst, float(np.abs(o[m] - orf[m]).max()))
    gpu.close()
    return cpu, {"value": worst, "mode": f"one-step teacher-forced, {Wp} worlds x {Tp} steps",
                 "vs": "fp64 DART-semantics oracle (DART itself absent: parity unpinned)"}


if __name__ == "__main__":
    main()
