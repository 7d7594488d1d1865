"""Phase breakdown of the one-world-per-wavefront kernel (wave_tree.hpp) on
BASELINE config 5's workload (512 iCub-class worlds standing, models/icub.urdf).

Needs the debug build with shader-clock phase counters:
    make -C gym-ignition_amd BUILD=build_prof LIB=libmwstep_prof.so EXTRA=-DMW_WAVE_PROF
    MWSTEP_LIB=gym-ignition_amd/libmwstep_prof.so python scripts/wave_prof.py [W] [pgs]
Prints shader-clock cycles per world-step of every phase (sum over worlds / worlds / steps)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import numpy as np  # noqa: E402

from mwstep import get_model_file  # noqa: E402
from mwstep import native as N  # noqa: E402
from mwstep.sim import Simulator  # noqa: E402

from lcp_dumps import save_dumps  # noqa: E402


W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
PGS = int(sys.argv[2]) if len(sys.argv) > 2 else 50
print(f"exact={os.environ.get('MW_PROF_EXACT', '1')} warm={os.environ.get('MW_PROF_WARM', '0')}")
T = int(os.environ.get("MW_PROF_T", "20"))
PHASES = ["dof_force (PID)", "ABA (uniform)", "integrate + detect + row setup", "responses (lane = row)",
          "Delassus (lane = column)", "PGS + exact LCP", "rows total (responses .. integrate)", "whole substep"]

if os.environ.get("MW_PROF_MODEL", "icub") == "scene3":
    # the bench's scene leg (bench.scene_leg): three stacked cubes per world
    from mwstep.scene import Scene
    sc = Scene(n_worlds=W, pgs_iters=50)
    sc.set_ground_plane(True, 1.0)
    rng = np.random.default_rng(42)
    for k, p in enumerate([(0, -0.15, 0.101), (0, 0.15, 0.101), (0, 0, 0.301)]):
        sc.insert_model(get_model_file("cube"), tuple(p) + (1, 0, 0, 0), f"cube{k + 1}")
        pose = np.column_stack([np.full(W, p[0]) + rng.uniform(-0.01, 0.01, W), np.full(W, p[1]),
                                np.full(W, p[2]) + rng.uniform(0, 0.02, W), np.ones(W), np.zeros((W, 3))])
        sc.reset_base_pose(k, pose)
    sc.run(paused=True)
    sc.run_device(100)
    fn = N.lib().mw_debug_scene_prof
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 22)()
    fn(buf)
    t0 = time.perf_counter()
    for _ in range(T):
        sc.run()          # blocking runs: the counters are read after the last
    dt = time.perf_counter() - t0
    fn(buf)
    ns = max(buf[18], 1)
    print(f"scene 3 cubes x{W}: {dt / T * 1e6:.1f} us per blocking run, {buf[18]} exact solves, unconverged {buf[15]}; "
          f"per solve: {buf[8] / ns:.2f} linear solves ({buf[10] / ns:.2f} in stage 2), {buf[9] / ns:.2f} rounds, "
          f"max {buf[11]}, {buf[13]} > 4; cycles: {buf[14] / ns:.0f} in solves, {buf[16] / ns:.0f} in sweeps, "
          f"{buf[17] / ns:.0f} in stage 1, {buf[12] / ns:.0f} in the whole exact solve")
    nst = max(buf[7], 1)
    for k, name in enumerate(["ABA + integrateVelocities", "contacts + row setup", "responses (lane = row)",
                              "Delassus (lane = column)", "PGS / exact LCP", "impulses .. integratePositions",
                              "whole step"]):
        print(f"  {name:40s} {buf[k] / nst:12.0f} cycles/world-step")
    print(f"  inside contacts: ground slots {buf[19] / nst:.0f}, shape pairs {buf[20] / nst:.0f} "
          f"(their first pass's narrow phase {buf[21] / nst:.0f}) cycles/world-step")
    save_dumps(N.lib().mw_debug_scene_dump, 8, "scene_dump.npz")
    sys.exit(0)
if os.environ.get("MW_PROF_MODEL", "icub") == "cube":
    # the bench's contacts leg (bench.contact_leg): cubes dropped from random poses
    sim = Simulator(get_model_file("cube"), n_worlds=W, pgs_iters=20)
    sim.set_ground_plane(True, 1.0)
    sim.enable_contacts(True)
    rng = np.random.default_rng(0)
    qq = rng.normal(size=(W, 4))
    qq /= np.linalg.norm(qq, axis=1, keepdims=True)
    sim.reset_base_pose(np.column_stack([rng.uniform(-5, 5, (W, 2)), rng.uniform(0.2, 0.6, W), qq]))
    sim.reset_base_velocity(np.column_stack([rng.uniform(-1, 1, (W, 3)), rng.uniform(-3, 3, (W, 3))]))
    sim.run(paused=True)
    sim.run_device(200)
    L = N.lib()
    fn = L.mw_debug_wave_prof
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 22)()
    fn(buf)
    t0 = time.perf_counter()
    sim.run_device(T)
    sim.get("q")
    dt = time.perf_counter() - t0
    fn(buf)
    print(f"cube x{W}: {dt / T * 1e6:.1f} us/step wall, unconverged {sim.lcp_unconverged()}")
    for k, name in enumerate(PHASES):
        print(f"  {name:40s} {buf[k] / W / T:12.0f} cycles/world-step")
    print(f"  exact LCP: {buf[8] / W / T:.2f} solves per world-step, max {buf[11]}, {buf[13]} world-steps > 4; "
          f"{buf[14] / W / T:.0f} cycles in the solves, {buf[16] / W / T:.0f} in the sweeps, "
          f"{buf[17] / W / T:.0f} in stage 1")
    save_dumps(L.mw_debug_wave_dump, 9, "wave_dump.npz")
    sys.exit(0)
from mwstep.models import ICUB_POSE, icub_pid_gains, icub_posture  # noqa: E402
sim = Simulator(get_model_file("icub"), n_worlds=W, pgs_iters=PGS, pose=ICUB_POSE)
names = sim.joint_names
sim.set_ground_plane(True, 1.0)
sim.enable_contacts(True)
sim.set_controller_period(1e-3)
for d, (p, dd) in enumerate(icub_pid_gains(names)):
    sim.set_pid(d, [p, 0.0, dd, -80.0, 80.0, 0.0, 0.0, -1.0])
sim.set_control_mode(N.MODE_POSITION)
post = np.tile(icub_posture(names), (W, 1))
sim.set("position_target", post)
# the bench leg's start: the wrapper's posture (bench.humanoid_leg); MW_PROF_RANDOM=1 adds U(-0.02, 0.02)
jit = np.random.default_rng(42).uniform(-0.02, 0.02, (W, sim.dofs)) if os.environ.get("MW_PROF_RANDOM", "0") != "0" else 0.0
sim.set("reset_q", post + jit)
sim.run(paused=True)
# solver options: MW_PROF_EXACT=0 -> PGS only; MW_PROF_WARM=1 -> warm-started sweeps
sim.set_lcp_solver(os.environ.get("MW_PROF_EXACT", "1") != "0")
if os.environ.get("MW_PROF_WARM", "0") != "0":
    sim.set_pgs_options(0.0, True)
sim.run_device(50)
L = N.lib()
fn = L.mw_debug_wave_prof
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 22)()
fn(buf)  # clear
t0 = time.perf_counter()
sim.run_device(T)
sim.get("q")
dt = time.perf_counter() - t0
fn(buf)
print(f"{W} worlds, PGS {PGS}, {T} steps: {dt / T * 1e6:.1f} us/step wall; contacts in world 0: {len(sim.contacts(0))}")
for k, name in enumerate(PHASES):
    print(f"  {name:40s} {buf[k] / W / T:12.0f} cycles/world-step")
print(f"  exact LCP: {buf[8] / W / T:.2f} linear solves and {buf[9] / W / T:.2f} rounds per world-step; "
      f"{buf[10] / W / T:.2f} of the solves in stage 2 (friction boxes); max per world-step {buf[11]} solves, "
      f"{buf[12]} in stage 2; {buf[13]} of {W * T} world-steps > 4 solves; "
      f"{buf[14] / W / T:.0f} cycles/world-step in the linear solves, {buf[15] / W / T:.0f} in the PGS sweeps "
      f"(PGS-only mode) / the whole exact solve incl. its per-stage sweeps (exact mode); "
      f"{buf[16] / W / T:.0f} in the per-stage sweeps, {buf[17] / W / T:.0f} in stage 1")
if buf[18] or buf[19]:
    print(f"  inside the first phase: [18] {buf[18] / W / T:.0f}, [19] {buf[19] / W / T:.0f} cycles/world-step "
          f"(ABA: outward pass 1, inward pass; joint-space step: tree passes + CRBA, factorisation + free solve)")
if buf[20]:
    print(f"  kernel prologue (entry to the first substep): {buf[20] / W / T:.0f} cycles/world-launch")
save_dumps(L.mw_debug_wave_dump, 9, "wave_dump.npz")
sim.close()
