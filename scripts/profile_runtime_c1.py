"""cProfile of BASELINE config 1's per-env path on the GPU backend (one
CartPole world through gym.make -> GazeboRuntime -> Task -> ScenarI/O mirror ->
mw_scene_run): where the time of one env step goes.
    python scripts/profile_runtime_c1.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-ignition_amd", "python"))
import gym_ignition_environments  # noqa: E402,F401
from gym_ignition_environments import randomizers  # noqa: E402
from mwstep import gym_module  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
gym = gym_module()
env = randomizers.cartpole_no_rand.CartpoleEnvNoRandomizations(
    env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))
env.seed(42)
env.reset()


def loop(n):
    for _ in range(n):
        if env.step(env.action_space.sample())[2]:
            env.reset()


loop(200)
t0 = time.perf_counter()
loop(steps)
dt = time.perf_counter() - t0
print(f"{steps / dt:.1f} env-steps/s, {dt / steps * 1e6:.1f} us/step (no profiler)")
pr = cProfile.Profile()
pr.enable()
loop(steps)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
env.close()
