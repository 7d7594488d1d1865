import cProfile, pstats, sys, os, time
sys.path.insert(0, "gym-ignition_amd/python")
import gym_ignition_environments  # noqa
from gym_ignition_environments import randomizers
from mwstep import gym_module
gym = gym_module()
env = randomizers.cartpole_no_rand.CartpoleEnvNoRandomizations(env=lambda **kw: gym.make("CartPoleDiscreteBalancing-Gazebo-v0", **kw))
env.seed(42); env.reset()
def run(n):
    for _ in range(n):
        if env.step(env.action_space.sample())[2]:
            env.reset()
run(200)
pr = cProfile.Profile(); pr.enable(); t0=time.perf_counter(); run(2000); dt=time.perf_counter()-t0; pr.disable()
print("us/step", dt/2000*1e6)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
