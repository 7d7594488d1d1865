"""Eager launches of the per-step env kernel for PMC counter passes
(rocprofv3 --pmc ... -- python3 scripts/profile_step.py): 4096 CartPole
worlds, 300 steps, one dispatch per step (no graph).  MW_TASK=PendulumSwingUp
MW_W=2048: the config-3 kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ignition_amd", "python"))
import torch  # noqa: E402

from mwstep.vecenv import VecEnv  # noqa: E402

W, T = int(os.environ.get("MW_W", "4096")), int(os.environ.get("MW_T", "300"))
task = os.environ.get("MW_TASK", "CartPoleDiscreteBalancing")
env = VecEnv(task, n_worlds=W)
env.reset()
if env.discrete:
    acts = torch.randint(0, 2, (T, W), device="cuda", dtype=torch.int32)
else:
    acts = (torch.rand((T, W), device="cuda") * 2 - 1) * 50.0
for t in range(T):
    env.step_raw(acts[t].data_ptr())
torch.cuda.synchronize()
print("ok", W, T)
