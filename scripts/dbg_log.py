import sys, numpy as np, torch
sys.path.insert(0, 'marl-gym-pybullet-drones_amd')
from gym_pybullet_drones_amd.utils.enums import ActionType
from gym_pybullet_drones_amd.vec_env import SwarmVecEnv
from gym_pybullet_drones_amd import _lib as L
E, D = 8192, 4
venv = SwarmVecEnv(task="multihover", num_envs=E, num_drones=D, act=ActionType.RPM, seed=5, precision=4)
venv.reset()
sw = venv.swarm
for _ in range(200):
    venv.step_t()
torch.cuda.synchronize()
full, total = sw.episode_log(cap=1 << 22)
env = sw.get_state(L.STATE_ENV).cpu().numpy()
print("total", total, "len(full)", len(full), "env state shape", env.shape)
print("episode counters sum", env[1].sum(), "max", env[1].max())
print("seq range", full["seq"].min() if len(full) else None, full["seq"].max() if len(full) else None)
