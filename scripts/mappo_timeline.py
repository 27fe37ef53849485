"""Dev: one PPO minibatch iteration (the captured graph) replayed a few times, for a
rocprofv3 --kernel-trace timeline of its kernels (scripts/mappo_timeline.sh)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
sys.path.insert(0, ROOT)
import torch
from gym_pybullet_drones_amd.envs import MultiHoverAviary, grid_layout
from gym_pybullet_drones_amd.mappo import MAPPO
from gym_pybullet_drones_amd.utils.enums import ActionType, Physics
E, D = int(os.environ.get("E", 16384)), 8
env_func = lambda seed=0: MultiHoverAviary(num_drones=D, act=ActionType.ONE_D_PID, physics=Physics.DYN,
                                           initial_xyzs=grid_layout(D))
m = MAPPO(env_func, training=True, seed=0, hidden_dim=256, actor_lr=3e-4, critic_lr=1e-3, rollout_steps=32,
          rollout_batch_size=E, opt_epochs=1, mini_batch_size=4096, output_dir="/tmp/qs_tl")
m.reset()
m.train_step()
torch.cuda.synchronize()
ag = m.agent
for _ in range(5):
    ag._graph.replay()
torch.cuda.synchronize()
print("ok")
