"""Workload for the bound-naming SQ passes: the bench's C5
(MultiHover 16 x 8192, ONE_D_PID, PYB_DW: step_kernel<float,0,4,30,0,1>), C4
(Spiral 5 x 8192, VEL, DYN: step_kernel<float,1,2,48,1,0>) and C3 (the headline,
MultiHover 8 x 16384, ONE_D_PID, DYN) step kernels, 40 control steps each from
staggered episode clocks (bench.py stagger_episodes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), ROOT]
import torch  # noqa: E402

from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout  # noqa: E402
from gym_pybullet_drones_amd.utils.enums import Physics  # noqa: E402
from bench import stagger_episodes  # noqa: E402

torch.cuda.set_device(0)
CFGS = [("C5", "multihover", 8192, 16, "one_d_pid", Physics.PYB_DW),
        ("C4", "spiral", 8192, 5, "vel", Physics.DYN),
        ("C3", "multihover", 16384, 8, "one_d_pid", Physics.DYN)]
for name, task, E, D, act, phys in CFGS:
    kw = dict(initial_xyzs=grid_layout(D)) if task == "multihover" else {}
    sw = QuadSwarm(task, num_envs=E, num_drones=D, act=act, precision=4, physics=phys, **kw)
    sw.reset(0)
    stagger_episodes(sw, task)
    for _ in range(40):
        sw.step(None)
    torch.cuda.synchronize()
    sw.close()
    print(name, "agents", E * D, flush=True)
