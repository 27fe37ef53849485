"""Workload for a rocprofv3 --pmc pass: the bench's C5 (MultiHover 16 drones x 8192
envs, ONE_D_PID, PYB_DW) and C3 step kernels, 30 control steps each, so the VALU
instruction count per agent-step can be read per kernel (profiles/r02_valu.json)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
import torch  # noqa: E402

from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout  # noqa: E402
from gym_pybullet_drones_amd.utils.enums import Physics  # noqa: E402

torch.cuda.set_device(0)
for E, D, phys in ((8192, 16, Physics.PYB_DW), (16384, 8, Physics.DYN)):
    sw = QuadSwarm("multihover", num_envs=E, num_drones=D, act="one_d_pid", precision=4, physics=phys,
                   initial_xyzs=grid_layout(D))
    sw.reset(0)
    for _ in range(30):
        sw.step(None)
    torch.cuda.synchronize()
    sw.close()
    print("agents", E * D, phys)
