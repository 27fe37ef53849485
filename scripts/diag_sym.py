"""Diagnostic: where does the fp32 kernel break the exact level-flight symmetry?"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import qs_oracle
from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout
G = grid_layout(8)
np.set_printoptions(precision=3, linewidth=200)
for prec in (4, 8):
    sw = QuadSwarm("multihover", num_envs=4, num_drones=8, act="one_d_pid", precision=prec, initial_xyzs=G)
    orc = qs_oracle.OracleSim(task="multihover", num_envs=4, num_drones=8, act="one_d_pid", precision=prec, initial_xyzs=G)
    sw.reset(11); orc.reset(11)
    for t in range(6):
        sw.step(None); orc.step(None); torch.cuda.synchronize()
        g = sw.get_state(0).cpu().numpy(); o = orc.get_state(0)
        print(f"prec {prec} t={t} max|quat xyz| gpu {np.abs(g[3:6]).max():.3e} oracle {np.abs(o[3:6]).max():.3e}"
              f" max|w| gpu {np.abs(g[10:13]).max():.3e} oracle {np.abs(o[10:13]).max():.3e}"
              f" max|vel xy| gpu {np.abs(g[7:9]).max():.3e} oracle {np.abs(o[7:9]).max():.3e}"
              f" pid int_rpy gpu {np.abs(g[20:23]).max():.3e} oracle {np.abs(o[20:23]).max():.3e}"
              f" rpm spread gpu {np.abs(g[13:17]-g[13:14]).max():.3e} oracle {np.abs(o[13:17]-o[13:14]).max():.3e}")
    # one-step probe from an exactly level state: which field goes non-zero first?
    st = orc.get_state(0)
    sw.set_state(0, torch.as_tensor(st))
    for block in (1, 2, 3):
        sw.set_state(block, torch.as_tensor(orc.get_state(block)))
    sw.step(None); orc.step(None); torch.cuda.synchronize()
    g = sw.get_state(0).cpu().numpy(); o = orc.get_state(0)
    d = np.abs(g - o).max(axis=1)
    print("per-field max |gpu-oracle| after one injected step:", d)
