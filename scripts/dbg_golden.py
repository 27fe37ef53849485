"""Dev: locate the first golden-vector mismatch of the kernel (which step, which obs columns)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "tests", "golden")]
import make_golden as mg
from gym_pybullet_drones_amd.envs import QuadSwarm
GOLD = np.load(os.path.join(ROOT, "tests", "golden", "oracle_golden.npz"))
name = sys.argv[1] if len(sys.argv) > 1 else "mh_rpm_d4"
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 8
kw = dict(mg.CASES[name]); kw.pop("aux", None)
sw = QuadSwarm(num_envs=mg.E, precision=prec, **kw)
o0 = sw.reset(mg.SEED).cpu().numpy()
print("obs0 maxdiff", np.abs(o0 - GOLD[f"{name}/obs0"]).max())
act = torch.zeros((mg.E, sw.num_drones, sw.act_dim), device=sw.device)
for t in range(mg.STEPS):
    r = sw.step(None, actions_out=act)
    o = r.obs.cpu().numpy(); g = GOLD[f"{name}/obs"][t]
    bad = np.argwhere(np.abs(o - g) > 2e-6 + 2e-6 * np.abs(g))
    if len(bad):
        print("step", t, "nbad", len(bad), "cols", sorted(set(bad[:, 2].tolist()))[:40], "reset_error", sw.reset_error())
        print("term", r.terminated.cpu().numpy(), "trunc", r.truncated.cpu().numpy())
        print("pos got", o[:, :, 0:3].round(4).tolist()); print("pos want", g[:, :, 0:3].round(4).tolist())
        e, d, c = bad[0]
        print("env", e, "drone", d, "row got", np.round(o[e, d, 12:], 4).tolist())
        print("               want", np.round(g[e, d, 12:], 4).tolist())
        break
else:
    print("all steps match")
