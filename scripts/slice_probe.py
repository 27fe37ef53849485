"""Dev: first-exceed steps of the fp32 kernel (the library QS_DEV_LIB selects)
and of the exact-fp32 oracle on the full-size test slices and a few 64-env
seeds of the sensitive configs (tests/test_gpu_tolerance.py shapes)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import trajectory as tj  # noqa: E402
from gym_pybullet_drones_amd.envs.swarm import grid_layout  # noqa: E402

G8, G16 = grid_layout(8).tolist(), grid_layout(16).tolist()
CFGS = {
    "C3v": (dict(task="multihover", num_drones=8, act="vel", initial_xyzs=G8), 16384),
    "C4": (dict(task="spiral", num_drones=5, act="vel"), 8192),
    "C5": (dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, physics="pyb", aux=("dw",)), 8192),
}
B = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)
oracle = "oracle" in sys.argv[1:]
names = [a for a in sys.argv[1:] if a in CFGS] or list(CFGS)
for name in names:
    cfg, full = CFGS[name]
    lo = full - 16 - 5
    subj = "oracle" if oracle else "kernel"
    r = tj.diverge(cfg, E=16, precision=4, steps=60, env_offset=lo, full_E=None if oracle else full, subject=subj)
    out = {"slice": {k: tj.first_exceed(r["curves"][k], b) for k, b in B.items()}}
    for sd in (11, 12, 13, 14):
        r = tj.diverge(cfg, E=64, precision=4, steps=60, seed=sd, subject=subj)
        out[f"s{sd}"] = {k: tj.first_exceed(r["curves"][k], b) for k, b in (("pos", 1e-4), ("vel", 1e-3))}
    print(subj, name, json.dumps(out), flush=True)
