"""Divergence curves of the fp32 (and fp64) HIP kernel from the fp64 oracle per
BASELINE config, free-running over >= 2 episodes (profiles/r02_tolerance_curves.json).
GPU script; test infrastructure (uses the oracle as the checker)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import trajectory as tj  # noqa: E402
from gym_pybullet_drones_amd.envs.swarm import grid_layout  # noqa: E402

G8, G16 = grid_layout(8).tolist(), grid_layout(16).tolist()
CFGS = {
    "C2": dict(task="multihover", num_drones=4, act="rpm"),
    "C2p": dict(task="multihover", num_drones=4, act="rpm", physics="pyb"),
    "C3": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8),
    "C3p": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8, physics="pyb"),
    "C3v": dict(task="multihover", num_drones=8, act="vel", initial_xyzs=G8),
    "C4": dict(task="spiral", num_drones=5, act="vel"),
    "C5": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, physics="pyb", aux=("dw",)),
    "C5d": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, aux=("dw",)),
}
out = {}
names = sys.argv[1:] or list(CFGS)
for name in names:
    cfg = CFGS[name]
    steps = 1156 if cfg["task"] == "spiral" else 484
    for prec in (4, 8):
        t0 = time.time()
        r = tj.diverge(cfg, E=64, precision=prec, steps=steps)
        cv = r["curves"]
        rec = {k: v for k, v in r.items() if k != "curves"}
        rec["first_pos_gt"] = {b: tj.first_exceed(cv["pos"], b) for b in (1e-6, 1e-5, 1e-4, 1e-3)}
        rec["first_rew_gt"] = {b: tj.first_exceed(cv["rew"], b) for b in (1e-5, 1e-4)}
        bound = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4) if prec == 4 else dict(pos=1e-9, quat=1e-9, vel=1e-8, rew=1e-9)
        rec["first_exceed_bound"] = {k: tj.first_exceed(cv[k], b) for k, b in bound.items()}
        rec["first_exceed_1e-6"] = {k: tj.first_exceed(cv[k], 1e-6 if k != "vel" else 1e-5) for k in bound}
        rec["max"] = {k: float(v.max()) for k, v in cv.items()}
        rec["at"] = {str(s): {k: float(cv[k][s]) for k in cv} for s in (9, 19, 29, 59, 119, 241, steps - 1)}
        out[f"{name}_fp{prec * 8}"] = rec
        print(name, prec * 8, json.dumps(rec), f"{time.time() - t0:.1f}s", flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "tolerance_curves.json"), "w") as f:
    json.dump(out, f, indent=1)
