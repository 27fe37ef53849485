"""fp32 horizons of the kernel against those of an exact fp32 restatement.

For each sensitive config and seed: the first control step (0-based index) at
which the fp32 HIP kernel, and the oracle's own fp32 instantiation (IEEE
division / sqrt, libm transcendentals), depart from the fp64 oracle past the
fp32 bounds, from the same reset draws and Philox actions (tests/trajectory.py
diverge, identical tie handling).  The oracle side is the reference's own
sensitivity to fp32 rounding; a kernel horizon that matches it is intrinsic to
the closed loop, not added by the kernel.  GPU script (test infrastructure).
  python scripts/horizon_compare.py [E] [steps] [seeds] [out.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import trajectory as tj  # noqa: E402
from gym_pybullet_drones_amd.envs.swarm import grid_layout  # noqa: E402

G8, G16 = grid_layout(8).tolist(), grid_layout(16).tolist()
CFGS = {
    "C3v": dict(task="multihover", num_drones=8, act="vel", initial_xyzs=G8),
    "C4": dict(task="spiral", num_drones=5, act="vel"),
    "C5": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, physics="pyb", aux=("dw",)),
    "C5d": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, aux=("dw",)),
    "mh_gnd_drag_d4": dict(task="multihover", num_drones=4, act="one_d_pid", aux=("gnd", "drag", "dw")),
    "pyb_gnd_drag_dw_d4": dict(task="multihover", num_drones=4, act="one_d_pid", physics="pyb",
                               aux=("gnd", "drag", "dw")),
}
BOUND = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)

if __name__ == "__main__":
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    seeds = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(11, 19))
    out_path = sys.argv[4] if len(sys.argv) > 4 else None
    res = dict(E=E, steps=steps, seeds=seeds, bound=BOUND, configs={})
    for name, cfg in CFGS.items():
        rec = {}
        for subj in ("kernel", "oracle"):
            rec[subj] = {k: [] for k in BOUND}
            for sd in seeds:
                r = tj.diverge(cfg, E=E, precision=4, steps=steps, seed=sd, subject=subj)
                for k, b in BOUND.items():
                    rec[subj][k].append(tj.first_exceed(r["curves"][k], b))
        rec["mean"] = {s: {k: float(np.mean(v)) for k, v in rec[s].items()} for s in ("kernel", "oracle")}
        rec["kernel_minus_oracle"] = {k: [a - b for a, b in zip(rec["kernel"][k], rec["oracle"][k])] for k in BOUND}
        res["configs"][name] = rec
        print(name, json.dumps(rec["mean"]), "kernel-oracle per seed:", json.dumps(rec["kernel_minus_oracle"]),
              flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)
