"""Generate tests/golden/oracle_golden.npz from the CPU oracle (fp64).

The reference itself cannot be executed here, so these vectors
pin the restatement against regressions and are replayed by the HIP kernel in
tests/test_gpu_golden.py.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "marl-gym-pybullet-drones_amd")]
import qs_oracle  # noqa: E402
from gym_pybullet_drones_amd.envs.swarm import grid_layout  # noqa: E402

CASES = {
    "mh_rpm_d4": dict(task="multihover", num_drones=4, act="rpm"),
    "mh_onedpid_d8": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=grid_layout(8)),
    "mh_vel_d3": dict(task="multihover", num_drones=3, act="vel"),
    "spiral_vel_d5": dict(task="spiral", num_drones=5, act="vel"),
    "mh_dw_d16": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=grid_layout(16), aux=("dw",)),
    "mh_onedpid_d8_pyb": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=grid_layout(8),
                              physics="pyb"),
}
E, STEPS, SEED = 3, 40, 123


def generate():
    out = {}
    for name, kw in CASES.items():
        s = qs_oracle.OracleSim(num_envs=E, precision=8, **kw)
        out[f"{name}/obs0"] = s.reset(SEED)
        obs, rew, te, tr, act = [], [], [], [], []
        for _ in range(STEPS):
            r = s.step(None)
            obs.append(r["obs"]); rew.append(r["reward"]); te.append(r["terminated"]); tr.append(r["truncated"])
            act.append(r["actions"])
        out[f"{name}/obs"] = np.stack(obs)
        out[f"{name}/reward"] = np.stack(rew)
        out[f"{name}/terminated"] = np.stack(te)
        out[f"{name}/truncated"] = np.stack(tr)
        out[f"{name}/actions"] = np.stack(act)
        out[f"{name}/state"] = s.get_state(0)
        out[f"{name}/env"] = s.get_state(1)
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **generate())
    print("wrote", os.path.join(HERE, "oracle_golden.npz"))
