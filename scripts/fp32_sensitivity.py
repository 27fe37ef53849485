"""fp32 sensitivity horizons of the reference's own closed loop (CPU, oracle only).

For each config: the fp64 oracle (the reference's precision) against
  * 'once'  : the same run with its state rounded once to fp32 at control step k0;
  * 'fp32'  : the oracle's fp32 instantiation (IEEE division / sqrt, libm expf, no
              contraction: an exact fp32 restatement, none of the kernel's
              approximations) from the same reset draws and Philox actions.
Prints the first control step at which each field passes its fp32 bound (None:
never within the window).  Used to size FP32_HORIZON / FREE_HORIZON_FP32
(DESIGN.md §2): a kernel horizon at or above the 'fp32' one is intrinsic to the
loop, not added by the kernel.
  python scripts/fp32_sensitivity.py [E] [steps] [k0]
"""
import json
import sys
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..", "tests"),
                os.path.join(HERE, "..", "marl-gym-pybullet-drones_amd")]
import qs_oracle  # noqa: E402

BOUND = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)


def grid(D):
    cols = int(np.ceil(np.sqrt(D)))
    rows = int(np.ceil(D / cols))
    return [[(i % cols - (cols - 1) / 2), (i // cols - (rows - 1) / 2), 0.5] for i in range(D)]


G4, G8, G16 = grid(4), grid(8), grid(16)
CFGS = {
    "C3v": dict(task="multihover", num_drones=8, act="vel", initial_xyzs=G8),
    "C4": dict(task="spiral", num_drones=5, act="vel"),
    "C4p": dict(task="spiral", num_drones=5, act="vel", physics="pyb"),
    "C5": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, physics="pyb", aux=("dw",)),
    "C5dyn": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, aux=("dw",)),
    "mh_dw_d8": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8, aux=("dw",)),
    "pyb_dw_d4": dict(task="multihover", num_drones=4, act="one_d_pid", physics="pyb", aux=("dw",)),
    "mh_gnd_drag_d4": dict(task="multihover", num_drones=4, act="one_d_pid", aux=("gnd", "drag", "dw")),
    "pyb_gnd_drag_dw_d4": dict(task="multihover", num_drones=4, act="one_d_pid", physics="pyb",
                               aux=("gnd", "drag", "dw")),
    "meetup_vel_d4": dict(task="meetup", num_drones=4, act="vel"),
    "C3": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8),
    "C2": dict(task="multihover", num_drones=4, act="rpm"),
}


def curves(cfg, mode, E=64, steps=60, k0=0, seed=11):
    a = qs_oracle.OracleSim(num_envs=E, precision=8, **cfg)
    b = qs_oracle.OracleSim(num_envs=E, precision=4 if mode == "fp32" else 8, **cfg)
    a.reset(seed)
    b.reset(seed)
    out = {k: np.zeros(steps) for k in BOUND}
    for t in range(steps):
        if mode == "once" and t == k0:
            b.set_state(0, b.get_state(0).astype(np.float32).astype(np.float64))
        ra, rb = a.step(None), b.step(None)
        sa, sb = a.get_state(0).astype(np.float64), b.get_state(0).astype(np.float64)
        for k, sl in (("pos", slice(0, 3)), ("quat", slice(3, 7)), ("vel", slice(7, 10))):
            out[k][t] = np.abs(sa[sl] - sb[sl]).max()
        out["rew"][t] = np.abs(np.asarray(ra["reward"], np.float64) - np.asarray(rb["reward"], np.float64)).max()
    a.close()
    b.close()
    return out


def first_exceed(c, b):
    i = np.nonzero(c > b)[0]
    return int(i[0]) + 1 if len(i) else None


if __name__ == "__main__":
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    k0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    names = sys.argv[4].split(",") if len(sys.argv) > 4 else list(CFGS)
    res = {}
    for n in names:
        res[n] = {}
        for mode in ("once", "fp32"):
            cv = curves(CFGS[n], mode, E, steps, k0)
            res[n][mode] = {k: first_exceed(cv[k], BOUND[k]) for k in BOUND}
        print(n, json.dumps(res[n]), flush=True)
    print(json.dumps(dict(E=E, steps=steps, k0=k0, seed=11, first_exceed=res)))
