"""Dev: per-workgroup phase timestamps of the tile path's weight-gradient launch
(ppo_small_wgrad_kernel) from the QS_TILE_STAMPS dev build (s_memrealtime, 100 MHz,
thread 0): 0 entry, 1 wave 0's contraction done (the LDS ring drained),
2 the KL gate read, 3 done (sink written).
  bash scripts/build_dev_step.sh tstamps -DQS_TILE_STAMPS
  QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_tstamps.so python scripts/wgrad_stamps.py C3/8 ..."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402
from gym_pybullet_drones_amd.mappo import agent as agent_mod  # noqa: E402
import learner_mb  # noqa: E402


def gtiles(I):   # 64×64 tiles per net: W2's 4×4, then W1's 4×⌈I/64⌉ (ppo_small.hip s_gtiles)
    return 16 + 4 * ((I + 63) // 64)


def main():
    torch.cuda.init()
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
    for shape in sys.argv[1:] or ["C3/8"]:
        learner_mb.per_minibatch_us(shape, reps=1, small=True)
        torch.cuda.synchronize()
        D, O, A, mb, T, E = learner_mb.SHAPES[shape]
        off = (ctypes.c_int64 * L.QS_PPO_SMALL_LAYOUT_N)()
        assert L.load().qs_ppo_small_layout(mb, D, O, D * O, A, off, len(off)) == 0
        Sa, Sc = off[27], off[28]
        na, nc = gtiles(O) * Sa, gtiles(D * O) * Sc
        nvec = (2 * 256 + A * 256 + 2 * A) + (3 * 256 + 1)
        nv = (16 * nvec + 255) // 256   # kSGW = 4 waves
        n = na + nc + nv
        buf = (ctypes.c_ulonglong * (n * 4))()
        f = L.load().qs_dev_wgrad_stamps
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        assert f(buf, n * 4) == 0
        s = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
        t0 = s[:, 0].min()
        rel = (s - t0) * 0.01
        print(f"== {shape}: actor tile-chunks {na} (S {Sa}), critic tile-chunks {nc} (S {Sc}), vector WGs {nv}")
        for name, sl in (("actor", slice(0, na)), ("critic", slice(na, na + nc)), ("vector", slice(na + nc, n))):
            r = rel[sl]
            line = f"  {name:6s} entry {np.median(r[:, 0]):6.2f} (max {r[:, 0].max():6.2f})"
            if name != "vector":
                line += (f"  contraction {np.median(r[:, 1] - r[:, 0]):6.2f} (max {(r[:, 1] - r[:, 0]).max():6.2f})"
                         f"  gate {np.median(r[:, 2] - r[:, 1]):6.2f}  sink {np.median(r[:, 3] - r[:, 2]):6.2f}")
            line += f"  end {np.median(r[:, 3]):6.2f} (max {r[:, 3].max():6.2f}) us"
            print(line)
        ent = np.sort(rel[:, 0])
        print("  entry quantiles (us):", [round(float(ent[int(q * (n - 1))]), 2) for q in (0, 0.25, 0.5, 0.6, 0.75, 0.9, 1)])


if __name__ == "__main__":
    main()
