"""Dev: phase timestamps of the small-path tile kernel (ppo_small_fb_kernel /
the critic tiles) from the QS_TILE_STAMPS dev build (s_memrealtime, 100 MHz,
thread 0 of each workgroup):
  0 entry  1 loads issued + X tile staged  2 layer 1 done  3 layer 2 + head partials
  4 loss head / dZ2  5 dH1 contraction + stores  6 arrival counted  7 last tile's loss sums
  bash scripts/build_dev_step.sh tstamps -DQS_TILE_STAMPS
  QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_tstamps.so python scripts/tile_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402
import learner_mb  # noqa: E402


def dump(label, nwg, nA=None):
    lib = L.load()
    buf = (ctypes.c_ulonglong * (nwg * 8))()
    f = lib.qs_dev_tile_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert f(buf, nwg * 8) == 0
    s = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.int64)
    t0 = s[:, 0].min()
    rel = (s - t0) * 0.01   # µs
    print(f"== {label}: {nwg} workgroups; entry spread {rel[:, 0].min():.2f} .. {rel[:, 0].max():.2f} us")
    names = ["entry", "staged", "layer1", "layer2+head", "loss/dZ2", "dH1", "arrived"]
    for k in range(1, 7):
        d = rel[:, k] - rel[:, k - 1]
        print(f"  {names[k - 1]:>12s} -> {names[k]:<12s} median {np.median(d):7.2f} us  max {d.max():7.2f} us")
    if nA is not None and 0 < nA < nwg:   # the actor's and the critic's tiles apart
        for nm, sl in (("actor", slice(0, nA)), ("critic", slice(nA, nwg))):
            r = rel[sl]   # (stamp 5, dH1 done: the tiles' last phase since the per-tile tail moved to launch 2)
            ph = "  ".join(f"{np.median(r[:, k] - r[:, k - 1]):6.2f}" for k in range(1, 6))
            print(f"  {nm:>6s} tiles: phases 1-5 median [{ph}] us; entry .. dH1 max {np.max(r[:, 5] - r[:, 0]):7.2f} us; "
                  f"last {r[:, 5].max():.2f} us")
    if os.environ.get("QS_STAMPS2"):   # the QS_TILE_STAMPS2 build: 6 = layer 1 issued, 7 = H1 stored
        for nm, sl in (("actor", slice(0, nA)), ("critic", slice(nA, nwg))) if nA else (("all", slice(0, nwg)),):
            r = rel[sl]
            print(f"  {nm:>6s} layer 1: staged -> MFMAs issued {np.median(r[:, 6] - r[:, 1]):6.2f}  -> H1 stored "
                  f"{np.median(r[:, 7] - r[:, 6]):6.2f}  -> barrier {np.median(r[:, 2] - r[:, 7]):6.2f} us")
        return
    last = rel[:, 7][s[:, 7] > 0]
    print(f"  arrivals end {rel[:, 6].max():.2f} us; last tile done at {last.max() if len(last) else float('nan'):.2f} us")


def main():
    torch.cuda.init()
    if len(sys.argv) > 1:   # per-rank shapes (scripts/learner_mb.py RANK_SHAPES) on the tile path
        from gym_pybullet_drones_amd.mappo import agent as agent_mod
        agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
        for shape in sys.argv[1:]:
            learner_mb.per_minibatch_us(shape, reps=1, small=True)
            torch.cuda.synchronize()
            D, O, A, mb, T, E = learner_mb.SHAPES[shape]
            t16, t32 = (mb * D + 15) // 16 + (mb + 15) // 16, (mb * D + 31) // 32 + (mb + 31) // 32
            rb = (3 if t32 > 256 and O <= 256 and (D * O <= 256 or (mb * D + 47) // 48 + (mb + 15) // 16 <= 256)
                  else 2) if (A == 1 and t16 > 256) else (
                2 if A > 1 and t16 > 256 and O <= 256 and (mb * D + 31) // 32 + (mb + 15) // 16 <= 256 else 1)
            # (ppo_small.hip s_layout)
            nA = (mb * D + 16 * rb - 1) // (16 * rb)
            rbc = 1 if rb > 1 and nA + (mb + 15) // 16 <= 256 else rb   # (ppo_small.hip s_layout)
            nC = (mb + 16 * rbc - 1) // (16 * rbc)
            dump(f"{shape} tile path ({16 * rb}/{16 * rbc}-row tiles) (actor tiles {nA}, critic tiles {nC})", nA + nC, nA)
        return
    for name, shape in (("ref small step", "ref"),):
        learner_mb.per_minibatch_us(shape, reps=1, small=True)
        torch.cuda.synchronize()
        D, O, A, mb, T, E = learner_mb.SHAPES[shape]
        nA, nC = (mb * D + 15) // 16, (mb + 15) // 16
        dump(f"{name} (actor tiles {nA}, critic tiles {nC})", nA + nC)
    for mb in (256, 4096):
        learner_mb.kernels(mb)
        torch.cuda.synchronize()
        dump(f"critic tiles at {mb} rows", (mb + 15) // 16)


if __name__ == "__main__":
    main()
