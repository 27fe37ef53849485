"""Dev: the C2 config alone (MultiHover 4-drone x 4096 envs, RPM, DYN, the
reference's diagonal layout, so rejected reset draws go to reset_search_kernel).
Staggered episodes, `--steps` eager steps; run under rocprofv3 --kernel-trace
--stats for per-kernel times, or with a QS_X_RSTATS dev library (QS_DEV_LIB)
for the search kernel's per-workgroup counters."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from gym_pybullet_drones_amd.envs import QuadSwarm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=60)
ap.add_argument("--warmup", type=int, default=10)
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--drones", type=int, default=4)
a = ap.parse_args()
sw = QuadSwarm("multihover", num_envs=a.envs, num_drones=a.drones, act="rpm", precision=4)
sw.reset(0)
bench.stagger_episodes(sw, "multihover")
for _ in range(a.warmup):
    sw.step(None)
torch.cuda.synchronize()
_, e0 = sw.episode_log(cap=0)
t0 = time.perf_counter()
for _ in range(a.steps):
    sw.step(None)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
_, e1 = sw.episode_log(cap=0)
assert sw.reset_error() == 0
print(f"C2 probe: {a.steps} steps, {dt / a.steps * 1e6:.1f} us/step wall (eager), "
      f"{(e1 - e0) / a.steps:.1f} episodes ended per step", flush=True)
sw.close()
