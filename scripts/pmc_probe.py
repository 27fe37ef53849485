"""Workload for rocprofv3 --pmc passes: a known-byte calibration copy with the step
kernel's access width (one dword per lane), then the bench's C3 step kernel.
Counters are read back by scripts/pmc_report.py."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
import torch  # noqa: E402
from gym_pybullet_drones_amd import _lib as L  # noqa: E402
from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout  # noqa: E402

N_CAL = 1 << 26   # 256 MiB each way: larger than the 256 MiB Infinity Cache together
E, D, STEPS = int(os.environ.get("PMC_ENVS", 16384)), 8, 20
PREC = int(os.environ.get("PMC_PRECISION", 4))   # 8: the fp64 headline leg's step_kernel<double, ...>
torch.cuda.set_device(0)
lib = L.load()
src = torch.rand(N_CAL, device="cuda")
dst = torch.empty_like(src)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(3):
    L.check(lib.qs_calib_copy(L.ptr(dst), L.ptr(src), N_CAL, st), "calib")
sw = QuadSwarm("multihover", num_envs=E, num_drones=D, act="one_d_pid", precision=PREC, initial_xyzs=grid_layout(D))
slots = 8
obs = torch.empty((slots, E, D, sw.obs_dim), device="cuda")
act = torch.empty((slots, E, D, sw.act_dim), device="cuda")
rew = torch.empty((slots, E), dtype=sw.reward.dtype, device="cuda")
te = torch.empty((slots, E), dtype=torch.uint8, device="cuda")
tr = torch.empty((slots, E), dtype=torch.uint8, device="cuda")
sw.reset(0, obs=obs[0])
for t in range(10 + STEPS):
    k = t % slots
    sw.step(None, obs=obs[k], reward=rew[k], terminated=te[k], truncated=tr[k], actions_out=act[k])
torch.cuda.synchronize()
print("calib bytes each way", N_CAL * 4, "agents", E * D, "precision", PREC)
