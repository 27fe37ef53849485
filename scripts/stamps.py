"""Dev: per-wave phase timestamps of the step kernel (QS_STAMPS=1)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
os.environ["QS_STAMPS"] = "1"
import numpy as np, torch
from gym_pybullet_drones_amd import _lib as L
from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout
from gym_pybullet_drones_amd.utils.enums import Physics
sys.path.insert(0, ROOT)
from bench import stagger_episodes
# config: C3 (default), C5, C4 — python scripts/stamps.py [NAME]  (needs a QS_STAMPS_BUILD library)
CFG = {"C3": ("multihover", 16384, 8, "one_d_pid", Physics.DYN), "C5": ("multihover", 8192, 16, "one_d_pid", Physics.PYB_DW),
       "C4": ("spiral", 8192, 5, "vel", Physics.DYN)}[sys.argv[1] if len(sys.argv) > 1 else "C3"]
task, E, D, actn, phys = CFG
kw = dict(initial_xyzs=grid_layout(D)) if task == "multihover" else {}
sw = QuadSwarm(task, num_envs=E, num_drones=D, act=actn, precision=4, physics=phys, **kw)
obs = torch.empty((E, D, sw.obs_dim), device="cuda"); act = torch.empty((E, D, sw.act_dim), device="cuda")
sw.reset(0, obs=obs)
stagger_episodes(sw, task)
for t in range(20):
    sw.step(None, obs=obs, actions_out=act)
torch.cuda.synchronize()
G = -(-E // (64 // D))
buf = np.zeros(G * 8, np.uint64)
lib = L.load(); lib.qs_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
L.check(lib.qs_debug_stamps(sw._h, buf.ctypes.data_as(ctypes.c_void_p), G * 8), "stamps")
st = buf.reshape(G, 8).astype(np.float64) * 10e-3   # 100 MHz → µs
t0 = st[:, 0].min()
names = ["start", "loads used", "action/pid done", "substeps done", "reward/reset done", "obs waited", "obs stored"]
print("phase (µs, relative to first wave start): p10 / median / p90")
for k in range(7):
    v = st[:, k] - t0
    print(f"{names[k]:20s} {np.percentile(v,10):7.2f} {np.median(v):7.2f} {np.percentile(v,90):7.2f}")
d = np.diff(st[:, :7], axis=1)
print("per-wave phase durations median:", np.round(np.median(d, axis=0), 2))
print("last wave obs stored at %.2f us; waves started by: p50 %.2f, max %.2f" % (
    (st[:, 6] - t0).max(), np.median(st[:, 0] - t0), (st[:, 0] - t0).max()))
# how many waves are in each phase over time (0.5 us bins)
bins = np.arange(0, (st[:, 6] - t0).max() + 0.5, 0.5)
for b in bins:
    ph = [(((st[:, k] - t0) <= b) & ((st[:, k + 1] - t0) > b)).sum() for k in range(6)]
    print(f"t={b:5.1f}  " + " ".join(f"{n:5d}" for n in ph))
