"""Dev: where the fixed per-window cost of bench.py's sim leg goes (the driver
times 20 control steps): wall time of the timed region's pieces, each the
median of 50 repetitions on the C3 workload (16 384 envs x 8 drones)."""
import os
import statistics
import sys
import time

import torch

if os.environ.get("WP_SPIN"):   # hipDeviceScheduleSpin on torch's own HIP runtime, before its context exists
    import ctypes
    hip = [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l][0]
    assert ctypes.CDLL(hip).hipSetDeviceFlags(1) == 0

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd")]
from gym_pybullet_drones_amd.envs import QuadSwarm, grid_layout  # noqa: E402

torch.cuda.set_device(0)
E, D, K = 16384, 8, int(os.environ.get("STEPS", 20))
sw = QuadSwarm("multihover", num_envs=E, num_drones=D, act="one_d_pid", precision=4, initial_xyzs=grid_layout(D))
obs = torch.empty((K, E, D, sw.obs_dim), device="cuda")
sw.reset(0, obs=obs[0])
for k in range(5):
    sw.step(None, obs=obs[k])
torch.cuda.synchronize()
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for k in range(K):
        sw.step(None, obs=obs[k])
g.replay()
torch.cuda.synchronize()
cur = torch.cuda.current_stream()


def med(fn, n=50):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts)


def events_window():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(cur)
    g.replay()
    b.record(cur)
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    return a, b


ev = []
ev_end = torch.cuda.Event()


def kernel_us():
    a, b = events_window()
    ev.append(a.elapsed_time(b) * 1e3)


print(f"K={K}")
print(f"sync alone                         {med(torch.cuda.synchronize):8.1f} us")
print(f"sync + sync                        {med(lambda: (torch.cuda.synchronize(), torch.cuda.synchronize())):8.1f} us")
print(f"replay + sync                      {med(lambda: (g.replay(), torch.cuda.synchronize())):8.1f} us")
print(f"replay + stream sync               {med(lambda: (g.replay(), cur.synchronize())):8.1f} us")
print(f"events + replay + 2 sync (bench)   {med(events_window):8.1f} us")
print(f"replay + event sync                {med(lambda: (ev_end.record(cur) if g.replay() is None else None, ev_end.synchronize())):8.1f} us")
def spin_window():   # the end of the window noticed by polling the last event, then the device sync
    b = torch.cuda.Event()
    g.replay()
    b.record(cur)
    while not b.query():
        pass
    torch.cuda.synchronize()


print(f"replay + spin on event + sync      {med(spin_window):8.1f} us")
try:   # the graph launched straight through the HIP runtime (torch's replay bookkeeping skipped)
    import ctypes
    hip = ctypes.CDLL([l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l][0])
    ex = ctypes.c_void_p(g.raw_cuda_graph_exec())
    st = ctypes.c_void_p(cur.cuda_stream)
    print(f"hipGraphLaunch + sync              {med(lambda: (hip.hipGraphLaunch(ex, st), torch.cuda.synchronize())):8.1f} us")
except Exception as e:   # (older torch: no raw_cuda_graph_exec)
    print("hipGraphLaunch probe skipped:", e)
med(kernel_us)
print(f"event-timed graph                  {statistics.median(ev):8.1f} us  ({statistics.median(ev) / K:.2f} us/step)")
sw.close()
