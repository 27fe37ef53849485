"""Dev: the kernels of one C3 learner minibatch from a rocprofv3 kernel trace of
`scripts/learner_mb.py one` (graph replays of the default iteration): the window
between two consecutive fused-actor launches, each kernel's start / end relative to
it, the device-busy union and the idle gaps (no kernel running) inside it.  The
profiler serialises some of the two streams' overlap, so durations here are an
upper bound on what the graph replay spends."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "mlp3f_actor_kernel" in r["Kernel_Name"]]
periods = sorted(zip(idx[:-1], idx[1:]), key=lambda ab: int(rows[ab[1]]["Start_Timestamp"]) - int(rows[ab[0]]["Start_Timestamp"]))
a, b = periods[len(periods) // 2]   # the median minibatch
t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
iv = []
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    iv.append((s, e))
    print(f"{s / 1e3:8.2f} {e / 1e3:8.2f} {(e - s) / 1e3:7.2f}  {r['Kernel_Name'][:100]}")
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e in sorted(iv):
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((cur_e, s))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
if cur_e < t1 - t0:
    gaps.append((cur_e, t1 - t0))
print(f"minibatch period {(t1 - t0) / 1e3:.2f} us, {b - a} kernels, device busy {busy / 1e3:.2f} us, "
      f"idle {sum(g[1] - g[0] for g in gaps) / 1e3:.2f} us in {len(gaps)} gaps:")
for g0, g1 in gaps:
    print(f"   idle {g0 / 1e3:8.2f} .. {g1 / 1e3:8.2f}  ({(g1 - g0) / 1e3:.2f} us)")
