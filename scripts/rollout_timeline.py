"""Dev: the kernels of one rollout control step from a rocprofv3 kernel trace:
everything between two consecutive launches of the step kernel whose name
contains argv[2] (e.g. 'step_kernel<float, 1,'), taken from the middle of the
trace, with the step's total device time and the time per kernel family."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = sys.argv[2] if len(sys.argv) > 2 else "step_kernel"
idx = [i for i, r in enumerate(rows) if pat in r["Kernel_Name"]]
# consecutive launches inside one rollout: the pair with the median period (a
# pair that straddles a PPO update is far longer)
pairs = sorted(zip(idx[:-1], idx[1:]), key=lambda ab: int(rows[ab[1]]["Start_Timestamp"]) - int(rows[ab[0]]["Start_Timestamp"]))
a, b = pairs[len(pairs) // 4]
t0 = int(rows[a]["Start_Timestamp"])
fam = collections.defaultdict(float)
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    fam[r["Kernel_Name"][:60]] += (e - s) / 1e3
    print(f"{s / 1e3:8.2f} {e / 1e3:8.2f} {(e - s) / 1e3:7.2f}  {r['Kernel_Name'][:90]}")
print(f"step period {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.2f} us, kernels {b - a}")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v:8.2f} us  {k}")
