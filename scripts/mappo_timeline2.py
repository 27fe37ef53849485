"""Dev: timeline of a few PPO minibatches from a rocprofv3 kernel trace (start/end
of every kernel, relative to the minibatch's first kernel), to read the critical
path of the two-stream update."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "mlp3f_actor" in r["Kernel_Name"] or "mlp3_fwd_kernel<1, true>" in r["Kernel_Name"]]
pick = idx[len(idx) // 2: len(idx) // 2 + 3]
for a, b in zip(pick[:-1], pick[1:]):
    t0 = int(rows[a]["Start_Timestamp"])
    # kernels that start in [a, b) (both streams)
    print("---- minibatch")
    for r in rows[a - 6:b]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:8.2f} {e / 1e3:8.2f} {(e - s) / 1e3:7.2f}  q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3s}  {r['Kernel_Name'][:70]}")
