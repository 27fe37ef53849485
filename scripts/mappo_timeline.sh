#!/bin/bash
# Kernel timeline of one PPO minibatch iteration (last graph replay of scripts/mappo_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 scripts/mappo_timeline.py > gpurun_out/tl.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/tl.log; exit $rc; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/tl/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/tl/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last replay: kernels after the last adam_commit but one
ends = [i for i, r in enumerate(rows) if "adam_commit" in r["Kernel_Name"]]
a, b = ends[-3] + 1, ends[-1] + 1
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{s/1e3:8.1f} {e/1e3:8.1f} {(e-s)/1e3:7.1f}  q{r.get("Queue_Id","?"):>3} {r["Kernel_Name"][:90]}')
PY
rm -f gpurun_out/tl/*kernel_trace.csv
