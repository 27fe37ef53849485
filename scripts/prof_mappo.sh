#!/bin/bash
# Kernel-trace stats of the full-MAPPO bench leg (which kernels the PPO update spends its time in).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-mappo}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --mappo-iters 1 --configs 0 --pyb 0 --mappo-t32 0 ${BENCH_EXTRA:-} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rc=$rc"
python3 - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_${TAG}/run_kernel_stats.csv")))
tot=sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):6.2f}% {int(r["Calls"]):8d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}')
print("total ms", tot/1e6)
# the fused MLP kernels by launch size (minibatch vs rollout inference)
import collections
agg=collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/prof_${TAG}/run_kernel_trace.csv")):
    if "mlp3" in r["Kernel_Name"]:
        agg[(r["Kernel_Name"][:48], r.get("Grid_Size_X", r.get("Grid_Size")))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (k, g), v in sorted(agg.items()):
    print(f"{k:48s} grid {g:>8s} calls {len(v):6d} avg {sum(v)/len(v)/1e3:9.2f} us")
PY
rm -f gpurun_out/prof_${TAG}/run_kernel_trace.csv
