#!/bin/bash
# Kernel-trace stats of the full-MAPPO bench leg (which kernels the PPO update spends its time in).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-mappo}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --mappo-iters 1 > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rc=$rc"
python3 - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_${TAG}/run_kernel_stats.csv")))
tot=sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {float(r["Percentage"]):6.2f}% {int(r["Calls"]):8d} {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}')
print("total ms", tot/1e6)
PY
rm -f gpurun_out/prof_${TAG}/run_kernel_trace.csv
