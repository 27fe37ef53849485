#!/bin/bash
# Dev: C2 reset-search sizes (dev builds of build_dev_step.sh) under rocprofv3 kernel stats,
# then the learner's dW2 split-K chunking A/B on the bench's MAPPO leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in p2base p4 p4g64 p1 p2base; do
  QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v_$v -o run --output-format csv -- python3 scripts/c2_probe.py --steps 150 > gpurun_out/v_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python3 - <<PY
import csv
rows = {r["Name"][:40]: r for r in csv.DictReader(open("gpurun_out/prof_v_$v/run_kernel_stats.csv")) if "qs::" in r["Name"]}
tot = 0
for k, r in rows.items():
    if "reset_search" in k or "step_kernel" in k:
        print("$v", k, "avg", round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
  rm -f gpurun_out/prof_v_$v/*trace*.csv
done
for v in "" "--splitk 32768x256=1024" ""; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 --mappo-configs "" $v > gpurun_out/abk.json 2> gpurun_out/abk.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc [$v]"; tail -3 gpurun_out/abk.err; exit $rc; }
  python3 -c "
import json; m=json.load(open('gpurun_out/abk.json'))['mappo']; print('[$v]', round(m['value']), round(m['ms_per_train_step'], 1), round(m['learner_roofline']['frac'], 4))"
done
