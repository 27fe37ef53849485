#!/bin/bash
# Round 4 learner probe, one box: isolated kernel times (learner_kbench), the MAPPO
# T=32 leg with one / two streams, and a kernel-trace timeline of a few minibatches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-lp}
timeout -k 10 240 python3 -u scripts/learner_kbench.py > gpurun_out/${TAG}_kbench.txt 2>&1 || { echo "kbench rc=$?"; tail -5 gpurun_out/${TAG}_kbench.txt; exit 1; }
cat gpurun_out/${TAG}_kbench.txt
for v in "--side-stream 1" "--side-stream 0" "--side-stream 0 --w1-stream 0"; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-steps 32 --mappo-t32 0 --mappo-configs "" $v > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc [$v]"; tail -3 gpurun_out/${TAG}.err; exit $rc; }
  python3 -c "
import json; m=json.load(open('gpurun_out/${TAG}.json'))['mappo']; print('[$v]', round(m['value']), round(m['ms_per_train_step'], 1), m['phase_ms'], round(m['learner_roofline']['frac'], 4), 'us/mb', round(m['phase_ms']['update']*1e3/1280, 1))"
done
for v in "--side-stream 1" "--side-stream 0"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --mappo-iters 1 --configs 0 --pyb 0 --mappo-t32 0 --mappo-configs "" --mappo-steps 32 $v > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "prof rc=$rc"; tail -3 gpurun_out/prof_${TAG}.log; exit $rc; }
  f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
  echo "==== timeline [$v]"
  python3 scripts/mappo_timeline2.py "$f"
  rm -rf gpurun_out/prof_${TAG}
done
