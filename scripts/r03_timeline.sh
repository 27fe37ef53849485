#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tl}
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --mappo-iters 1 --configs 0 --pyb 0 --mappo-t32 0 --mappo-steps 32 ${BENCH_EXTRA:-} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rc=$rc"
f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python3 scripts/mappo_timeline2.py "$f" > gpurun_out/${TAG}_timeline.txt; cat gpurun_out/${TAG}_timeline.txt
rm -rf gpurun_out/prof_${TAG}
