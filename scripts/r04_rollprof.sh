#!/bin/bash
# Kernel timeline of one rollout control step of a MAPPO trainer config
# (LEG=C4 default: Spiral, VEL, norm_obs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-rp}; LEG=${LEG:-C4}; PAT=${PAT:-step_kernel<float, 1,}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --mappo-iters 1 --configs 0 --pyb 0 --fp64 0 --mappo-t32 0 \
  --mappo-configs $LEG ${BENCH_EXTRA:-} > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_${TAG}.log; exit $rc; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python3 scripts/rollout_timeline.py "$f" "$PAT" > gpurun_out/${TAG}_timeline.txt
tail -16 gpurun_out/${TAG}_timeline.txt
# the headline C3 trainer leg's rollout step (always in the bench's MAPPO legs)
python3 scripts/rollout_timeline.py "$f" "step_kernel<float, 0, 4, 30, 1, 0>" > gpurun_out/${TAG}_timeline_c3.txt
tail -14 gpurun_out/${TAG}_timeline_c3.txt
rm -rf gpurun_out/prof_${TAG}
