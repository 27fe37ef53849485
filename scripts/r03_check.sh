#!/bin/bash
# Round-3 GPU check: the new T8 / learner / surfaces tests, then the MAPPO kernel
# split with the critic on the main stream (per-kernel durations not inflated by
# the second stream).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_train_step.py tests/test_gpu_learner.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r03_tests.log; [ $rc -eq 0 ] || exit $rc
[ "${PROF:-1}" = "1" ] || exit 0
TAG=r03m1 BENCH_EXTRA="--side-stream 0" bash scripts/prof_mappo.sh
