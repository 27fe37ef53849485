#!/bin/bash
# One GPU session: parity tests → bench → rocprofv3 kernel-trace summary.
# Stops at the first GPU fault/abort/timeout (exit 124/134/137/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
TAG=${TAG:-r01}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_${TAG}.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err
if fatal $rc; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_${TAG}.log
  find gpurun_out/prof_${TAG} -name "*stats*" | head
  rm -f gpurun_out/prof_${TAG}/*trace*.csv
fi
exit 0
