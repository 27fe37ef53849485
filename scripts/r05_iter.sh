#!/bin/bash
# Round 5 iteration on one box: the tile path's tests (single rank, the forced
# exchange, two gloo ranks), the learner probes, optionally the whole -m gpu
# suite.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-it}
PT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
if [ -n "${TESTS:-tests/test_gpu_small_multirank.py tests/test_gpu_learner.py}" ]; then
  timeout -k 10 600 $PT ${TESTS:-tests/test_gpu_small_multirank.py tests/test_gpu_learner.py} -k "${TESTK:-small or gate or allreduce}" > gpurun_out/${TAG}_new.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_new.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROBE:-ranks ref}" ]; then
  timeout -k 10 400 python3 -u scripts/learner_mb.py ${PROBE:-ranks ref} > gpurun_out/${TAG}_probe.log 2>&1
  rc=$?; cat gpurun_out/${TAG}_probe.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
fi
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 900 $PT tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
