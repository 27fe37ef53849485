#!/bin/bash
# The whole -m gpu suite, one process, per-test timeout; log under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03s}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/${TAG}_suite.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/${TAG}_suite.log | tail -15; exit $rc
