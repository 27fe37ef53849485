#!/bin/bash
# Horizon comparison (kernel vs exact-fp32 oracle over seeds) + the tolerance / free-running tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/learner_kbench.py sumadam 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python3 -u scripts/horizon_compare.py 64 60 11,12,13,14,15,16,17,18 gpurun_out/r03_horizons.json > gpurun_out/r03_hz.log 2>&1
rc=$?; cat gpurun_out/r03_hz.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_tolerance.py tests/test_gpu_parity.py -k "tolerance or free_running or full_size" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_tol.log 2>&1
rc=$?; tail -15 gpurun_out/r03_tol.log; exit $rc
