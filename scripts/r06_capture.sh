#!/bin/bash
# graph captures right after eager all-reduces (world-1 RCCL),
# the captured all-reduce on the capture group (product) and on the default group
# (round 5's hazard, no drain) — QS_CAPTURE_K minibatches per capture window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
N=${N:-10}
timeout -k 10 300 python -u scripts/capture_probe.py capture $N > gpurun_out/cap_probe_capture.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/cap_probe_capture.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/capture_probe.py default $N > gpurun_out/cap_probe_default.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/cap_probe_default.log | tail -4; echo "default rc=$rc"
exit 0
