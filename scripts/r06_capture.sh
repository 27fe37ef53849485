#!/bin/bash
# graph captures right after eager all-reduces issued on the
# graphs' own capture stream (world-1 RCCL): the product path (mappo/collectives.py),
# then (DEFAULT=1, last: an abort is the expected outcome) round 5's pattern
# without its drain.  QS_CAPTURE_K minibatches per capture window.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
N=${N:-10}
timeout -k 10 300 python -u scripts/capture_probe.py capture $N > gpurun_out/cap_probe_capture.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/cap_probe_capture.log | tail -3; [ $rc -eq 0 ] || exit $rc
if [ "${DEFAULT:-0}" = "1" ]; then
  timeout -k 10 300 python -u scripts/capture_probe.py default $N > gpurun_out/cap_probe_default.log 2>&1; rc=$?
  grep -v amdgpu gpurun_out/cap_probe_default.log | grep -E "capture|hipError|terminate" | head -6; echo "default rc=$rc"
fi
exit 0
