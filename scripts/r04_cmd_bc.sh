#!/bin/bash
# Round-4 evidence parts B and C in one call (scripts/r04_evidence.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PART=B TAG=r04 bash scripts/r04_evidence.sh > gpurun_out/r04_B.txt 2>&1; rc=$?; cat gpurun_out/r04_B.txt; [ $rc -eq 0 ] || exit $rc
PART=C TAG=r04 bash scripts/r04_evidence.sh > gpurun_out/r04_C.txt 2>&1; rc=$?; cat gpurun_out/r04_C.txt; exit $rc
