#!/bin/bash
# Round-4 closing call: the whole -m gpu suite + the default bench line (evidence part A), smoke(), C4 learner variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PART=A TAG=r04g bash scripts/r04_evidence.sh > gpurun_out/r04g_A.txt 2>&1; rc=$?; cat gpurun_out/r04g_A.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04g_smoke.txt 2>&1; rc=$?; tail -2 gpurun_out/r04g_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/learner_mb.py C4v > gpurun_out/r04g_c4v.txt 2>&1; cat gpurun_out/r04g_c4v.txt
