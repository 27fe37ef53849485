#!/bin/bash
# Round-end evidence on one GPU box: every -m gpu test, the staggered-reset probe,
# then scripts/gpu_prof.sh (bench, kernel-trace stats, PMC traffic) and the MAPPO
# kernel split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/stagger_probe.sh || exit 1
TAG=$TAG LEARNER_TESTS=0 bash scripts/gpu_prof.sh || exit 1
rm -f gpurun_out/prof_${TAG}/*trace*.csv gpurun_out/pmc*_${TAG}/*trace*.csv
TAG=${TAG}m bash scripts/prof_mappo.sh
