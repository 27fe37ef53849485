#!/bin/bash
# Round 6 iteration on one box: the tile path's GPU tests, then the per-rank
# tile-path timing of this build and (AB=1) of the baseline build abso/base.so
# in the same call, then (PROF=1) a kernel trace of one shape.  Stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-it}
PT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
if [ -n "${TESTS-tests/test_gpu_small_multirank.py tests/test_gpu_learner.py}" ]; then
  timeout -k 10 600 $PT ${TESTS:-tests/test_gpu_small_multirank.py tests/test_gpu_learner.py} -k "${TESTK:-small or gate or allreduce}" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROBE-tiles}" ]; then
  timeout -k 10 400 python3 -u scripts/learner_mb.py ${PROBE:-tiles} > gpurun_out/${TAG}_probe.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_probe.log; [ $rc -eq 0 ] || exit $rc
  if [ "${AB:-0}" = "1" ]; then
    QS_DEV_LIB=$PWD/abso/base.so timeout -k 10 400 python3 -u scripts/learner_mb.py ${PROBE:-tiles} > gpurun_out/${TAG}_probe_base.log 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_probe_base.log; [ $rc -eq 0 ] || exit $rc
  fi
fi
if [ -n "${PROF:-}" ]; then
  n=$(echo $PROF | tr '/' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$n -o run --output-format csv -- \
    python3 scripts/learner_mb.py shape:$PROF > gpurun_out/${TAG}_prof_$n.log 2>&1
  rc=$?; grep minibatch gpurun_out/${TAG}_prof_$n.log; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/${TAG}_prof_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:12]: print('$PROF', r['Calls'].rjust(7), ('%9.2f' % (float(r['AverageNs'])/1e3)), 'us avg', r['Name'][:110])"
fi
if [ "${FULL:-0}" = "1" ]; then
  timeout -k 10 900 $PT tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
