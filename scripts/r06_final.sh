#!/bin/bash
# Round 6 closing evidence on one box: the whole -m gpu suite, smoke(), the
# default bench line; each step under its own limit, stopping at the first
# failure.  STEPS selects a subset ("tests smoke bench").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06}
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
      rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 1000 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
      rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
exit 0
