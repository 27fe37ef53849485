#!/bin/bash
# Kernel trace of the tile path at the per-rank shapes (scripts/learner_mb.py shape:NAME).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tp}
for sh in ${SHAPES:-C3/8 ref C5/8}; do
  n=$(echo $sh | tr '/' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$n -o run --output-format csv -- \
    python3 scripts/learner_mb.py shape:$sh > gpurun_out/${TAG}_$n.log 2>&1
  rc=$?; grep minibatch gpurun_out/${TAG}_$n.log; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/${TAG}_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:12]: print('$sh', r['Calls'].rjust(7), ('%9.2f' % (float(r['AverageNs'])/1e3)), 'us avg', r['Name'][:110])"
done
