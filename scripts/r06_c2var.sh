#!/bin/bash
# Dev probe: C2 kernel times (rocprofv3 --stats of scripts/c2_probe.py) for reset-helper
# variants (dev libraries lib_h<helpers per CU>c<chunks>.so, -DQS_HELP_PER_CU / -DQS_HELP_CHUNKS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARS:-h3c2 h3c3 h3c1}; do
  QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2v_$v -o run --output-format csv -- python3 scripts/c2_probe.py --steps 200 > gpurun_out/c2v_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/c2v_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v $(grep 'C2 probe' gpurun_out/c2v_$v.log)"
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:2]: print(r['Calls'].rjust(7), ('%9.2f' % (float(r['AverageNs'])/1e3)), 'us avg', ('%9.2f' % (float(r['MaxNs'])/1e3)), 'max', r['Name'][:70])"
done
