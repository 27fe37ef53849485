#!/bin/bash
# Round 6, C2 (MultiHover 4 drones x 4 096 envs, RPM, DYN): the reset-search tests,
# a short bench line (the configs legs), and a kernel trace of the C2 probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-c2}
PT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
if [ -n "${TESTS-tests/test_gpu_parity.py tests/test_reset_distribution.py}" ]; then
  timeout -k 10 900 $PT ${TESTS:-tests/test_gpu_parity.py tests/test_reset_distribution.py} -k "${TESTK:-reset or deferred or reseed or mh}" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --mappo 0 --pyb 0 --fp64 0 --rank-shapes '' > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['roofline']['frac'])
for k,v in d.get('configs',{}).items(): print(k, v.get('value'), v.get('roofline',{}).get('frac'), v.get('kernel_ms'), v.get('ms_per_step'))
"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 scripts/c2_probe.py --steps 200 > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; grep "C2 probe" gpurun_out/${TAG}_prof.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:6]: print(r['Calls'].rjust(7), ('%9.2f' % (float(r['AverageNs'])/1e3)), 'us avg', ('%9.2f' % (float(r['MaxNs'])/1e3)), 'max', r['Name'][:90])"
