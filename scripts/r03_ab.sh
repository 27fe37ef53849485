#!/bin/bash
# A/B of bench variants on one box: each VARIANT_n env string is extra bench.py args.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
i=0
for v in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 $v > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -3 gpurun_out/${TAG}_$i.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); m=d['mappo']
print('[$v]', 'MAPPO %.4g' % m['value'], 'update %.1f' % m['phase_ms']['update'], 'learner %.4f' % m['learner_roofline']['frac'])"
  i=$((i+1))
done
