#!/bin/bash
# Config-leg kernel times (C2 / C3-VEL / C4 / C5) for the product library and dev variants:
#   r03_cfgtime.sh VARIANT...   ("" = product; NAME = build/dev/lib_NAME.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  if [ -n "$v" ]; then export QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_$v.so; else unset QS_DEV_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 242 --warmup 10 --no-cpu-baseline --mappo 0 --pyb ${PYB:-0} > gpurun_out/cfg_$v.json 2> gpurun_out/cfg_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/cfg_$v.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/cfg_$v.json'))
print('[$v] C3 %.3f us' % (d['roofline']['kernel_ms']*1e3), ' '.join('%s %.2f us (%.3f)' % (k, c['kernel_ms']*1e3, c['roofline_frac']) for k, c in d['configs'].items()), ('PYB %.2f us' % (d['pyb']['kernel_ms']*1e3)) if d.get('pyb') else '')"
done
