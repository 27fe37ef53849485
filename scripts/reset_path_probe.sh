#!/bin/bash
# Dev: step-kernel time (staggered resets) with parts of the reset path compiled
# out (lib/var/*.so built with -DQS_X_<flag>; timing only, results not valid).
set -u
PRE=${PRE:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=marl-gym-pybullet-drones_amd/gym_pybullet_drones_amd/lib/var
for v in base NORESETDRAW NOLOG base; do
  lib=""; [ "$v" = base ] || lib="$PWD/$V/$v.so"
  QS_DEV_LIB="$lib" timeout -k 10 120 python bench.py --mappo 0 --pyb 0 --configs 0 --no-cpu-baseline > gpurun_out/rp.json 2>gpurun_out/rp.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/rp.json')); print('$v', round(d['roofline']['kernel_ms']*1e3, 3))"
done
