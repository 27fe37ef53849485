#!/bin/bash
# VERDICT r05 item 3 (C5, the D = 16 downwash): a proxy of the two-lanes-per-drone split
# from dev builds of the step kernel — dwhalf (half the pair terms per lane), epbhalf (two
# envs per wave: twice the waves, half of each idle), split_proxy (both: the split's
# instruction stream per wave with DPP instead of the per-lane permutes it would need)
# — each timed by the bench's config legs, and the SQ counters of C5 per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARS:-default dwhalf epbhalf split_proxy}; do
  lib=""; [ "$v" != default ] && lib=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_$v.so
  QS_DEV_LIB=$lib timeout -k 10 400 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --mappo 0 --pyb 0 --fp64 0 --rank-shapes '' > gpurun_out/c5p_$v.json 2> gpurun_out/c5p_$v.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c5p_$v.json').read().strip().splitlines()[-1])
c=d['configs']['C5']; print('$v', 'C5 kernel_ms', c.get('kernel_ms'), 'value', c.get('value'), 'hbm frac', (c.get('roofline') or {}).get('frac'), 'valu', c.get('valu_roofline'))"
done
