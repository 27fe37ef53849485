#!/bin/bash
# Round-6 dev A/B (profiles/r06_window_env.txt): the driver's 20-step window, sim leg only,
# with HSA_ENABLE_INTERRUPT=0 against the default, alternating three times on one box.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  for v in default poll; do
    if [ $v = poll ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --mappo 0 --configs 0 --pyb 0 --fp64 0 --no-cpu-baseline > gpurun_out/win_$v$i.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/win_$v$i.json').read().strip().splitlines()[-1]); t=d['timing']
print('$v', '%.4g'%d['value'], 'wall %.2f us/step'%(1e3*t['wall_ms_per_step']), 'event %.2f'%(1e3*t['event_ms_per_step']), 'fixed %.1f'%t['fixed_wall_us_per_window'])"
  done
done
