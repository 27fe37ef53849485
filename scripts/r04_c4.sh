#!/bin/bash
# Round 4: the C4 trainer leg (Spiral, VEL, norm_obs) with the actor on the
# two-kernel path and on the fused actor kernel (--fused-max-a 4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-c4}
for a in 1 4; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 \
    --mappo-configs C4 --fused-max-a $a > gpurun_out/${TAG}_a$a.json 2> gpurun_out/${TAG}_a$a.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc [a=$a]"; tail -5 gpurun_out/${TAG}_a$a.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_a$a.json'))
for k, m in [('C3', d['mappo'])] + list(d['mappo_configs'].items()):
    c = m['config']; print('a=$a', k, 'value', round(m['value']), 'ms', round(m['ms_per_train_step'], 1), 'phase', {q: round(v, 2) for q, v in m['phase_ms'].items()}, 'frac', round(m['learner_roofline']['frac'], 4), 'fused', c['fused_actor_kernel'], 'us/mb', round(m['phase_ms']['update'] * 1e3 / (10 * c['minibatches_per_epoch']), 1), 'rollout us/step', round(m['phase_ms']['rollout'] * 1e3 / c['rollout_steps'], 1))"
done
