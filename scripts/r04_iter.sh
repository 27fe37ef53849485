#!/bin/bash
# Round 4 iteration on one box: the new kernels' tests first, the whole -m gpu
# suite, then the MAPPO legs the round works on (C4, the reference's learner
# shape) and the learner probe.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-it}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_rollout_glue.py tests/test_gpu_train_step.py tests/test_gpu_normalizer.py tests/test_gpu_learner.py -k "${TESTK:-small or norm or rms or side_stream or sample or record or step or train}" > gpurun_out/${TAG}_new.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_new.log; [ $rc -eq 0 ] || exit $rc
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 600 $PT tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for leg in ${LEGS:-ref C4}; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 --mappo 1 \
    --mappo-configs $leg ${BENCH_ARGS:-} > gpurun_out/${TAG}_$leg.json 2> gpurun_out/${TAG}_$leg.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc [$leg]"; tail -5 gpurun_out/${TAG}_$leg.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$leg.json'))
for k, m in [('C3', d['mappo'])] + list(d['mappo_configs'].items()):
    c = m['config']; print('$leg', k, 'value', round(m['value']), 'ms', round(m['ms_per_train_step'], 1), 'phase', {q: round(v, 2) for q, v in m['phase_ms'].items()}, 'frac', round(m['learner_roofline']['frac'], 4), 'fused', c['fused_actor_kernel'], 'us/mb', round(m['phase_ms']['update'] * 1e3 / (10 * c['minibatches_per_epoch']), 1), 'rollout us/step', round(m['phase_ms']['rollout'] * 1e3 / c['rollout_steps'], 1))"
done
