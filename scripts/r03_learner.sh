#!/bin/bash
# Learner iteration on one GPU box: the fused-actor / learner / train_step tests,
# then the MAPPO leg alone (and optionally its kernel split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03l}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_fused_actor.py tests/test_gpu_learner.py tests/test_gpu_train_step.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/${TAG}_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 ${BENCH_EXTRA:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.err; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); m=d['mappo']
print('MAPPO', m['value'], m['ms_per_train_step'], m['phase_ms'], 'learner frac', m['learner_roofline']['frac'])"
[ "${PROF:-0}" = "1" ] && TAG=${TAG}p BENCH_EXTRA="${BENCH_EXTRA:-}" bash scripts/prof_mappo.sh
exit 0
