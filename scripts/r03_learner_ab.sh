#!/bin/bash
# Learner A/B in one box: the MAPPO T=256 leg with the default learner, with
# qs_wgrad_rm for dW2, and with the actor chain captured first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
for v in "" "--wgrad-rm 1" "--actor-first 1" "--wgrad-rm 1 --actor-first 1" ""; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 --mappo-configs "" $v > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc [$v]"; tail -3 gpurun_out/${TAG}.err; exit $rc; }
  python3 -c "
import json; m=json.load(open('gpurun_out/${TAG}.json'))['mappo']; print('[$v]', round(m['value']), round(m['ms_per_train_step'], 1), m['phase_ms'], round(m['learner_roofline']['frac'], 4))"
done
