#!/bin/bash
# Learner tests, then the MAPPO legs of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_learner_splitk.py -q -x --timeout 180 --timeout-method thread > gpurun_out/pyl.log 2>&1; rc=$?; tail -2 gpurun_out/pyl.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --configs 0 --pyb 0 --no-cpu-baseline --steps 64 > gpurun_out/lc.json 2>gpurun_out/lc.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/lc.json'))
for k in ('mappo', 'mappo_t32'): m=d[k]; print(k, round(m['value']/1e6, 3), m['phase_ms'], round(m['learner_roofline']['frac'], 4))"
done
