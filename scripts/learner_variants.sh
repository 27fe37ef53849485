#!/bin/bash
# Learner / reset-search variant sweep on one GPU box: tests, then bench legs per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py tests/test_learner_splitk.py tests/test_gpu_parity.py -q -x --timeout 180 --timeout-method thread > gpurun_out/pyl.log 2>&1; rc=$?; grep -E "^E  |Error|passed|failed|^FAILED" gpurun_out/pyl.log | head -30; [ $rc -eq 0 ] || exit 1
for v in "w1 1" "w1,w2 1" ",  1"; do set -- $v; w=${1//,/_}; w=${w// /}
timeout -k 10 300 python bench.py --configs 0 --pyb 0 --no-cpu-baseline --mappo-t32 0 --steps 64 --side-stream $2 --wgrad "$1" > gpurun_out/bm_$w$2.json 2>gpurun_out/bm_$w$2.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bm_$w$2.json')); m=d['mappo']; print('$1 ss=$2', m['value'], m['phase_ms'], m['learner_roofline']['frac'])"; done
for g in 512 1024; do
QS_RESET_GRID=$g timeout -k 10 300 python bench.py --mappo 0 --pyb 0 --no-cpu-baseline > gpurun_out/bc_$g.json 2>gpurun_out/bc_$g.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bc_$g.json')); c=d['configs']['C2']; print('grid $g C2', c['kernel_ms'], c['roofline_frac'], 'C3', d['roofline']['kernel_ms'])"; done
