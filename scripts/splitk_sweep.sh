#!/bin/bash
# Split-K chunk sweep of the learner's weight-gradient GEMMs (MAPPO leg only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for v in "" "32768x27=512" "32768x27=4096" "4096x216=256" "4096x216=4096" "32768x256=2048" "32768x256=512" "4096x256=256" "4096x256=4096"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --configs 0 --pyb 0 --no-cpu-baseline --mappo-t32 0 --steps 32 --mappo-iters 1 --splitk "$v" > gpurun_out/sk_$i.json 2>gpurun_out/sk_$i.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/sk_$i.json')); m=d['mappo']; print('[$v]', round(m['phase_ms']['update'],1), round(m['value']/1e6,3))"
done
timeout -k 10 300 python bench.py --mappo 0 --pyb 0 --no-cpu-baseline > gpurun_out/bc.json 2>gpurun_out/bc.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bc.json')); c=d['configs']['C2']; print('C2', c['kernel_ms'], c['roofline_frac'])"
