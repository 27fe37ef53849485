#!/bin/bash
# Step-kernel time with resets spread over the window (default) vs none until step 242.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for f in "" "--no-stagger" "" "--no-stagger"; do
  timeout -k 10 120 python bench.py --mappo 0 --pyb 0 --configs 0 --no-cpu-baseline $f > gpurun_out/st.json 2>gpurun_out/st.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/st.json')); print('[$f]', d['roofline']['kernel_ms'], d['roofline']['frac'], d['config']['episodes_ended_in_timed_window_rank0'])"
done
