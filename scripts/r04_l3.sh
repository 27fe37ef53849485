#!/bin/bash
# Round 4: what bounds the headline step kernel.  The C3
# rollout at 16 384 envs per GPU (≈40 MB touched per step: state, history, one
# obs slot — resident in the 256 MiB Infinity Cache between launches) and at
# 131 072 (≈300 MB per step: past it), kernel time per agent-step from HIP
# events, then FETCH_SIZE / WRITE_SIZE passes (separate runs, calibrated on
# qs_calib_copy) at both sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-l3}
for E in 16384 131072; do
  timeout -k 10 200 python3 bench.py --envs $E --steps 242 --warmup 20 --no-cpu-baseline --mappo 0 --pyb 0 --configs 0 \
    > gpurun_out/${TAG}_e$E.json 2> gpurun_out/${TAG}_e$E.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc E=$E"; tail -3 gpurun_out/${TAG}_e$E.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_e$E.json')); r=d['roofline']
print('E=$E kernel_ms', round(r['kernel_ms'], 5), 'ns/agent-step', round(r['kernel_ms'] * 1e6 / ($E * 8), 4), 'frac', round(r['frac'], 4), 'value', d['value'])"
  for C in FETCH_SIZE WRITE_SIZE; do
    PMC_ENVS=$E timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_${C}_$E -o run --output-format csv -- \
      python3 scripts/pmc_probe.py > gpurun_out/${TAG}_${C}_$E.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $C rc=$rc E=$E"; tail -3 gpurun_out/${TAG}_${C}_$E.log; exit $rc; }
  done
  python3 scripts/pmc_report.py gpurun_out/${TAG}_FETCH_SIZE_$E gpurun_out/${TAG}_WRITE_SIZE_$E $((1 << 28)) $((E * 8)) 418 $E 8 one_d_pid \
    > gpurun_out/${TAG}_pmc_$E.json && cat gpurun_out/${TAG}_pmc_$E.json
  rm -rf gpurun_out/${TAG}_FETCH_SIZE_$E gpurun_out/${TAG}_WRITE_SIZE_$E
done
