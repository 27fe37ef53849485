#!/bin/bash
# Round 6: DroneModel.CF2P on the GPU: its parity configs, then the simulator suites and a
# short sim-only bench (the CF2X kernels are instruction-identical to the previous build).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "cf2p" > gpurun_out/cf2p_par.log 2>&1
rc=$?; tail -5 gpurun_out/cf2p_par.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tolerance.py tests/test_gpu_surfaces.py > gpurun_out/cf2p_all.log 2>&1
rc=$?; tail -3 gpurun_out/cf2p_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --mappo 0 --no-cpu-baseline --pyb 1 --fp64 1 > gpurun_out/cf2p_bench.json 2>/dev/null
rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/cf2p_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'], 'pyb', d['pyb']['roofline_frac'], 'fp64', d['fp64']['roofline_frac'])
for k,v in d['configs'].items(): print(k, v['kernel_ms'], v['roofline_frac'])"
exit $rc
