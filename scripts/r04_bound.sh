#!/bin/bash
# Bound-naming SQ counter passes on the C5 / C4 / C3 step kernels (own runs,
# kernel-trace only; scripts/bound_probe.py drives 40 steps of each), summarised
# by scripts/bound_report.py into profiles/rNN_bound_counters.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/${TAG}_bound_a -o run --output-format csv -- python3 scripts/bound_probe.py > gpurun_out/${TAG}_bound_a.log 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/${TAG}_bound_b -o run --output-format csv -- python3 scripts/bound_probe.py > gpurun_out/${TAG}_bound_b.log 2>&1
rc=$?; echo "pass b rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/bound_report.py gpurun_out/${TAG}_bound_counters.json gpurun_out/${TAG}_bound_a gpurun_out/${TAG}_bound_b
rm -rf gpurun_out/${TAG}_bound_a gpurun_out/${TAG}_bound_b
