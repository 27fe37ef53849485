#!/bin/bash
# SQ counter pass on the step kernel (own run, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-sq}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/${TAG}_a -o run --output-format csv -- python3 scripts/pmc_probe.py > gpurun_out/${TAG}_a.log 2>&1
rc=$?; echo "sq_a rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH --kernel-trace -d gpurun_out/${TAG}_b -o run --output-format csv -- python3 scripts/pmc_probe.py > gpurun_out/${TAG}_b.log 2>&1
echo "sq_b rc=$?"
