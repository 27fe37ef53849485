#!/bin/bash
# Kernel iteration loop on one GPU box: parity tests → bench → SQ counters → phase stamps.
# Stops at the first GPU fault/abort/timeout (exit 124/134/137/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-it}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x --ignore=tests/test_gpu_learner.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; if fatal $rc; then exit $rc; fi
if [ "${SQ:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/${TAG}_sq -o run --output-format csv -- python3 scripts/pmc_probe.py > gpurun_out/${TAG}_sq.log 2>&1
  rc=$?; echo "sq rc=$rc"; if fatal $rc; then exit $rc; fi
fi
if [ "${STAMPS:-1}" = "1" ]; then
  make -s -C marl-gym-pybullet-drones_amd clean && make -s -C marl-gym-pybullet-drones_amd STAMPS=1 > /dev/null 2>&1
  timeout -k 10 120 python scripts/stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1
  rc=$?; echo "stamps rc=$rc"; cat gpurun_out/${TAG}_stamps.txt
fi
exit 0
