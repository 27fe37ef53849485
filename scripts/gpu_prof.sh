#!/bin/bash
# Evidence run: learner tests → bench (all legs) → kernel-trace stats → two separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) → per-launch HBM traffic summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "${LEARNER_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_learner.py -q -x > gpurun_out/learner_${TAG}.log 2>&1
  rc=$?; echo "learner tests rc=$rc"; tail -2 gpurun_out/learner_${TAG}.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err; if fatal $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --mappo 0 > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "kt rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcF_${TAG} -o run --output-format csv -- \
  python3 scripts/pmc_probe.py > gpurun_out/pmcF_${TAG}.log 2>&1
rc=$?; echo "pmcF rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcW_${TAG} -o run --output-format csv -- \
  python3 scripts/pmc_probe.py > gpurun_out/pmcW_${TAG}.log 2>&1
rc=$?; echo "pmcW rc=$rc"; if fatal $rc; then exit $rc; fi
python3 scripts/pmc_report.py gpurun_out/pmcF_${TAG} gpurun_out/pmcW_${TAG} $((1 << 28)) 131072 418 16384 8 one_d_pid \
  > gpurun_out/pmc_traffic_${TAG}.json && cat gpurun_out/pmc_traffic_${TAG}.json
exit 0
