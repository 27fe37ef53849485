#!/bin/bash
# Round-4 evidence on one GPU box, in parts (each fits one gpurun call):
#   PART=A  every -m gpu test, then the default bench line
#   PART=B  rocprofv3 kernel stats of the simulator legs, the PMC traffic passes
#           (FETCH_SIZE, WRITE_SIZE) and the MAPPO kernel split
#   PART=C  the L3-vs-HBM probe (scripts/r04_l3.sh), the bound-naming SQ passes
#           (scripts/r04_bound.sh), the learner variant timer and a rollout timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
fatal() { case "$1" in 0) return 1;; *) return 0;; esac; }
if [ "${PART:-A}" = "A" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_${TAG}.log; if fatal $rc; then exit $rc; fi
  timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_${TAG}.err; if fatal $rc; then exit $rc; fi
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'kernel_ms', d['roofline']['kernel_ms'], 'timing', d.get('timing'))
print('fp64', d['fp64']['kernel_ms'], d['fp64']['roofline_frac'])
print('pyb', d['pyb']['kernel_ms'], d['pyb']['roofline_frac'])
for k in ('mappo', 'mappo_t32'): m = d[k]; print(k, m['value'], m['ms_per_train_step'], 'frac', m['learner_roofline']['frac'])
for k, m in d.get('mappo_configs', {}).items(): print('mappo', k, m['value'], m['learner_roofline']['frac'], m['config']['learner_path'])
for k, v in d['configs'].items(): print(k, v['kernel_ms'], v['roofline_frac'])
print('cpu', d['cpu_baseline'])"
elif [ "${PART}" = "B" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python3 bench.py --steps 242 --warmup 20 --no-cpu-baseline --mappo 0 --fp64 0 > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "kt rc=$rc"; if fatal $rc; then exit $rc; fi
  rm -f gpurun_out/prof_${TAG}/*trace*.csv
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcF_${TAG} -o run --output-format csv -- \
    python3 scripts/pmc_probe.py > gpurun_out/pmcF_${TAG}.log 2>&1
  rc=$?; echo "pmcF rc=$rc"; if fatal $rc; then exit $rc; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcW_${TAG} -o run --output-format csv -- \
    python3 scripts/pmc_probe.py > gpurun_out/pmcW_${TAG}.log 2>&1
  rc=$?; echo "pmcW rc=$rc"; if fatal $rc; then exit $rc; fi
  python3 scripts/pmc_report.py gpurun_out/pmcF_${TAG} gpurun_out/pmcW_${TAG} $((1 << 28)) 131072 418 16384 8 one_d_pid \
    > gpurun_out/pmc_traffic_${TAG}.json && cat gpurun_out/pmc_traffic_${TAG}.json
  rm -rf gpurun_out/pmcF_${TAG} gpurun_out/pmcW_${TAG}
  TAG=${TAG}m bash scripts/prof_mappo.sh > gpurun_out/mappo_kernel_stats_${TAG}.txt 2>&1
  head -30 gpurun_out/mappo_kernel_stats_${TAG}.txt
else
  TAG=${TAG}_l3 bash scripts/r04_l3.sh > gpurun_out/l3_${TAG}.txt 2>&1; rc=$?; cat gpurun_out/l3_${TAG}.txt; if fatal $rc; then exit $rc; fi
  TAG=${TAG} bash scripts/r04_bound.sh > gpurun_out/bound_${TAG}.txt 2>&1; rc=$?; cat gpurun_out/bound_${TAG}.txt; if fatal $rc; then exit $rc; fi
  timeout -k 10 300 python3 scripts/learner_mb.py > gpurun_out/learner_mb_${TAG}.txt 2>&1; cat gpurun_out/learner_mb_${TAG}.txt
  TAG=${TAG}rp bash scripts/r04_rollprof.sh > gpurun_out/rollprof_${TAG}.txt 2>&1; tail -30 gpurun_out/rollprof_${TAG}.txt
fi
exit 0
