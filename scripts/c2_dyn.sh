#!/bin/bash
# Dev: C2 reset search, the per-workgroup counters (QS_X_RSTATS build), then kernel stats of the shipped build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-c2p}
[ "${PYTEST:-1}" = "1" ] && { timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "deferred_reset or episode_log" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc; }
QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_rstats.so timeout -k 10 120 python3 scripts/c2_probe.py --steps 20 --warmup 3 > gpurun_out/${TAG}_rstats.log 2>&1
rc=$?; echo "rstats rc=$rc"; tail -3 gpurun_out/${TAG}_rstats.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 scripts/c2_probe.py --steps 100 > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}_prof.log; [ $rc -eq 0 ] || exit $rc
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/prof_${TAG}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "qs::" in r["Name"]:
        print(r["Name"][:60], r["Calls"], "avg", round(float(r["AverageNs"])/1e3, 2), "min", round(float(r["MinNs"])/1e3, 2), "max", round(float(r["MaxNs"])/1e3, 2))
PY
rm -f gpurun_out/prof_${TAG}/*/*trace*.csv gpurun_out/prof_${TAG}/*trace*.csv 2>/dev/null; exit 0
