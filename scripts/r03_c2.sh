#!/bin/bash
# C2 reset-search check: the deferred-search parity tests, then the config legs under rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-c2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "deferred_reset or episode_log or free_running" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 242 --warmup 10 --no-cpu-baseline --mappo 0 --pyb 0 > gpurun_out/${TAG}_bench.json 2>gpurun_out/${TAG}_bench.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<PY
import csv, json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
for k, v in d["configs"].items(): print(k, round(v["kernel_ms"] * 1e3, 2), "us", round(v["roofline_frac"], 4))
import glob
f = glob.glob("gpurun_out/prof_${TAG}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "reset_search" in r["Name"] or "step_kernel<float, 0, 0" in r["Name"]:
        print(r["Name"][:60], r["Calls"], "avg", float(r["AverageNs"])/1e3, "min", float(r["MinNs"])/1e3, "max", float(r["MaxNs"])/1e3)
PY
rm -f gpurun_out/prof_${TAG}/*/*trace*.csv gpurun_out/prof_${TAG}/*trace*.csv 2>/dev/null; exit 0
