#!/bin/bash
# Every -m gpu test, then the default bench line (summary printed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; grep -E "^FAILED|Error" gpurun_out/${TAG}_pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/${TAG}_bench.err; [ $rc -eq 0 ] || exit $rc
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
print("value", d["value"], "frac", d["roofline"]["frac"], "kernel_ms", d["roofline"]["kernel_ms"], "ms/step", d["ms_per_step"])
if d.get("pyb"): print("pyb", d["pyb"])
for k in ("mappo", "mappo_t32"):
    m = d.get(k)
    if m: print(k, m["value"], m["ms_per_train_step"], m["phase_ms"], "frac", m["learner_roofline"]["frac"])
for k, v in (d.get("configs") or {}).items(): print(k, v["value"], v["kernel_ms"], v["roofline_frac"])
print("cpu", d.get("cpu_baseline"))
PY
