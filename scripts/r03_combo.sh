#!/bin/bash
# Dev: one GPU call for the reset-search / step-kernel / learner iteration:
# parity tests of the reset paths, the C2 probe (counters + kernel stats), the
# simulator legs of the bench, then a kernel trace of a few MAPPO minibatches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-cb}
timeout -k 10 400 python -u -m pytest ${PYTESTS:-tests/test_gpu_parity.py tests/test_gpu_tolerance.py} -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
PYTEST=0 TAG=${TAG}c2 bash scripts/c2_dyn.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 242 --warmup 10 --no-cpu-baseline --mappo 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
print("C3", round(d["roofline"]["kernel_ms"] * 1e3, 2), "us frac", round(d["roofline"]["frac"], 4), "PYB", round(d["pyb"]["kernel_ms"] * 1e3, 2), round(d["pyb"]["roofline_frac"], 4))
for k, v in d["configs"].items(): print(k, round(v["kernel_ms"] * 1e3, 2), "us", round(v["roofline_frac"], 4))
PY
[ "${TIMELINE:-1}" = "1" ] && TAG=${TAG}tl bash scripts/r03_timeline.sh
exit 0
