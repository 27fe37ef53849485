#!/bin/bash
# Kernel timeline of one C3 learner minibatch: rocprofv3 kernel
# trace of scripts/learner_mb.py one, analysed by scripts/learner_timeline.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-lt}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 scripts/learner_mb.py one > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_${TAG}.log; exit $rc; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python3 scripts/learner_timeline.py "$f" > gpurun_out/${TAG}_learner_timeline.txt
cat gpurun_out/${TAG}_learner_timeline.txt
rm -rf gpurun_out/prof_${TAG}
