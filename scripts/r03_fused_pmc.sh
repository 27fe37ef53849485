#!/bin/bash
# fused actor kernel: correctness test, isolated timing of the learner kernels,
# two SQ counter passes on qs_mlp3f_actor (each its own run, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-fz}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_actor.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/learner_kbench.py ${KB:-} > gpurun_out/${TAG}_kbench.txt 2>&1; rc=$?; cat gpurun_out/${TAG}_kbench.txt; [ $rc -eq 0 ] || exit $rc
[ "${PMC:-1}" = "1" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/${TAG}_pa -o run --output-format csv -- python3 scripts/learner_kbench.py fused > gpurun_out/${TAG}_pa.log 2>&1
echo "pmc a rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-trace -d gpurun_out/${TAG}_pb -o run --output-format csv -- python3 scripts/learner_kbench.py fused > gpurun_out/${TAG}_pb.log 2>&1
echo "pmc b rc=$?"
python3 - <<PY
import csv, glob, collections
for d in ("gpurun_out/${TAG}_pa", "gpurun_out/${TAG}_pb"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mlp3f_actor" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        v = sorted(v); print(f"{k:28s} median {v[len(v)//2]:.6g} (n={len(v)})")
PY
rm -rf gpurun_out/${TAG}_pa gpurun_out/${TAG}_pb
