#!/bin/bash
# Fused actor kernel: phase stamps (dev build), store/head-less variants, SQ counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ap}
D=marl-gym-pybullet-drones_amd/build/dev
for v in qs_f_stamp qs_f_nostore qs_f_nohead; do
  echo "==== $v"
  QS_DEV_LIB=$D/lib_$v.so timeout -k 10 120 python3 scripts/learner_kbench.py fused > gpurun_out/${TAG}_$v.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_$v.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/${TAG}_pa -o run --output-format csv -- python3 scripts/learner_kbench.py fused > gpurun_out/${TAG}_pa.log 2>&1
echo "pmc a rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC --kernel-trace -d gpurun_out/${TAG}_pb -o run --output-format csv -- python3 scripts/learner_kbench.py fused > gpurun_out/${TAG}_pb.log 2>&1
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
