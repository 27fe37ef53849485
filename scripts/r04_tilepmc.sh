#!/bin/bash
# SQ counters of the critic-tile launch (scripts/learner_mb.py kernels): three passes
# (wave states, instruction mix, instruction cache).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tp}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/${TAG}_pa -o run --output-format csv -- python3 scripts/learner_mb.py kernels > gpurun_out/${TAG}_pa.log 2>&1
echo "pmc a rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_MISC --kernel-trace -d gpurun_out/${TAG}_pb -o run --output-format csv -- python3 scripts/learner_mb.py kernels > gpurun_out/${TAG}_pb.log 2>&1
echo "pmc b rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/${TAG}_pc -o run --output-format csv -- python3 scripts/learner_mb.py kernels > gpurun_out/${TAG}_pc.log 2>&1
echo "pmc c rc=$?"
python3 - <<PY
import csv, glob, collections
for d in ("gpurun_out/${TAG}_pa", "gpurun_out/${TAG}_pb", "gpurun_out/${TAG}_pc"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            for tag in ("ppo_small_fb", "wgrad_t"):
                if tag in k:
                    acc[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for tag, cs in acc.items():
        for k, v in sorted(cs.items()):
            v = sorted(v); print(f"{tag:14s} {k:28s} median {v[len(v)//2]:.6g} (n={len(v)})")
PY
rm -rf gpurun_out/${TAG}_pa gpurun_out/${TAG}_pb gpurun_out/${TAG}_pc
