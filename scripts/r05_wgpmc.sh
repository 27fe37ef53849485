#!/bin/bash
# Counters of the tile path's kernels at one per-rank shape (scripts/learner_mb.py
# shape:NAME): wave states, instruction mix, L2 traffic — one pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-wp}; SH=${SH:-C3/8}
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${TAG}_p$N -o run --output-format csv -- \
    python3 scripts/learner_mb.py shape:$SH > gpurun_out/${TAG}_p$N.log 2>&1
  echo "pmc $N rc=$?"
}
N=a run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
N=b run SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM
N=c run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
python3 - <<PY
import csv, glob, collections
for d in ("gpurun_out/${TAG}_pa", "gpurun_out/${TAG}_pb", "gpurun_out/${TAG}_pc"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            for tag in ("ppo_small_fb", "ppo_small_wgrad", "ppo_small_apply"):
                if tag in k:
                    acc[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for tag, cs in acc.items():
        for k, v in sorted(cs.items()):
            v = sorted(v); print(f"${SH} {tag:16s} {k:30s} median {v[len(v)//2]:.6g} (n={len(v)})")
PY
rm -rf gpurun_out/${TAG}_pa gpurun_out/${TAG}_pb gpurun_out/${TAG}_pc
