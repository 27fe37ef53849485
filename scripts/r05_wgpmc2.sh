#!/bin/bash
# Counters of the weight-gradient launch with only the actor's blocks (dev lib_skip, QS_WG_SKIP=6)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_skip.so QS_WG_SKIP=${QS_WG_SKIP:-6}
TAG=w2
run() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${TAG}_p$N -o run --output-format csv -- \
    python3 scripts/learner_mb.py shape:${SH:-C3/8} > gpurun_out/${TAG}_p$N.log 2>&1
  echo "pmc $N rc=$?"
}
N=a run TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
N=b run TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TD_BUSY_max
N=c run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
N=d run TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
python3 - <<PY
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/${TAG}_p*")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "ppo_small_wgrad" in r["Kernel_Name"]:
                acc["wgrad"][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for tag, cs in acc.items():
        for k, v in sorted(cs.items()):
            v = sorted(v); print(f"{tag} {k:36s} median {v[len(v)//2]:.6g} (n={len(v)})")
PY
rm -rf gpurun_out/${TAG}_p?
