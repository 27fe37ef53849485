#!/bin/bash
# Round-6 closing evidence on one GPU box (the bench line itself: scripts/r06_final.sh):
#   PART=K  rocprofv3 kernel stats of the simulator legs, then the PMC traffic
#           passes (FETCH_SIZE, WRITE_SIZE: separate runs) on the C3 step kernel
#   PART=T  the tile path's kernel split at the per-rank shapes through the exchange
#           launches (learner_mb.py shape:NAME:force) with launch 2's MFMA fraction
# Each GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06}
if [ "${PART:-K}" = "K" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python3 bench.py --steps 242 --warmup 20 --no-cpu-baseline --mappo 0 --fp64 0 > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_rocprof_kernel_stats.csv
  rm -rf gpurun_out/prof_${TAG}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcF_${TAG} -o run --output-format csv -- \
    python3 scripts/pmc_probe.py > gpurun_out/pmcF_${TAG}.log 2>&1
  rc=$?; echo "pmcF rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcW_${TAG} -o run --output-format csv -- \
    python3 scripts/pmc_probe.py > gpurun_out/pmcW_${TAG}.log 2>&1
  rc=$?; echo "pmcW rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 scripts/pmc_report.py gpurun_out/pmcF_${TAG} gpurun_out/pmcW_${TAG} $((1 << 28)) 131072 417.75 16384 8 one_d_pid \
    > gpurun_out/${TAG}_pmc_traffic.json && cat gpurun_out/${TAG}_pmc_traffic.json
  rm -rf gpurun_out/pmcF_${TAG} gpurun_out/pmcW_${TAG}
else
  out=gpurun_out/${TAG}_tile_kernels.txt; : > $out
  for sh in ${SHAPES:-C3/8 C3/4 C4/4 C5/8 ref}; do
    n=$(echo $sh | tr '/' '_')
    mode=force; [ "$sh" = ref ] && mode=
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_t$n -o run --output-format csv -- \
      python3 scripts/learner_mb.py shape:$sh${mode:+:$mode} > gpurun_out/${TAG}_t$n.log 2>&1
    rc=$?; grep minibatch gpurun_out/${TAG}_t$n.log | tee -a $out; [ $rc -eq 0 ] || exit $rc
    f=$(find gpurun_out/${TAG}_t$n -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$sh" >> $out <<'EOF'
import csv, sys
f, sh = sys.argv[1], sys.argv[2]
# rows and input widths of the shape's actor / critic (learner_mb.py RANK_SHAPES / SHAPES)
D, O, mb = {"C3/8": (8, 27, 512), "C3/4": (8, 27, 1024), "C4/4": (5, 119, 1024), "C5/8": (16, 27, 512),
            "ref": (8, 27, 32)}[sh]
Ka, Ia, Kc, Ic = mb * D, O, mb, D * O
flop = 2 * Ka * 256 * (256 + Ia) + 2 * Kc * 256 * (256 + Ic)   # dW2 + dW1 of both nets
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    if "ppo_small" in r["Name"]:
        us = float(r["AverageNs"]) / 1e3
        extra = ""
        if "wgrad" in r["Name"]:
            tf = flop / (us * 1e-6) / 1e12
            extra = f"   {flop / 1e6:.0f} MFLOP -> {tf:.1f} TFLOP/s = {tf / 157.3:.3f} of the 157.3 fp32 MFMA peak"
        print(f"  {sh:5s} {r['Calls']:>6s} {us:8.2f} us avg  {r['Name'][:90]}{extra}")
EOF
    rm -rf gpurun_out/${TAG}_t$n
  done
  cat $out
fi
exit 0
