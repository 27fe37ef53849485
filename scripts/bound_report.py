"""Per-kernel summary of the bound-naming SQ passes (rocprofv3 counter CSVs):
wave time split into parked on s_waitcnt / barrier (SQ_WAIT_ANY: memory
latency), issue-stalled (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), the
VALU share of the issuing time, LDS instructions and the SQ busy fraction.
  python scripts/bound_report.py OUT.json DIR...   (DIR: rocprofv3 -d output)"""
import collections
import csv
import glob
import json
import sys

NAMES = {"step_kernel<float, 0, 4, 30, 0, 1>": "C5", "step_kernel<float, 1, 2, 48, 1, 0>": "C4",
         "step_kernel<float, 0, 4, 30, 1, 0>": "C3"}


def short(k):
    for pat, n in NAMES.items():
        if pat.replace(" ", "") in k.replace(" ", ""):
            return n
    return None


acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = short(r["Kernel_Name"])
            if n:
                acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for n, c in sorted(acc.items()):
    med = {k: sorted(v)[len(v) // 2] for k, v in c.items()}
    rec = {"counters_median_per_launch": med, "launches": max(len(v) for v in c.values())}
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if k in med:
                rec[k.replace("SQ_", "").lower() + "_frac_of_wave_cycles"] = med[k] / wc
    if "SQ_ACTIVE_INST_ANY" in med and "SQ_ACTIVE_INST_VALU" in med:
        rec["valu_share_of_issuing"] = med["SQ_ACTIVE_INST_VALU"] / med["SQ_ACTIVE_INST_ANY"]
    if "SQ_WAVES" in med and wc:
        rec["wave_cycles_per_wave_quad"] = wc / med["SQ_WAVES"]
    out[n] = rec
    print(n, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in rec.items()
                         if k != "counters_median_per_launch"}))
json.dump(out, open(sys.argv[1], "w"), indent=1)
