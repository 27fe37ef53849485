"""Summarise rocprofv3 --pmc passes into per-launch HBM traffic for the step kernel.

FETCH_SIZE / WRITE_SIZE (KiB) are calibrated on qs_calib_copy (known bytes, dword
per lane — the step kernel's access width) as MI355X_MICROARCH.md §HBM prescribes."""
import csv
import glob
import json
import sys


def load(d):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def per_kernel(rows, counter):
    acc = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = r["Kernel_Name"]
        acc.setdefault(k, []).append(float(r["Counter_Value"]))
    return acc


def main(fetch_dir, write_dir, calib_bytes, agents, alg_bytes, envs=16384, drones=8, act="one_d_pid", precision=4):
    f = per_kernel(load(fetch_dir), "FETCH_SIZE")
    w = per_kernel(load(write_dir), "WRITE_SIZE")
    cal = [k for k in f if "calib_copy" in k][0]
    step = [k for k in f if "step_kernel" in k][0]
    cf = calib_bytes / (sum(f[cal]) / len(f[cal]) * 1024)
    cw = calib_bytes / (sum(w[cal]) / len(w[cal]) * 1024)
    sf = sorted(f[step])[len(f[step]) // 2] * 1024 * cf
    sw = sorted(w[step])[len(w[step]) // 2] * 1024 * cw
    out = {"fetch_scale": cf, "write_scale": cw, "step_fetch_bytes": sf, "step_write_bytes": sw,
           "step_traffic_bytes": sf + sw, "traffic_per_agent_step": (sf + sw) / agents,
           "algorithmic_per_agent_step": alg_bytes, "launches": len(f[step]),
           "workload": {"envs": envs, "drones": drones, "act": act}}
    if int(precision) != 4:   # the fp64 kernel's summary (float32 workloads keep the round-1 key set)
        out["workload"]["precision"] = int(precision)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5]),
         *(int(x) for x in sys.argv[6:8]), *sys.argv[8:10])
