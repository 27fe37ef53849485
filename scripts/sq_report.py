import csv, glob, sys, collections
for d in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        v = sorted(v)
        print(f"{d}: {k:24s} median {v[len(v)//2]:.4g}  (n={len(v)})")
