"""Dev: print the kernel timeline (start offsets / durations, us) of a window of a
rocprofv3 --kernel-trace csv: python scripts/timeline_report.py <trace.csv> [skip] [count]."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 40
win = rows[skip:skip + cnt]
t0 = int(win[0]["Start_Timestamp"])
for r in win:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:9.2f} {e / 1e3:9.2f} {(e - s) / 1e3:8.2f} q{r.get('Queue_Id', '?'):>3s} {r['Kernel_Name'][:90]}")
