"""Dev: table of kernel resource usage from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(r"remark:\s+" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0] + ("_spill" if "Spill" in key else "")] = int(m.group(1))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print(f'{r["name"][:70]:70s} v{r.get("VGPRs")} a{r.get("AGPRs")} spill{r.get("VGPRs_spill")} occ{r.get("Occupancy")} lds{r.get("LDS")}')
