#!/bin/bash
# Rebuild the extension with each EXTRA flag set and time the bench (dev tuning).
# Variants are separated by ';' in VARIANTS, e.g. VARIANTS="base;-DQS_NT_OBS".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
i=0
for v in "${VS[@]}"; do
  ex="$v"; [ "$v" = "base" ] && ex=""
  make -s -C marl-gym-pybullet-drones_amd clean && make -s -j16 -C marl-gym-pybullet-drones_amd EXTRA="$ex" > /dev/null 2>&1 || { echo "build failed: $v"; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --mappo 0 --pyb ${PYB:-0} --configs ${CONFIGS:-0} --steps ${STEPS:-640} > gpurun_out/var_$i.json 2>/dev/null
  rc=$?; if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; exit $rc; fi
  python3 - "$v" "gpurun_out/var_$i.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
out = "variant [%s] kernel_us %.2f value %.3e" % (sys.argv[1], d["roofline"]["kernel_ms"] * 1e3, d["value"])
if d.get("pyb"):
    out += " pyb_us %.2f" % (d["pyb"]["kernel_ms"] * 1e3)
for k, c in (d.get("configs") or {}).items():
    out += " %s_us %.2f" % (k, c["kernel_ms"] * 1e3)
print(out)
PY
  i=$((i+1))
done
