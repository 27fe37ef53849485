#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for a in 0 1 2 4 8 16 6 7 31; do
  QS_ABLATE=$a timeout -k 10 120 python bench.py --steps 256 --warmup 32 --no-cpu-baseline > gpurun_out/abl_$a.json 2>/dev/null
  rc=$?; case $rc in 124|134|137|139) echo "abort $rc"; exit $rc;; esac
  python -c "import json;d=json.load(open('gpurun_out/abl_$a.json'));print('ablate $a kernel_us %.2f'%(d['roofline']['kernel_ms']*1e3))"
done
