#!/bin/bash
# Round-6 dev A/B: the tile path's K-chunk sums in launch 2 by each tile's last chunk
# (XCD-local, after qs_ppo_small_xcd_probe) against launch 3 (QS_XCD_PROBE=0), one box — run on the
# build of that experiment (reverted: profiles/r06_chunk_sums_local.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in local launch3 local launch3; do
  if [ $v = launch3 ]; then export QS_XCD_PROBE=0; else unset QS_XCD_PROBE; fi
  QS_SHAPES="C3/8 C3/4 C5/8" timeout -k 10 300 python3 -u scripts/learner_mb.py tiles > gpurun_out/loc_ab.log 2>&1 || { tail -3 gpurun_out/loc_ab.log; exit 1; }
  grep "force': True" gpurun_out/loc_ab.log | sed "s/^/$v /"
done
