#!/bin/bash
# K-chunk size sweep of the tile path's weight gradients (dev lib_skip, QS_SMALL_GQ quads per chunk)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for gq in ${GQS:-32 64 128}; do
  QS_SMALL_GQ=$gq QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_skip.so timeout -k 10 120 python3 scripts/learner_mb.py shape:C3/8 shape:C5/8 shape:C3/4 shape:C3/2 2>&1 | grep minibatch | sed "s/^/gq $gq /"
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done
