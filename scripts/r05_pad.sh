#!/bin/bash
# Transposed-activation row pad sweep of the tile path (QS_SMALL_PAD, floats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for pad in ${PADS:-16 48 80 144 272 1040}; do
  QS_SMALL_PAD=$pad timeout -k 10 120 python3 scripts/learner_mb.py shape:C3/8 shape:C5/8 2>&1 | grep minibatch | sed "s/^/pad $pad /"
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done
