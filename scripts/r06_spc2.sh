#!/bin/bash
# Dev sweep: launch 2's steps per K-chunk (QS_WG_SPC="actor,critic", 32-row steps) at
# the per-rank shapes, per-minibatch time through the exchange path (learner_mb.py
# tiles, dev build lib_sw.so = -DQS_DEV_BUILD), to fit s_chunks' cost model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_sw.so
sweep() {
  local sh=$1; shift
  for spc in "$@"; do
    QS_SHAPES=$sh QS_WG_SPC=$spc QS_DEV_LIB=$LIB timeout -k 10 200 python3 -u scripts/learner_mb.py tiles > gpurun_out/spc2.log 2>&1 || { tail -3 gpurun_out/spc2.log; exit 1; }
    grep "force': True" gpurun_out/spc2.log | sed "s/^/spc $spc /"
  done
}
sweep C3/8 16,16 8,8 7,6 8,16 11,16 10,8 12,8 16,8
sweep C3/4 32,16 16,16 13,13 16,8 20,16 24,16 32,32 12,12
sweep C4/4 16,16 12,11 20,16 32,16 10,10 16,8 32,32
sweep C5/8 13,13 16,16 24,16 32,16 16,8 20,16 32,8
