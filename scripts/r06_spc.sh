#!/bin/bash
# Dev probe: launch 2's chunk sizes (QS_WG_SPC="actor,critic" steps per chunk) at one
# per-rank shape: per-workgroup stamps and the per-minibatch time (exchange path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
SH=${SH:-C3/8}
for spc in ${SPCS:-8,8 6,8 8,4 6,4 4,4}; do
  QS_WG_SPC=$spc QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_spc.so timeout -k 10 200 python3 -u scripts/wgrad_stamps.py $SH > gpurun_out/spc.log 2>&1 || exit 1
  echo "== spc $spc"; grep -v amdgpu gpurun_out/spc.log | head -4
  QS_SHAPES=$SH QS_WG_SPC=$spc QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_spc.so timeout -k 10 200 python3 -u scripts/learner_mb.py tiles > gpurun_out/spc2.log 2>&1 || exit 1
  grep minibatch gpurun_out/spc2.log
done
