#!/bin/bash
# Round-6 dev A/B (profiles/r06_wgrad_32row.txt): the tile-path tests, then the per-rank tile
# timing of the tree's build against build/dev/lib_g64.so (scripts/build_dev_step.sh g64
# "-DQS_GBK=64" on the 32-row-stage source of that experiment, since reverted), then chunk
# sweeps (scripts/r06_spc.sh).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=g32 PROBE= bash scripts/r06_iter.sh || exit 1
for lib in default g64 default g64; do
  if [ $lib = default ]; then unset QS_DEV_LIB; else export QS_DEV_LIB=$PWD/marl-gym-pybullet-drones_amd/build/dev/lib_$lib.so; fi
  timeout -k 10 300 python3 -u scripts/learner_mb.py tiles > gpurun_out/g32_tiles.log 2>&1 || { tail -5 gpurun_out/g32_tiles.log; exit 1; }
  grep minibatch gpurun_out/g32_tiles.log | grep "True}" | sed "s/^/$lib /"
done
unset QS_DEV_LIB
SH=C3/8 SPCS="16,16 8,8 8,16 6,8 4,4" bash scripts/r06_spc.sh || exit 1
SH=C3/4 SPCS="32,16 16,8 16,16 12,8 8,8" bash scripts/r06_spc.sh || exit 1
