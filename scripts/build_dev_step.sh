#!/bin/bash
# Dev variants of the whole libquadswarm.so (step kernels included):
#   build_dev_step.sh NAME "HIPCC FLAGS"   -> build/dev/lib_NAME.so (QS_DEV_LIB=<path> selects it)
# e.g. build_dev_step.sh floor "-DQS_X_NOCOMPUTE" (the probes: csrc/step_kernel_dev.h)
set -eu
cd "$(dirname "$0")/../marl-gym-pybullet-drones_amd"
name=$1; extra=$2
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I../include -DQS_DEV_BUILD $extra"
mkdir -p build/dev/$name
for u in quadswarm step_mh step_spiral step_marl learner normalizer ppo_small rollout; do
  /opt/rocm/bin/hipcc $FLAGS -c -o build/dev/$name/$u.o csrc/$u.hip &
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared -o build/dev/lib_$name.so build/dev/$name/*.o
rm -rf build/dev/$name
echo "built build/dev/lib_$name.so"
