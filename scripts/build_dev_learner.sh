#!/bin/bash
# Dev variants of libquadswarm.so with learner probe flags (QS_DEV_LIB=<path> selects one).
set -eu
cd "$(dirname "$0")/../marl-gym-pybullet-drones_amd"
make -j8 >/dev/null
mkdir -p build/dev
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I../include"
for v in "$@"; do
  name=$(echo "$v" | tr 'A-Z' 'a-z' | tr -c 'a-z0-9\n' '_')
  /opt/rocm/bin/hipcc $FLAGS -D$v -c -o build/dev/learner_$name.o csrc/learner.hip
  /opt/rocm/bin/hipcc $FLAGS -shared -o build/dev/lib_$name.so build/quadswarm.o build/step_mh.o build/step_spiral.o build/step_marl.o build/dev/learner_$name.o
  rm -f build/dev/learner_$name.o
  echo "built build/dev/lib_$name.so"
done
