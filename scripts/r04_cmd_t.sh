timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner.py -k "four_outputs or small" > gpurun_out/r04t_t.log 2>&1; rc=$?; tail -3 gpurun_out/r04t_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/learner_mb.py base ref > gpurun_out/r04t_mb.txt 2>&1 && QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_notall.so timeout -k 10 120 python3 scripts/learner_mb.py base >> gpurun_out/r04t_mb.txt 2>&1; cat gpurun_out/r04t_mb.txt
QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_tstamps.so timeout -k 10 200 python3 scripts/tile_stamps.py > gpurun_out/r04t_stamps.txt 2>&1; cat gpurun_out/r04t_stamps.txt
for K in 20 484; do timeout -k 10 200 python3 bench.py --steps $K --warmup 20 --no-cpu-baseline --mappo 0 --pyb 0 --configs 0 --fp64 0 > gpurun_out/r04t_b$K.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/r04t_b$K.json')); print('steps $K value', d['value'], 'timing', d['timing'])"; done
