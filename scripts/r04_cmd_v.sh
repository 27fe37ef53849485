for f in 0 1; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 --mappo-configs "" --fp64 $f > gpurun_out/r04v_f$f.json 2>/dev/null && python3 -c "
import json; m=json.load(open('gpurun_out/r04v_f$f.json'))['mappo']; print('fp64 leg $f: mappo', round(m['value']), m['phase_ms'])"; done
QS_DEV_LIB=marl-gym-pybullet-drones_amd/build/dev/lib_notall.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs 0 --pyb 0 --mappo-t32 0 --mappo-configs "" --fp64 0 > gpurun_out/r04v_nt.json 2>/dev/null && python3 -c "
import json; m=json.load(open('gpurun_out/r04v_nt.json'))['mappo']; print('notall: mappo', round(m['value']), m['phase_ms'])"
