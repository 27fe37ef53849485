run() { timeout -k 10 200 python3 bench.py --steps 20 --warmup 20 $2 --no-cpu-baseline --mappo 0 --pyb 0 --configs 0 --fp64 0 > gpurun_out/r04y_$1.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/r04y_$1.json')); t=d['timing']; print('$1: value %.4g wall %.3f us event %.3f us fixed %.1f us' % (d['value'], t['wall_ms_per_step']*1e3, t['event_ms_per_step']*1e3, t['fixed_wall_us_per_window']))"; }
run base ""; run after "--rewarm 1"; run before "--rewarm-before 1"; run base2 ""; run after2 "--rewarm 1"; run before2 "--rewarm-before 1"
