import sys, os
sys.path[:0] = ["/root/repo/tests", "/root/repo/oracle", "/root/repo/marl-gym-pybullet-drones_amd"]
import trajectory as tj, test_gpu_parity as P
for name, cfg in P.CONFIGS.items():
    if len(sys.argv) > 1 and name not in sys.argv[1:]:
        continue
    for prec in (4, 8):
        r = tj.diverge(cfg, E=16, precision=prec, steps=30, seed=11)
        b = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4) if prec == 4 else dict(pos=1e-7, quat=1e-7, vel=1e-6, rew=1e-7)
        print(name, prec, {k: tj.first_exceed(r["curves"][k], v) for k, v in b.items()}, "ties", r["flag_ties"], flush=True)
