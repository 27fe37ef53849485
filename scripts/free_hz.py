"""First-exceed steps of the fp32 kernel and of the exact-fp32 oracle against the
fp64 oracle for every free-running parity config (E=16, seed 11, FREE_STEPS):
the numbers behind tests/test_gpu_parity.py FREE_HORIZON_FP32.  GPU script."""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "marl-gym-pybullet-drones_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import trajectory as tj  # noqa: E402

spec = importlib.util.spec_from_file_location("tgp", os.path.join(ROOT, "tests", "test_gpu_parity.py"))
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
B = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)
out = {}
for name, cfg in m.CONFIGS.items():
    rec = {}
    for subj in ("kernel", "oracle"):
        r = tj.diverge(cfg, E=16, precision=4, steps=m.FREE_STEPS, seed=11, subject=subj)
        rec[subj] = {k: tj.first_exceed(r["curves"][k], b) for k, b in B.items()}
        rec[subj + "_ties"] = [r["flag_ties"], r["rew_ties"]]
    out[name] = rec
    print(name, json.dumps(rec), flush=True)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(out, f, indent=1)
