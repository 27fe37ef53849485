"""Dev probe: time qs_mlp3_fwd / qs_mlp3_bwd alone on the actor minibatch shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402

from gym_pybullet_drones_amd import _lib as L  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
I = int(sys.argv[2]) if len(sys.argv) > 2 else 27
A = int(sys.argv[3]) if len(sys.argv) > 3 else 1
if os.environ.get("QS_LIB"):
    L.LIB_PATH = os.environ["QS_LIB"]
lib = L.load()
f = lambda *s: torch.randn(*s, device="cuda") * 0.1
x, w1, b1, w2, b2, w3, b3 = f(K, I), f(256, I), f(256), f(256, 256), f(256), f(A, 256), f(A)
pack = torch.empty(int(lib.qs_mlp3_pack_floats(I)), device="cuda")
h1, h2, out = torch.empty(256, K, device="cuda"), torch.empty(256, K, device="cuda"), torch.empty(K, A, device="cuda")
dout, dz2, dz1 = f(K, A), torch.empty(256, K, device="cuda"), torch.empty(256, K, device="cuda")
T = int(lib.qs_mlp3_tiles(K, I))
pa, pb = torch.empty(T, 256 * (1 + A) + A, device="cuda"), torch.empty(T, 256, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: L.ptr(t)
L.check(lib.qs_mlp3_pack(I, 256, P(w1), P(w2), P(pack), st))
fwd = lambda: L.check(lib.qs_mlp3_fwd(K, I, 256, A, P(x), P(pack), P(b1), P(b2), P(w3), P(b3), P(h1), P(h2), P(out), st))
bwd = lambda: L.check(lib.qs_mlp3_bwd(K, I, 256, A, P(dout), P(h1), P(h2), P(pack), P(w3), P(dz2), P(dz1), P(pa), P(pb),
                                      st))
for name, fn, fl in (("fwd", fwd, 2 * K * (I * 256 + 256 * 256 + 256 * A)), ("bwd", bwd, 2 * K * 256 * 256)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{name} K={K} I={I} A={A}: {us:.1f} us  {fl / us / 1e6:.1f} TFLOP/s", flush=True)
