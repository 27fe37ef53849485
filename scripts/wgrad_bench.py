"""Dev: qs_wgrad_rm against torch.bmm row-chunk GEMMs at the actor's dW2 shape
(K agent rows x 256 x 256), HIP-event timing over back-to-back launches."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-gym-pybullet-drones_amd"))
import torch  # noqa: E402

from gym_pybullet_drones_amd import _lib as L  # noqa: E402

lib = L.load()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
A = torch.randn(K, 256, device="cuda")
B = torch.tanh(torch.randn(K, 256, device="cuda"))

def st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

flop = 2.0 * K * 256 * 256


def timeit(fn, n=50):
    """us per call: n calls captured in one HIP graph (no host launch overhead)"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for C in (16, 32, 64, 128):
    if K % (8 * C):
        continue
    part = torch.empty(C, 256, 256, device="cuda")
    us = timeit(lambda: L.check(lib.qs_wgrad_rm(K, 256, 256, L.ptr(A), L.ptr(B), C, L.ptr(part), st()), "wgrad_rm"))
    err = (part.double().sum(0) - A.double().t() @ B.double()).abs().max().item()
    print(f"qs_wgrad_rm K={K} C={C}: {us:.2f} us, {flop / us / 1e6:.1f} TFLOP/s, max|err| {err:.2e}", flush=True)
for S in (16, 32):
    part = torch.empty(S, 256, 256, device="cuda")
    us = timeit(lambda: torch.bmm(A.view(S, K // S, 256).transpose(1, 2), B.view(S, K // S, 256), out=part))
    print(f"torch.bmm S={S}: {us:.2f} us, {flop / us / 1e6:.1f} TFLOP/s", flush=True)
