"""Dev: device time of the inference forward qs_mlp3_fwd (the rollout's actor,
no saved activations) at the trainer legs' shapes, graph-timed.  Run once per
library (QS_DEV_LIB selects a dev build, e.g. one with another QS_M3_WIDE_I):
  python scripts/mlp3_fwd_probe.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402

SHAPES = [("C3 rollout", 131072, 27, 1), ("C4 rollout", 40960, 119, 4), ("C5 rollout", 65536, 72, 1),
          ("C4 I=64", 40960, 64, 4), ("C4 I=96", 40960, 96, 4)]


def main():
    lib = L.load()
    dev = "cuda"
    for name, K, I, A in SHAPES:
        g = torch.Generator(device=dev).manual_seed(K + I)
        X = torch.randn((K, I), device=dev, generator=g)
        W1 = torch.randn((256, I), device=dev, generator=g) * 0.1
        W2 = torch.randn((256, 256), device=dev, generator=g) * 0.06
        b1, b2 = torch.zeros(256, device=dev), torch.zeros(256, device=dev)
        W3, b3 = torch.randn((A, 256), device=dev, generator=g) * 0.06, torch.zeros(A, device=dev)
        pack = torch.empty(int(lib.qs_mlp3_pack_floats(I)), device=dev)
        out = torch.empty((K, A), device=dev)
        st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(lib.qs_mlp3_pack(I, 256, L.ptr(W1), L.ptr(W2), L.ptr(pack), st()), "qs_mlp3_pack")
        fn = lambda: L.check(lib.qs_mlp3_fwd(K, I, 256, A, L.ptr(X), L.ptr(pack), L.ptr(b1), L.ptr(b2), L.ptr(W3),
                                             L.ptr(b3), None, None, L.ptr(out), st()), "qs_mlp3_fwd")
        fn()
        ref = torch.tanh(torch.tanh(X @ W1.t() + b1) @ W2.t() + b2) @ W3.t() + b3
        torch.cuda.synchronize()
        err = float((out - ref).abs().max())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for _ in range(10):
                    fn()
        torch.cuda.synchronize()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        fl = 2 * K * (I * 256 + 256 * 256 + 256 * A)
        print(f"{os.environ.get('QS_DEV_LIB', 'default'):>28s} {name:12s} K={K:6d} I={I:3d} A={A}  {us:7.1f} us  "
              f"{fl / us / 1e6:6.1f} TFLOP/s  max|err| {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
