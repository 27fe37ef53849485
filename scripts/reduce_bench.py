"""Dev: column sums of a [K, 256] fp32 gradient (the bias gradient) by several torch routes."""
import torch
dev = "cuda"


def timeit(fn, reps=100):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 10 * 1e3


for K, N in ((32768, 256), (4096, 256), (32768, 1)):
    dy = torch.randn(K, N, device=dev)
    ones = torch.ones(K, device=dev)
    ones_r = torch.ones(1, K, device=dev)
    out = torch.empty(N, device=dev)
    ref = dy.double().sum(0)
    S = max(1, K // 1024)
    cands = {
        "sum0": lambda: torch.sum(dy, 0, out=out),
        "mv": lambda: torch.mv(dy.t(), ones, out=out),
        "mm": lambda: torch.mm(ones_r, dy, out=out.view(1, N)),
        "split_sum": lambda: torch.sum(dy.view(S, K // S, N).sum(1), 0, out=out),
    }
    res = []
    for k, f in cands.items():
        t = timeit(f)
        f(); torch.cuda.synchronize()
        err = float((out.double() - ref).abs().max())
        res.append(f"{k}:{t:.1f}us(err {err:.1e})")
    print(f"K {K} N {N}: " + "  ".join(res), flush=True)
