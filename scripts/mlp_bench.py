"""Dev: time the actor/critic MLP forward+backward of one PPO minibatch with torch's
nn.Linear vs a split-K weight gradient (bmm over row chunks + sum)."""
import sys, time
import torch

torch.manual_seed(0)
dev = "cuda"


class LinearSK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, splits):
        ctx.save_for_backward(x, w)
        ctx.splits = splits
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w if ctx.needs_input_grad[0] else None
        S, K = ctx.splits, x.shape[0]
        if S > 1 and K % S == 0:
            dw = torch.bmm(dy.reshape(S, K // S, -1).transpose(1, 2), x.reshape(S, K // S, -1)).sum(0)
        else:
            dw = dy.t() @ x
        return dx, dw, dy.sum(0), None


def mlp(x, layers, splits):
    for i, l in enumerate(layers):
        x = LinearSK.apply(x, l.weight, l.bias, splits) if splits else l(x)
        if i < len(layers) - 1:
            x = torch.tanh(x)
    return x


def run(rows, din, splits, reps=50):
    layers = [torch.nn.Linear(din, 256).to(dev), torch.nn.Linear(256, 256).to(dev), torch.nn.Linear(256, 1).to(dev)]
    x = torch.randn(rows, din, device=dev)
    g = torch.randn(rows, 1, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for l in layers:
                l.weight.grad = None; l.bias.grad = None
            mlp(x, layers, splits).backward(g)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        mlp(x, layers, splits).backward(g)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for rows, din in ((32768, 27), (4096, 216), (32768, 72), (4096, 576)):
    res = [f"{s}:{run(rows, din, s):.0f}us" for s in (0, 1, 4, 8, 16, 32, 64)]
    print(f"rows {rows} din {din}: " + "  ".join(res), flush=True)
