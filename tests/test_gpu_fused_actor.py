"""qs_mlp3f_actor (the actor's forward, policy loss head and backward in one
launch, 16-row tiles on the f32 MFMA) against plain torch autograd of the
reference's expressions: MLPActor AG:87-148 + compute_policy_loss AG:602-640 and
the backward of policy_loss + ent_coef·entropy_loss (AG:733)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _net(I, A, seed):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(I, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(), nn.Linear(256, A)).cuda()


@pytest.mark.parametrize("mb,D,I,A", [(4096, 8, 27, 1), (96, 3, 27, 1), (37, 5, 72, 2), (16, 8, 100, 4)])
def test_fused_actor_matches_autograd(mb, D, I, A):
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    dev = "cuda"
    net = _net(I, A, 3)
    logstd = nn.Parameter(torch.full((A,), -0.5, device=dev) + 0.1 * torch.randn(A, device=dev))
    TE = 3 * mb + 5   # rollout env-timesteps; the minibatch samples mb of them
    g = torch.Generator(device=dev).manual_seed(1)
    table = torch.randn(TE, D, I, device=dev, generator=g)
    act = torch.randn(TE, D, A, device=dev, generator=g)
    adv = torch.randn(TE, device=dev, dtype=torch.float64, generator=g)
    idx = torch.randperm(TE, device=dev, generator=g)[:mb]
    x = table[idx].reshape(mb * D, I)
    with torch.no_grad():
        d0 = torch.distributions.Normal(net(x), logstd.exp())
        lp0 = d0.log_prob(act[idx].reshape(-1, A)).sum(-1) + 0.05 * torch.randn(mb * D, device=dev, generator=g)
    logp_old = torch.zeros(TE, D, device=dev)
    logp_old[idx] = lp0.reshape(mb, D)
    clip, ent = 0.2, 0.01
    K = mb * D
    # --- reference: autograd of the torch expressions
    z1 = net[0](x); h1 = torch.tanh(z1); z2 = net[2](h1); h2 = torch.tanh(z2); mean = net[4](h2)
    for t in (z1, z2, mean):
        t.retain_grad()
    dist = torch.distributions.Normal(mean, logstd.exp())
    logp = dist.log_prob(act[idx].reshape(-1, A)).sum(-1, keepdim=True)
    ratio = torch.exp(logp - logp_old[idx].reshape(-1, 1))
    a_ = adv[idx].repeat_interleave(D).reshape(-1, 1)
    pl = -torch.min(ratio * a_, torch.clamp(ratio, 1 - clip, 1 + clip) * a_).mean()
    el = -dist.entropy().sum(-1).mean()
    kl = (logp_old[idx].reshape(-1, 1) - logp).mean()
    (pl + ent * el).backward()
    # --- the fused kernel
    f32 = dict(device=dev, dtype=torch.float32)
    pack = torch.empty(int(lib.qs_mlp3f_pack_floats(I)), **f32)
    import ctypes
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.qs_mlp3f_pack(I, L.ptr(net[0].weight), L.ptr(net[2].weight), L.ptr(pack), stream), "qs_mlp3f_pack")
    G = int(lib.qs_mlp3f_tiles(K))
    xa = torch.full((K, I), np.nan, **f32)
    H1, dZ2, dZ1 = (torch.full((K, 256), np.nan, **f32) for _ in range(3))   # row-major
    partA = torch.empty((G, 256 * (1 + A) + A), **f32)
    partB = torch.empty((G, 256), **f32)
    dls = torch.empty(A, **f32)
    klo = torch.empty(1, **f32)
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    work = torch.zeros(int(lib.qs_mlp3f_work_bytes(K)), dtype=torch.uint8, device=dev)
    mean_out = torch.empty((K, A), **f32)
    for rep in range(2):   # the workspace is left ready for the next call
        acc.zero_()
        L.check(lib.qs_mlp3f_actor(K, I, D, A, L.ptr(table), L.ptr(idx), L.ptr(pack), L.ptr(net[0].bias),
                                   L.ptr(net[2].bias), L.ptr(net[4].weight), L.ptr(net[4].bias), L.ptr(logstd), 1.0,
                                   L.ptr(act), L.ptr(logp_old), L.ptr(adv), clip, ent, L.ptr(xa), L.ptr(H1), L.ptr(dZ2),
                                   L.ptr(dZ1), L.ptr(partA), L.ptr(partB), L.ptr(dls), L.ptr(klo), L.ptr(acc),
                                   L.ptr(work), L.ptr(mean_out), stream), "qs_mlp3f_actor")
        torch.cuda.synchronize()
        assert torch.equal(xa, x)
        torch.testing.assert_close(mean_out, mean.detach(), rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(H1, h1.detach(), rtol=0, atol=2e-6)
        s2 = float(z2.grad.abs().max())
        torch.testing.assert_close(dZ2, z2.grad, rtol=1e-3, atol=1e-4 * s2)
        s1 = float(z1.grad.abs().max())
        torch.testing.assert_close(dZ1, z1.grad, rtol=1e-3, atol=1e-4 * s1)
        pa, pb = partA.double().sum(0), partB.double().sum(0)
        for got, want in ((pa[:256], net[2].bias.grad), (pa[256:256 + 256 * A].reshape(A, 256), net[4].weight.grad),
                          (pa[256 + 256 * A:], net[4].bias.grad), (pb, net[0].bias.grad)):
            sc = float(want.abs().max())
            torch.testing.assert_close(got.float(), want, rtol=1e-3, atol=1e-4 * sc)
        torch.testing.assert_close(dls, logstd.grad, rtol=1e-4, atol=1e-6)
        assert float(klo) == pytest.approx(float(kl), rel=1e-4, abs=1e-7)
        assert float(acc[0]) == pytest.approx(float(pl), rel=1e-5, abs=1e-8)
        assert float(acc[2]) == pytest.approx(float(el), rel=1e-6)
        assert float(acc[3]) == pytest.approx(float(kl), rel=1e-4, abs=1e-7)
        # weight gradients from the kernel's activations: dW2 = dZ2ᵀ·H1, dW1 = dZ1ᵀ·Xa
        for got, want in ((dZ2.double().t() @ H1.double(), net[2].weight.grad), (dZ1.double().t() @ xa.double(), net[0].weight.grad)):
            sc = float(want.abs().max())
            torch.testing.assert_close(got.float(), want, rtol=1e-3, atol=1e-4 * sc)


@pytest.mark.parametrize("K,N,M,C", [(32768, 256, 256, 64), (4096, 256, 256, 64), (2048, 128, 256, 4), (1024, 256, 128, 1)])
def test_wgrad_rm_matches_fp64(K, N, M, C):
    """qs_wgrad_rm chunk partials (the actor's dW2 = dZ2ᵀ·H1 from the fused
    kernel's row-major activations) against an fp64 matmul per chunk."""
    import ctypes
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(K, N, device="cuda", generator=g)
    B = torch.tanh(torch.randn(K, M, device="cuda", generator=g))
    part = torch.full((C, N, M), np.nan, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.qs_wgrad_rm(K, N, M, L.ptr(A), L.ptr(B), C, L.ptr(part), stream), "qs_wgrad_rm")
    torch.cuda.synchronize()
    want = torch.bmm(A.double().view(C, K // C, N).transpose(1, 2), B.double().view(C, K // C, M))
    torch.testing.assert_close(part.double(), want, rtol=0, atol=2e-6 * (K // C) ** 0.5 * 4)
    # a replay is bit-identical (fixed summation order)
    again = torch.empty_like(part)
    L.check(lib.qs_wgrad_rm(K, N, M, L.ptr(A), L.ptr(B), C, L.ptr(again), stream), "qs_wgrad_rm")
    torch.cuda.synchronize()
    assert torch.equal(part, again)
    # shapes the kernel does not take are refused
    assert lib.qs_wgrad_rm(K, 96, M, L.ptr(A), L.ptr(B), C, L.ptr(part), stream) != 0


@pytest.mark.parametrize("mb,D,I,A", [(4096, 8, 27, 1), (96, 3, 27, 1), (37, 5, 72, 2), (2560, 5, 119, 4)])
def test_folded_dw1_matches_fp64(mb, D, I, A):
    """qs_mlp3f_actor_w1 (dW1 = dZ1ᵀ·X folded into the fused launch, VERDICT r04
    item 2): each workgroup's [256][I] partial against an fp64 matmul of the
    unfolded launch's dZ1 and Xa over the workgroup's 128 rows, their sum against
    autograd's W1 gradient; every other output bit-identical to qs_mlp3f_actor's."""
    import ctypes
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    dev = "cuda"
    net = _net(I, A, 4)
    logstd = nn.Parameter(torch.full((A,), -0.5, device=dev))
    TE = 2 * mb + 3
    g = torch.Generator(device=dev).manual_seed(7)
    table = torch.randn(TE, D, I, device=dev, generator=g)
    act = torch.randn(TE, D, A, device=dev, generator=g)
    adv = torch.randn(TE, device=dev, dtype=torch.float64, generator=g)
    idx = torch.randperm(TE, device=dev, generator=g)[:mb]
    x = table[idx].reshape(mb * D, I)
    with torch.no_grad():
        d0 = torch.distributions.Normal(net(x), logstd.exp())
        lp0 = d0.log_prob(act[idx].reshape(-1, A)).sum(-1) + 0.05 * torch.randn(mb * D, device=dev, generator=g)
    logp_old = torch.zeros(TE, D, device=dev)
    logp_old[idx] = lp0.reshape(mb, D)
    clip, ent = 0.2, 0.01
    K = mb * D
    mean = net(x)
    dist = torch.distributions.Normal(mean, logstd.exp())
    logp = dist.log_prob(act[idx].reshape(-1, A)).sum(-1, keepdim=True)
    ratio = torch.exp(logp - logp_old[idx].reshape(-1, 1))
    a_ = adv[idx].repeat_interleave(D).reshape(-1, 1)
    pl = -torch.min(ratio * a_, torch.clamp(ratio, 1 - clip, 1 + clip) * a_).mean()
    (pl + ent * (-dist.entropy().sum(-1).mean())).backward()
    f32 = dict(device=dev, dtype=torch.float32)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    pack = torch.empty(int(lib.qs_mlp3f_pack_floats(I)), **f32)
    L.check(lib.qs_mlp3f_pack(I, L.ptr(net[0].weight), L.ptr(net[2].weight), L.ptr(pack), stream), "qs_mlp3f_pack")
    G = int(lib.qs_mlp3f_tiles(K))
    outs = []
    for fold in (False, True):
        o = dict(xa=torch.full((K, I), np.nan, **f32), H1=torch.full((K, 256), np.nan, **f32),
                 dZ2=torch.full((K, 256), np.nan, **f32), dZ1=torch.full((K, 256), np.nan, **f32),
                 pA=torch.empty((G, 256 * (1 + A) + A), **f32), pB=torch.empty((G, 256), **f32),
                 dls=torch.empty(A, **f32), kl=torch.empty(1, **f32), acc=torch.zeros(4, dtype=torch.float64, device=dev),
                 pw1=torch.full((G, 256, I), np.nan, **f32) if fold else None)
        work = torch.zeros(int(lib.qs_mlp3f_work_bytes(K)), dtype=torch.uint8, device=dev)
        L.check(lib.qs_mlp3f_actor_w1(K, I, D, A, L.ptr(table), L.ptr(idx), L.ptr(pack), L.ptr(net[0].bias),
                                      L.ptr(net[2].bias), L.ptr(net[4].weight), L.ptr(net[4].bias), L.ptr(logstd), 1.0,
                                      L.ptr(act), L.ptr(logp_old), L.ptr(adv), clip, ent, L.ptr(o["xa"]), L.ptr(o["H1"]),
                                      L.ptr(o["dZ2"]), None if fold else L.ptr(o["dZ1"]), L.ptr(o["pA"]), L.ptr(o["pB"]),
                                      L.ptr(o["dls"]), L.ptr(o["kl"]), L.ptr(o["acc"]), L.ptr(work), None,
                                      L.ptr(o["pw1"]), stream), "qs_mlp3f_actor_w1")
        torch.cuda.synchronize()
        outs.append(o)
    ref, got = outs
    for k in ("xa", "H1", "dZ2", "pA", "pB", "dls", "kl", "acc"):
        assert torch.equal(ref[k], got[k]), k
    assert torch.isnan(got["dZ1"]).all()   # not stored when folded
    # per workgroup (128 rows): the fp64 contraction of the unfolded launch's dZ1 and Xa
    rows = torch.arange(G * 128, device=dev).clamp(max=K - 1)
    valid = (torch.arange(G * 128, device=dev) < K).double().view(G, 128, 1)
    dz = ref["dZ1"].double()[rows].view(G, 128, 256) * valid
    xa = ref["xa"].double()[rows].view(G, 128, I) * valid
    want = torch.bmm(dz.transpose(1, 2), xa)
    sc = float(want.abs().max())
    torch.testing.assert_close(got["pw1"].double(), want, rtol=0, atol=1e-5 * sc)
    total = got["pw1"].double().sum(0).float()
    s0 = float(net[0].weight.grad.abs().max())
    torch.testing.assert_close(total, net[0].weight.grad, rtol=1e-3, atol=1e-4 * s0)
