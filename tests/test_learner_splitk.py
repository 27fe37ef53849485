"""Split-K weight gradient of the learner MLPs (agent._LinearSplitK) against plain
nn.Linear autograd: same forward, gradients equal up to fp32 reduction order.
Runs on the CPU (the split path is device-independent) and, marked gpu, on cuda:0."""
import copy

import pytest
import torch

from gym_pybullet_drones_amd.mappo.agent import MLP, _splitk_chunks


def _grads(net, x, g):
    for p in net.parameters():
        p.grad = None
    net(x).backward(g)
    return [p.grad.clone() for p in net.parameters()]


def _check(device, rows, din):
    torch.manual_seed(0)
    net = MLP(din, 1, [256, 256], act='tanh').to(device)
    x = torch.randn(rows, din, device=device)
    g = torch.randn(rows, 1, device=device)
    assert _splitk_chunks(rows) > 1
    got = _grads(net, x, g)
    ref_net = copy.deepcopy(net)
    want = []
    for p in ref_net.parameters():
        p.grad = None
    out = x
    for i, fc in enumerate(ref_net.fcs):   # plain nn.Linear path
        out = fc(out)
        out = torch.tanh(out) if i < len(ref_net.fcs) - 1 else out
    out.backward(g)
    want = [p.grad for p in ref_net.parameters()]
    with torch.no_grad():
        torch.testing.assert_close(net(x), ref_net(x), rtol=0, atol=0)
    for a, b in zip(got, want):
        scale = float(b.abs().max())
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * scale)


def test_splitk_chunks():
    assert [_splitk_chunks(r) for r in (96, 2048, 4096, 32768, 131072, 3000)] == [1, 2, 4, 32, 64, 2]


@pytest.mark.parametrize("rows,din", [(4096, 27), (8192, 216)])
def test_splitk_matches_linear_cpu(rows, din):
    _check("cpu", rows, din)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,din", [(32768, 27), (4096, 216)])
def test_splitk_matches_linear_gpu(rows, din):
    _check("cuda", rows, din)


def _plain(net, x, g):
    for p in net.parameters():
        p.grad = None
    out = x
    for i, fc in enumerate(net.fcs):
        out = fc(out)
        out = torch.tanh(out) if i < len(net.fcs) - 1 else out
    out.backward(g)
    return out.detach(), [p.grad.clone() for p in net.parameters()]


@pytest.mark.gpu
@pytest.mark.parametrize("rows,din,hidden,A", [(32768, 27, 256, 1), (4096, 216, 256, 1), (8192, 72, 256, 4),
                                               (16400, 595, 256, 2), (32768, 119, 256, 4), (65536, 72, 256, 1),
                                               (4096, 30, 64, 2), (2048, 20, 512, 1)])
def test_fused_tanh_mlp_matches_autograd(rows, din, hidden, A):
    """_TanhMLP3 (hipBLASLt GEMMs + qs_mlp_* kernels, grads accumulated into .grad
    buffers) against nn.Linear/torch.tanh autograd."""
    torch.manual_seed(1)
    net = MLP(din, A, [hidden, hidden], act='tanh').cuda()
    ref = copy.deepcopy(net)
    x = torch.randn(rows, din, device="cuda")
    g = torch.randn(rows, A, device="cuda") / rows
    want_out, want = _plain(ref, x, g)
    for p in net.parameters():
        p.grad = torch.full_like(p, 0.25)   # accumulates onto existing .grad
    assert net._fused_ok(x)
    out = net(x)
    out.backward(g)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.detach(), want_out, rtol=1e-5, atol=1e-5)
    for p, w in zip(net.parameters(), want):
        scale = float(w.abs().max())
        torch.testing.assert_close(p.grad - 0.25, w, rtol=1e-4, atol=1e-5 * scale + 1e-7)
    # a rerun gives bit-identical gradients (fixed-order reductions), also with the
    # reductions deferred into one multi-task launch (the learner's minibatch path)
    grads = [p.grad.clone() for p in net.parameters()]
    for p in net.parameters():
        p.grad.fill_(0.25)
    net(x).backward(g)
    for p, q in zip(net.parameters(), grads):
        assert torch.equal(p.grad, q)
    from gym_pybullet_drones_amd.mappo.agent import deferred_sums
    for p in net.parameters():
        p.grad.fill_(0.25)
    with deferred_sums():
        net(x).backward(g)
    for p, q in zip(net.parameters(), grads):
        assert torch.equal(p.grad, q)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,din,A", [(32768, 27, 1), (20000, 72, 4), (65536, 72, 1), (40960, 119, 4)])
def test_fused_inference_forward(rows, din, A):
    """The rollout's no-grad actor forward through qs_mlp3_fwd (no saved activations)
    against the plain nn.Linear / torch.tanh forward."""
    torch.manual_seed(2)
    net = MLP(din, A, [256, 256], act='tanh').cuda()
    x = torch.randn(rows, din, device="cuda")
    with torch.no_grad():
        got = net(x)
        out = x
        for i, fc in enumerate(net.fcs):
            out = fc(out)
            out = torch.tanh(out) if i < len(net.fcs) - 1 else out
    torch.testing.assert_close(got, out, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("envsteps,D,din,A", [(4096, 8, 27, 1), (256, 8, 27, 1), (600, 5, 72, 4)])
def test_group_rows_forward_bit_identical(envsteps, D, din, A):
    """qs_mlp3_fwd_group_rows (batch row r = table row rows[r // D]·D + r % D, the
    actor's minibatch read from the rollout table) against qs_mlp3_fwd on the
    gathered rows: the same kernel arithmetic, so identical bits (outputs and the
    saved activations); the 8-wave kernel at every size (the forward's choice
    since round 5)."""
    from gym_pybullet_drones_amd.mappo.agent import _M3Work
    torch.manual_seed(3)
    net = MLP(din, A, [256, 256], act='tanh').cuda()
    for p in net.parameters():
        p.grad = torch.zeros_like(p)
    table = torch.randn(3 * envsteps * D, din, device="cuda")
    idx = torch.randperm(3 * envsteps, device="cuda")[:envsteps]
    rows = (idx[:, None] * D + torch.arange(D, device="cuda")).reshape(-1)
    w_g, w_p = _M3Work(net, envsteps * D, "cuda"), _M3Work(net, envsteps * D, "cuda")
    w_g.repack()
    w_p.repack()
    got = w_g.forward(table, rows=idx, group=D).clone()
    want = w_p.forward(table[rows].contiguous()).clone()
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert torch.equal(w_g.h1, w_p.h1) and torch.equal(w_g.h2, w_p.h2)


@pytest.mark.gpu
@pytest.mark.parametrize("wgrad", [('w1',), ('w1', 'w2'), ()])
@pytest.mark.parametrize("rows,din,A", [(128, 216, 1), (1024, 27, 1), (4096, 216, 1), (32768, 27, 1), (1000, 27, 2)])
def test_m3work_matches_autograd(rows, din, A, wgrad, monkeypatch):
    """The direct iteration's _M3Work forward + backward (+ the fixed-order sums)
    against nn.Linear / torch.tanh autograd, including the small batches of the
    8-wave kernels, with the weight gradients on qs_mlp_wgrad or split-K GEMMs."""
    from gym_pybullet_drones_amd.mappo.agent import _M3Work, _flush_sums
    monkeypatch.setattr(_M3Work, "wgrad", wgrad)
    torch.manual_seed(4)
    net = MLP(din, A, [256, 256], act='tanh').cuda()
    ref = copy.deepcopy(net)
    x = torch.randn(rows, din, device="cuda")
    g = torch.randn(rows, A, device="cuda") / rows
    want_out, want = _plain(ref, x, g)
    for p in net.parameters():
        p.grad = torch.zeros_like(p)
    w = _M3Work(net, rows, "cuda")
    w.repack()
    out = w.forward(x).clone()
    tasks = []
    w.backward(x, g, tasks)
    _flush_sums(tasks)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, want_out, rtol=1e-5, atol=1e-5)
    for p, wg in zip(net.parameters(), want):
        scale = float(wg.abs().max())
        torch.testing.assert_close(p.grad, wg, rtol=1e-4, atol=1e-5 * scale + 1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,M,bt", [(32768, 256, 27, 0), (4096, 256, 216, 0), (32768, 256, 256, 1),
                                      (4096, 256, 256, 1), (2048, 64, 40, 1), (128, 32, 5, 0)])
def test_wgrad_kernel_matches_matmul(K, N, M, bt):
    """qs_mlp_wgrad's chunk partials: each chunk equals AT[:, chunk]·B[chunk] (fp64
    reference, fp32 tolerance) and their sum is the weight gradient."""
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    torch.manual_seed(5)
    at = torch.randn(N, K, device="cuda")
    b = torch.randn(M, K, device="cuda") if bt else torch.randn(K, M, device="cuda")
    bk = b.t() if bt else b
    C = int(lib.qs_mlp_wgrad_chunks(K, N, M))
    assert C >= 1
    part = torch.full((C, N, M), float("nan"), device="cuda")
    L.check(lib.qs_mlp_wgrad(K, N, M, L.ptr(at), L.ptr(b), bt, C, L.ptr(part), None), "qs_mlp_wgrad")
    torch.cuda.synchronize()
    R = K // C
    want = torch.stack([at[:, c * R:(c + 1) * R].double() @ bk[c * R:(c + 1) * R].double() for c in range(C)])
    torch.testing.assert_close(part.double(), want, rtol=1e-5, atol=1e-5 * R ** 0.5)
    assert lib.qs_mlp_wgrad(K + 1, N, M, L.ptr(at), L.ptr(b), bt, C, L.ptr(part), None) != 0   # K not a multiple of 32·C


@pytest.mark.gpu
@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("K,M", [(32768, 27), (4096, 216), (1024, 72), (128, 256)])
def test_wgrad_x_matches_fp64_matmul(K, M, blocked):
    """qs_mlp_wgrad_x: chunk partials of dW = ATᵀ-contraction with the layer
    input, summed in chunk order, against an fp64 matmul."""
    import ctypes
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    torch.manual_seed(3)
    at = torch.randn(256, K, device="cuda")
    x = torch.randn(K, M, device="cuda")
    C = int(lib.qs_mlp_wgrad_x_chunks(K, M))
    assert C == K // 128
    part = torch.full((C, 256, M), float("nan"), device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    src = at.reshape(256, K // 8, 8).permute(1, 0, 2).contiguous() if blocked else at   # [K/8][256][8]
    L.check(lib.qs_mlp_wgrad_x(K, 256, M, L.ptr(src), int(blocked), L.ptr(x), L.ptr(part), st), "qs_mlp_wgrad_x")
    want = at.double() @ x.double()
    got = part.double().sum(0)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-4 * float(want.abs().max()) / 100)
    assert lib.qs_mlp_wgrad_x_chunks(K + 64, M) == 0 and lib.qs_mlp_wgrad_x_chunks(K, 300) == 0
