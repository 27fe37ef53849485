"""MAPPO agent: shared-weight Gaussian actor + centralized critic, PPO update on device.

Same model and loss semantics as gym_pybullet_drones/mappo/agent.py:
  MLP (safe_control_gym/math_and_models/neural_networks.py:18-54, default init)
  MLPActor AG:87-148 (logstd init -0.5, Normal(mean, exp(logstd)))
  CentralizedCritic AG:164-223 (D·O → hidden → hidden → 1 on concatenated obs)
  MAPPOActorCritic.step AG:389-415 (batched sample; v returned as zeros)
  compute_policy_loss AG:602-640, compute_value_loss AG:642-700, update AG:702-772
  (actor Adam step only if approx_kl <= 1.5·target_kl; critic step always;
  max_grad_norm configured but not applied — as in the reference)

MI355X-specific structure:
  * actor and critic parameters/gradients live in one flat fp32 buffer each;
    autograd accumulates into `.grad` views of it, so one RCCL all-reduce per
    model and one fused Adam launch (qs_adam_gated, HIP) update everything;
  * the KL gate is evaluated on the device by that kernel — no host sync per
    minibatch — so a whole update iteration (gather, forward, backward, both
    optimizer steps, stats) is captured once as a HIP graph and replayed;
  * under torch.distributed, approx_kl and the gradients are averaged across
    ranks before the gate/step, so every rank takes the same branch.
"""
import ctypes
import math
import os
from collections import defaultdict

import torch
import torch.distributed as tdist
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib as L
from . import collectives
from .collectives import capture_collectives, collective_group  # noqa: F401  (re-exported)


def get_activation(name):
    return getattr(torch, name) if name in ("tanh", "relu", "sigmoid") else (getattr(F, name) if name else (lambda x: x))


def _splitk_chunks(rows, min_rows=1024):
    """Row chunks of the split-K weight gradient: the largest power of two S with
    rows / S >= min_rows that divides rows (1 = plain GEMM)."""
    s = 1
    while rows % (2 * s) == 0 and rows // (2 * s) >= min_rows and s < 64:
        s *= 2
    return s


class _LinearSplitK(torch.autograd.Function):
    """nn.Linear with a split-K weight gradient.  A PPO minibatch's dW = dYᵀ X
    reduces over 32 768 rows into a 256×256 result: as one GEMM that is a few dozen
    output tiles on a 256-CU chip (hipBLASLt ran it at ~30 TFLOP/s); as S batched
    GEMMs over row chunks plus a sum over S it fills the chip (actor fwd+bwd
    587 → 339 µs per minibatch, scripts/mlp_bench.py).  Same math; fp32 rounding
    of the reduction order only."""

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
        if S > 1:
            dw = torch.bmm(dy.reshape(S, K // S, -1).transpose(1, 2), x.reshape(S, K // S, -1)).sum(0)
        else:
            dw = dy.t() @ x
        return dx, dw, dy.sum(0), None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_DEFER = None   # reductions queued while a minibatch backward runs (deferred_sums)


def _sum_partials(G, P, part, d0, n0, d1=None, n1=0, d2=None):
    """d += Σ_g part[g] (qs_mlp_sum_partials), or queued for one multi-task launch."""
    if _DEFER is not None:
        _DEFER.append((G, P, part, d0, n0, d1, n1, d2))
        return
    L.check(L.load().qs_mlp_sum_partials(G, P, L.ptr(part), L.ptr(d0), n0, L.ptr(d1), n1, L.ptr(d2), _stream()),
            "qs_mlp_sum_partials")


def _flush_sums(tasks):
    lib = L.load()
    for i in range(0, len(tasks), 16):   # qs_mlp_sum_partials_multi takes up to 16 tasks
        chunk = tasks[i:i + 16]
        n = len(chunk)
        arr = lambda ct, vals: (ct * n)(*vals)
        vp = ctypes.c_void_p
        L.check(lib.qs_mlp_sum_partials_multi(
            n, arr(ctypes.c_int32, [t[0] for t in chunk]), arr(ctypes.c_int64, [t[1] for t in chunk]),
            arr(vp, [t[2].data_ptr() for t in chunk]), arr(vp, [t[3].data_ptr() for t in chunk]),
            arr(ctypes.c_int64, [t[4] for t in chunk]),
            arr(vp, [t[5].data_ptr() if t[5] is not None else None for t in chunk]),
            arr(ctypes.c_int64, [t[6] for t in chunk]),
            arr(vp, [t[7].data_ptr() if t[7] is not None else None for t in chunk]), _stream()),
            "qs_mlp_sum_partials_multi")


class deferred_sums:
    """Within the block, the MLP backward's bias / weight-gradient reductions are
    queued and issued as one qs_mlp_sum_partials_multi launch at exit (8 small
    launches per PPO minibatch become one)."""

    def __enter__(self):
        global _DEFER
        self._prev, _DEFER = _DEFER, []
        return self

    def __exit__(self, *exc):
        global _DEFER
        tasks, _DEFER = _DEFER, self._prev
        if exc[0] is None and tasks:
            _flush_sums(tasks)
        return False


def _splitk_into(dst, dy, x):
    """dst += dyᵀ·x (a weight gradient) as S row-chunk GEMMs + a fixed-order sum."""
    K = x.shape[0]
    S = _splitk_chunks(K)
    if S == 1:
        dst.addmm_(dy.t(), x)
        return
    part = torch.bmm(dy.reshape(S, K // S, -1).transpose(1, 2), x.reshape(S, K // S, -1))
    _sum_partials(S, part[0].numel(), part, dst, dst.numel())


def _splitk_nt(dst, a, b, b_rows_are_k):
    """dst[N][M] += a·bᵀ (b [M][K], b_rows_are_k False: b [K][M]) with a [N][K]: a
    weight gradient from transposed activations, as S K-chunk GEMMs + a fixed-order sum."""
    K = a.shape[1]
    S = _splitk_chunks(K)
    bk = b.t() if b_rows_are_k else b   # [K][M] view
    if S == 1:
        dst.addmm_(a, bk)
        return
    a3 = a.view(a.shape[0], S, K // S).transpose(0, 1)                                  # [S][N][K/S]
    b3 = b.view(b.shape[0], S, K // S).permute(1, 2, 0) if b_rows_are_k else b.view(S, K // S, -1)   # [S][K/S][M]
    part = torch.bmm(a3, b3)
    _sum_partials(S, part[0].numel(), part, dst, dst.numel())


class _TanhMLP3(torch.autograd.Function):
    """The reference MLP with two tanh hidden layers and a linear head
    (neural_networks.py:18-54), forward and backward, on the MI355X path.
    Hidden width 256 (the reference MAPPO's hidden_dim, learn_mappo.py:196):
    qs_mlp3_fwd / qs_mlp3_bwd fuse both layers, bias + tanh and the head on the
    f32 MFMA with the pre-activations kept on chip; the weight gradients are
    split-K GEMMs.  Other widths: hipBLASLt GEMMs for the contractions, HIP kernels for everything between them
    (qs_mlp_bias_tanh: bias + tanh, and the head's row dot products in the same
    pass; qs_mlp_tanh_bwd: the head backward fused with tanh's, and the bias /
    head-weight gradient partials; qs_mlp_sum_partials: fixed-order reductions,
    accumulated straight into the parameters' .grad buffers).  Used by MLP when
    every parameter already has a .grad buffer (the learner's flat buffers), so
    the backward returns no tensors for autograd to add."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        lib, st = L.load(), _stream()
        K, N1, N2, A = x.shape[0], w1.shape[0], w2.shape[0], w3.shape[0]
        ctx.fused = N1 == N2 == 256 and A <= 4 and x.shape[1] <= 1024 and _m3_shape_ok(K, x.shape[1])
        if ctx.fused:   # qs_mlp3_fwd: both layers and the head on MFMA, activations kept transposed [N][K]
            I = x.shape[1]
            pack = torch.empty(int(lib.qs_mlp3_pack_floats(I)), device=x.device, dtype=torch.float32)
            L.check(lib.qs_mlp3_pack(I, N1, L.ptr(w1), L.ptr(w2), L.ptr(pack), st), "qs_mlp3_pack")
            h1 = torch.empty((N1, K), device=x.device, dtype=x.dtype)
            h2 = torch.empty((N2, K), device=x.device, dtype=x.dtype)
            out = torch.empty((K, A), device=x.device, dtype=x.dtype)
            L.check(lib.qs_mlp3_fwd(K, I, N1, A, L.ptr(x), L.ptr(pack), L.ptr(b1), L.ptr(b2), L.ptr(w3), L.ptr(b3),
                                    L.ptr(h1), L.ptr(h2), L.ptr(out), st), "qs_mlp3_fwd")
            ctx.save_for_backward(x, w1, b1, w2, b2, w3, b3, h1, h2, pack)
            return out
        h1 = torch.mm(x, w1.t())
        L.check(lib.qs_mlp_bias_tanh(K, N1, L.ptr(h1), L.ptr(b1), L.ptr(h1), 0, None, None, None, st), "qs_mlp_bias_tanh")
        h2 = torch.mm(h1, w2.t())
        out = torch.empty((K, A), device=x.device, dtype=x.dtype)
        L.check(lib.qs_mlp_bias_tanh(K, N2, L.ptr(h2), L.ptr(b2), L.ptr(h2), A, L.ptr(w3), L.ptr(b3), L.ptr(out), st),
                "qs_mlp_bias_tanh")
        ctx.save_for_backward(x, w1, b1, w2, b2, w3, b3, h1, h2)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w1, b1, w2, b2, w3, b3, h1, h2 = ctx.saved_tensors[:9]
        lib, st = L.load(), _stream()
        K, N1, N2, A = x.shape[0], w1.shape[0], w2.shape[0], w3.shape[0]
        dout = dout.contiguous()
        if ctx.fused:   # qs_mlp3_bwd: head + tanh backward, dH1ᵀ = W2ᵀ·dZ2ᵀ on MFMA, tanh backward, bias partials
            pack = ctx.saved_tensors[9]
            G = int(lib.qs_mlp3_tiles(K, x.shape[1]))
            dz2 = torch.empty_like(h2)   # [N][K]
            dz1 = torch.empty_like(h1)
            part_a = torch.empty((G, N2 * (1 + A) + A), device=x.device, dtype=torch.float32)
            part_b = torch.empty((G, N1), device=x.device, dtype=torch.float32)
            L.check(lib.qs_mlp3_bwd(K, x.shape[1], N2, A, L.ptr(dout), L.ptr(h1), L.ptr(h2), L.ptr(pack), L.ptr(w3),
                                    L.ptr(dz2), L.ptr(dz1), L.ptr(part_a), L.ptr(part_b), st), "qs_mlp3_bwd")
            _sum_partials(G, part_a.shape[1], part_a, b2.grad, N2, w3.grad, A * N2, b3.grad)
            _sum_partials(G, N1, part_b, b1.grad, N1)
            _splitk_nt(w2.grad, dz2, h1, True)    # dW2 = dZ2ᵀ·H1
            _splitk_nt(w1.grad, dz1, x, False)    # dW1 = dZ1ᵀ·X
            dx = dz1.t() @ w1 if ctx.needs_input_grad[0] else None
            return dx, None, None, None, None, None, None
        G = int(lib.qs_mlp_bwd_blocks(K))
        # head + second tanh: dz2 = (dout·w3) ⊙ (1 − h2²); b2, w3, b3 gradients
        dz2 = torch.empty_like(h2)
        part = torch.empty((G, N2 * (1 + A) + A), device=x.device, dtype=torch.float32)
        L.check(lib.qs_mlp_tanh_bwd(K, N2, None, L.ptr(dout), A, L.ptr(w3), L.ptr(h2), L.ptr(dz2), L.ptr(part), st),
                "qs_mlp_tanh_bwd")
        _sum_partials(G, part.shape[1], part, b2.grad, N2, w3.grad, A * N2, b3.grad)
        dh1 = torch.mm(dz2, w2)
        _splitk_into(w2.grad, dz2, h1)
        # first tanh (in place on dh1): b1 gradient
        part1 = torch.empty((G, N1), device=x.device, dtype=torch.float32)
        L.check(lib.qs_mlp_tanh_bwd(K, N1, L.ptr(dh1), None, 0, None, L.ptr(h1), L.ptr(dh1), L.ptr(part1), st),
                "qs_mlp_tanh_bwd")
        _sum_partials(G, N1, part1, b1.grad, N1)
        _splitk_into(w1.grad, dh1, x)
        dx = dh1 @ w1 if ctx.needs_input_grad[0] else None
        return dx, None, None, None, None, None, None


# (rows K, gradient width M) → minimum rows per split-K chunk of the direct
# iteration's weight gradients (default 1024)
_SPLITK_MIN_ROWS = {}


class _M3Work:
    """Static workspace and launches of one 256-wide tanh MLP (qs_mlp3_fwd / bwd)
    at a fixed batch of K rows, outside autograd: the update iteration drives the
    actor's and the critic's on two streams (MAPPOAgent._iteration_streams).  Same
    kernels and reductions as _TanhMLP3; every buffer, the split-K partials
    included, is allocated once, so the captured graph never allocates and
    nothing is freed while the other stream may still use it."""

    # weight gradients on qs_mlp_wgrad ('w1', 'w2'); default: split-K hipBLASLt GEMMs,
    # measured faster at the bench's sizes (update 2 446 ms vs 2 781 with 'w1')
    wgrad = ()

    def __init__(self, mlp, K, device):
        f0, f1, f2 = mlp.fcs
        lib = L.load()
        self.mlp, self.K, self.I, self.A = mlp, K, f0.in_features, f2.out_features
        f32 = dict(device=device, dtype=torch.float32)
        self.pack = torch.empty(int(lib.qs_mlp3_pack_floats(self.I)), **f32)
        self.h1, self.h2 = torch.empty((256, K), **f32), torch.empty((256, K), **f32)
        self.dz1, self.dz2 = torch.empty((256, K), **f32), torch.empty((256, K), **f32)
        self.out = torch.empty((K, self.A), **f32)
        G = int(lib.qs_mlp3_tiles(K, self.I))
        self.G = G
        self.part_a = torch.empty((G, 256 * (1 + self.A) + self.A), **f32)
        self.part_b = torch.empty((G, 256), **f32)
        # dW1 = dZ1ᵀ·X (and dW2 = dZ2ᵀ·H1 when 'w2' is in wgrad): chunk partials of
        # the MFMA weight-gradient kernel (qs_mlp_wgrad) where it takes the shape;
        # otherwise split-K GEMMs (rows per chunk >= the _SPLITK_MIN_ROWS entry)
        self.C2 = int(lib.qs_mlp_wgrad_chunks(K, 256, 256)) if 'w2' in self.wgrad else 0
        self.C1 = int(lib.qs_mlp_wgrad_chunks(K, 256, self.I)) if 'w1' in self.wgrad else 0
        m2, m1 = _SPLITK_MIN_ROWS.get((K, 256), 1024), _SPLITK_MIN_ROWS.get((K, self.I), 1024)
        self.S2 = self.C2 or _splitk_chunks(K, m2)
        self.S1 = self.C1 or _splitk_chunks(K, m1)
        self.pw2 = torch.empty((self.S2, 256, 256), **f32) if self.S2 > 1 or self.C2 else None
        self.pw1 = torch.empty((self.S1, 256, self.I), **f32) if self.S1 > 1 or self.C1 else None

    def repack(self):
        """The pack image from the current weights (qs_adam_multi_pack keeps it
        current across the update's Adam steps)."""
        f0, f1, _ = self.mlp.fcs
        L.check(L.load().qs_mlp3_pack(self.I, 256, L.ptr(f0.weight), L.ptr(f1.weight), L.ptr(self.pack), _stream()),
                "qs_mlp3_pack")

    def forward(self, x, rows=None, xg=None, group=1):
        """out = MLP(x) (x [K][I]); rows: x is the whole table and batch row r is
        x[rows[r]] (gathered in the kernel, copied to xg); group G > 1: batch row
        r is x[rows[r // G]·G + r % G] (no copy)."""
        lib, st = L.load(), _stream()
        f0, f1, f2 = self.mlp.fcs
        tail = (L.ptr(self.pack), L.ptr(f0.bias), L.ptr(f1.bias), L.ptr(f2.weight), L.ptr(f2.bias), L.ptr(self.h1),
                L.ptr(self.h2), L.ptr(self.out), st)
        if rows is None:
            L.check(lib.qs_mlp3_fwd(self.K, self.I, 256, self.A, L.ptr(x), *tail), "qs_mlp3_fwd")
        elif group > 1:
            L.check(lib.qs_mlp3_fwd_group_rows(self.K, self.I, 256, self.A, L.ptr(x), L.ptr(rows), int(group), *tail),
                    "qs_mlp3_fwd_group_rows")
        else:
            L.check(lib.qs_mlp3_fwd_rows(self.K, self.I, 256, self.A, L.ptr(x), L.ptr(rows), L.ptr(xg), *tail),
                    "qs_mlp3_fwd_rows")
        return self.out

    def forward_value(self, x, rows, xg, ret, D, dv, acc, work):
        """The critic forward over the gathered rows with compute_value_loss's head
        folded in (qs_mlp3_fwd_rows_value): dv = d(value loss)/dv, acc[1] += the loss."""
        lib, st = L.load(), _stream()
        f0, f1, f2 = self.mlp.fcs
        L.check(lib.qs_mlp3_fwd_rows_value(self.K, self.I, int(D), L.ptr(x), L.ptr(rows), L.ptr(xg), L.ptr(self.pack),
                                           L.ptr(f0.bias), L.ptr(f1.bias), L.ptr(f2.weight), L.ptr(f2.bias),
                                           L.ptr(self.h1), L.ptr(self.h2), L.ptr(self.out), L.ptr(ret), L.ptr(dv),
                                           L.ptr(acc), L.ptr(work), st), "qs_mlp3_fwd_rows_value")
        return self.out

    def pack_segment(self, fb):
        """(pack, w1 offset, w2 offset, I) of this MLP inside FlatBuffers fb."""
        f0, f1, _ = self.mlp.fcs
        ids = [id(p) for p in fb.params]
        return (self.pack, fb.offsets[ids.index(id(f0.weight))][0], fb.offsets[ids.index(id(f1.weight))][0], self.I)

    def _splitk(self, dst, a, b, b_rows_are_k, part, S):
        """a·bᵀ over K in S chunks (see _splitk_nt) into the preallocated partials;
        S = 1: dst = a·bᵀ, one GEMM (the direct iteration's .grad views hold
        nothing else: the single-rank qs_mlp_sum_adam never writes them, the
        multi-rank Adam zeroes them)."""
        K = a.shape[1]
        bk = b.t() if b_rows_are_k else b
        if S == 1:
            torch.mm(a, bk, out=dst)
            return None
        a3 = a.view(a.shape[0], S, K // S).transpose(0, 1)
        b3 = b.view(b.shape[0], S, K // S).permute(1, 2, 0) if b_rows_are_k else b.view(S, K // S, -1)
        torch.bmm(a3, b3, out=part)
        return (S, part[0].numel(), part, dst, dst.numel(), None, 0, None)

    def _wgrad(self, dst, at, b, b_transposed, part, C):
        """Chunk partials of dst = atᵀ-contraction (qs_mlp_wgrad), summed later as one task."""
        N, M = part.shape[1], part.shape[2]
        L.check(L.load().qs_mlp_wgrad(self.K, N, M, L.ptr(at), L.ptr(b), int(b_transposed), int(C), L.ptr(part),
                                      _stream()), "qs_mlp_wgrad")
        return (C, N * M, part, dst, dst.numel(), None, 0, None)

    def backward(self, x, dout, tasks, whole=None):
        """Gradients of the parameters' .grad views (+=); the fixed-order partial
        sums are appended to `tasks` (one qs_mlp_sum_partials_multi launch later).
        A weight gradient small enough for one GEMM (S = 1) is accumulated into its
        .grad view directly; that view is appended to `whole` (qs_mlp_sum_adam
        must still visit it: every gradient element is one of its task columns)."""
        lib, st = L.load(), _stream()
        f0, f1, f2 = self.mlp.fcs
        N, A = 256, self.A
        L.check(lib.qs_mlp3_bwd(self.K, self.I, N, A, L.ptr(dout), L.ptr(self.h1), L.ptr(self.h2), L.ptr(self.pack),
                                L.ptr(f2.weight), L.ptr(self.dz2), L.ptr(self.dz1), L.ptr(self.part_a),
                                L.ptr(self.part_b), st), "qs_mlp3_bwd")
        tasks.append((self.G, self.part_a.shape[1], self.part_a, f1.bias.grad, N, f2.weight.grad, A * N, f2.bias.grad))
        tasks.append((self.G, N, self.part_b, f0.bias.grad, N, None, 0, None))
        w2 = (self._wgrad(f1.weight.grad, self.dz2, self.h1, 1, self.pw2, self.C2) if self.C2 else
              self._splitk(f1.weight.grad, self.dz2, self.h1, True, self.pw2, self.S2))    # dW2 = dZ2ᵀ·H1
        w1 = (self._wgrad(f0.weight.grad, self.dz1, x, 0, self.pw1, self.C1) if self.C1 else
              self._splitk(f0.weight.grad, self.dz1, x, False, self.pw1, self.S1))        # dW1 = dZ1ᵀ·X
        for dst, t in ((f1.weight.grad, w2), (f0.weight.grad, w1)):
            if t is not None:
                tasks.append(t)
            elif whole is not None:
                whole.append(dst)


class _F16Work(_M3Work):
    """The shared actor's minibatch step on qs_mlp3f_actor: forward, the policy
    loss head and the backward of every 16-row tile in one launch (the
    activations never leave the registers between the layers), then the
    split-K weight-gradient GEMMs dW2 = dZ2ᵀ·H1, dW1 = dZ1ᵀ·Xa.  Same partial
    rows and reduction tasks as _M3Work.backward."""

    w1_stream = True   # dW1 on a third stream beside dW2 (False: after it, one stream)
    # dW1 inside the fused launch (qs_mlp3f_actor_w1, opt-in): measured slower — C3 235–242 vs
    # 220–222 µs per minibatch, C4 276 vs 245–248 (the epilogue lengthens the launch every
    # other kernel of the minibatch waits on); default: the split-K GEMMs
    fold_w1 = False

    def __init__(self, mlp, K, device):
        f0, f1, f2 = mlp.fcs
        lib = L.load()
        self.mlp, self.K, self.I, self.A = mlp, K, f0.in_features, f2.out_features
        f32 = dict(device=device, dtype=torch.float32)
        self.pack = torch.empty(int(lib.qs_mlp3f_pack_floats(self.I)), **f32)
        self.h1, self.dz1, self.dz2 = (torch.empty((K, 256), **f32) for _ in range(3))   # row-major (qs_mlp3f_actor)
        self.xa = torch.empty((K, self.I), **f32)
        self.G = G = int(lib.qs_mlp3f_tiles(K))
        self.part_a = torch.empty((G, 256 * (1 + self.A) + self.A), **f32)
        self.part_b = torch.empty((G, 256), **f32)
        self.work = torch.zeros(int(lib.qs_mlp3f_work_bytes(K)), dtype=torch.uint8, device=device)
        self.mean = None   # tests: set to a [K][A] tensor to receive the actor output
        # split-K GEMMs for both weight gradients (qs_mlp_wgrad_x measured slower for dW1:
        # 19 µs + a 256-row partial sum vs 15.5 µs at 32 768 rows)
        # dW2: 2 048-row chunks (half the partials of 1 024 at equal GEMM time: the
        # reduction reads 4 MB less per minibatch; measured -3 µs)
        m2, m1 = _SPLITK_MIN_ROWS.get((K, 256), 2048), _SPLITK_MIN_ROWS.get((K, self.I), 1024)
        self.C2 = self.C1 = 0
        self.S2, self.S1 = _splitk_chunks(K, m2), _splitk_chunks(K, m1)
        self.pw2 = torch.empty((self.S2, 256, 256), **f32) if self.S2 > 1 else None
        self.pw1 = torch.empty((self.S1, 256, self.I), **f32) if self.S1 > 1 and not self.fold_w1 else None
        # folded dW1: one [256][I] partial per 128-row workgroup (dZ1 is then never stored)
        self.pw1f = torch.empty((G, 256, self.I), **f32) if self.fold_w1 else None

    def repack(self):
        f0, f1, _ = self.mlp.fcs
        L.check(L.load().qs_mlp3f_pack(self.I, L.ptr(f0.weight), L.ptr(f1.weight), L.ptr(self.pack), _stream()),
                "qs_mlp3f_pack")

    def pack_segment(self, fb):
        pk, w1, w2, I = super().pack_segment(fb)
        return pk, w1, w2, I | L.QS_PACK_F16

    def _splitk_rm(self, dst, dy, x, part, S):
        """dst = dyᵀ·x over K rows (dy [K][N], x [K][M], both row-major) as S row-chunk
        GEMMs into the preallocated partials (S = 1: one GEMM straight into dst)."""
        K = dy.shape[0]
        if S == 1:
            torch.mm(dy.t(), x, out=dst)
            return None
        torch.bmm(dy.view(S, K // S, -1).transpose(1, 2), x.view(S, K // S, -1), out=part)
        return (S, part[0].numel(), part, dst, dst.numel(), None, 0, None)

    def step(self, table, idx, D, actor, rollouts, clip, ent_coef, kl, acc, tasks, whole, after_actor=None):
        """qs_mlp3f_actor over the minibatch's agent rows (env-timesteps idx, D rows
        each, straight from the rollout table), then the weight gradients.
        after_actor(): called right after the fused launch is issued (the caller
        forks work onto another stream behind it)."""
        f0, f1, f2 = self.mlp.fcs
        logstd = actor.logstd
        fold = self.pw1f is not None
        L.check(L.load().qs_mlp3f_actor_w1(
            self.K, self.I, D, self.A, L.ptr(table), L.ptr(idx), L.ptr(self.pack), L.ptr(f0.bias), L.ptr(f1.bias),
            L.ptr(f2.weight), L.ptr(f2.bias), L.ptr(logstd), float(actor.action_scale), L.ptr(rollouts.act),
            L.ptr(rollouts.logp), L.ptr(rollouts.adv_env), float(clip), float(ent_coef), L.ptr(self.xa),
            L.ptr(self.h1), L.ptr(self.dz2), None if fold else L.ptr(self.dz1), L.ptr(self.part_a),
            L.ptr(self.part_b), L.ptr(logstd.grad), L.ptr(kl), L.ptr(acc), L.ptr(self.work), L.ptr(self.mean),
            L.ptr(self.pw1f), _stream()),
            "qs_mlp3f_actor_w1")
        N, A = 256, self.A
        tasks.append((self.G, self.part_a.shape[1], self.part_a, f1.bias.grad, N, f2.weight.grad, A * N, f2.bias.grad))
        tasks.append((self.G, N, self.part_b, f0.bias.grad, N, None, 0, None))
        if after_actor is not None:
            after_actor()
        if fold:
            w2 = self._splitk_rm(f1.weight.grad, self.dz2, self.h1, self.pw2, self.S2)   # dW2 = dZ2ᵀ·H1
            w1 = (self.G, N * self.I, self.pw1f, f0.weight.grad, N * self.I, None, 0, None)
        elif self.w1_stream:
            # dW1's small GEMMs (a few dozen workgroups each) beside dW2's on a third
            # stream; joined before the caller's reductions
            cur = torch.cuda.current_stream()
            if getattr(self, '_s3', None) is None or self._s3.device != cur.device:
                self._s3 = torch.cuda.Stream(device=cur.device)
            self._s3.wait_stream(cur)
            with torch.cuda.stream(self._s3):
                w1 = self._splitk_rm(f0.weight.grad, self.dz1, self.xa, self.pw1, self.S1)   # dW1 = dZ1ᵀ·Xa
            w2 = self._splitk_rm(f1.weight.grad, self.dz2, self.h1, self.pw2, self.S2)   # dW2 = dZ2ᵀ·H1
            cur.wait_stream(self._s3)
        else:
            w2 = self._splitk_rm(f1.weight.grad, self.dz2, self.h1, self.pw2, self.S2)   # dW2 = dZ2ᵀ·H1
            w1 = self._splitk_rm(f0.weight.grad, self.dz1, self.xa, self.pw1, self.S1)    # dW1 = dZ1ᵀ·Xa
        for dst, t in ((f1.weight.grad, w2), (f0.weight.grad, w1)):
            if t is not None:
                tasks.append(t)
            elif whole is not None:
                whole.append(dst)


# the small-minibatch path (qs_ppo_small_step: both nets' forward / backward
# in 16-row tiles, the weight gradients and the Adam steps in two or three
# launches; with several ranks qs_ppo_small_grads + one all-reduce +
# qs_ppo_small_adam) takes minibatches of at most this many actor rows (mb·D,
# at most QS_PPO_SMALL_MAX_ROWS); larger ones run the split-K path
# (_iteration_direct)
# (measured per minibatch through the exchange path, profiles/r05_rank_shapes.txt: the
# tile path at 4 096 / 5 120 / 8 192 actor rows 73 / 120 / 120-133 µs against the direct
# iteration's 317 / 193 / 158-226 µs; at 16 384 rows 185 against 163)
_SMALL_MAX_ROWS = 8192
_SMALL_MAX_IN = 640   # widest net input the tile kernels take (Spiral's 595-wide critic)


def _mlp256(fb, mlp, logstd, w2t, lib_struct, w1p=None):
    """qs_mlp256 of a 256-wide tanh MLP (and the actor's logstd) inside FlatBuffers fb;
    w1p: the padded W1 copy qs_ppo_small_step keeps current (None: no copy)."""
    ids = [id(p) for p in fb.params]
    off = lambda t: fb.offsets[ids.index(id(t))][0] if t is not None else -1
    f0, f1, f2 = mlp.fcs
    q = lib_struct()
    q.params, q.exp_avg, q.exp_avg_sq, q.step = (fb.flat.data_ptr(), fb.exp_avg.data_ptr(), fb.exp_avg_sq.data_ptr(),
                                                 fb.step.data_ptr())
    q.w2t = w2t.data_ptr()
    q.w1, q.b1, q.w2, q.b2, q.w3, q.b3 = (off(f0.weight), off(f0.bias), off(f1.weight), off(f1.bias), off(f2.weight),
                                          off(f2.bias))
    q.logstd = off(logstd)
    q.in_, q.out = f0.in_features, f2.out_features
    q.lr, q.beta1, q.beta2, q.eps = fb.lr, fb.betas[0], fb.betas[1], fb.eps
    q.w1p = w1p.data_ptr() if w1p is not None else None
    return q


# widest actor output the fused actor step takes (qs_mlp3f_actor: A <= 4;
# bench.py --fused-max-a).  Measured on C4's 4-wide VEL actor: 237-250 us per
# minibatch fused vs ~292 on the two-kernel path
_F16_MAX_A = 4


class _CriticTiles:
    """The centralized critic's minibatch step for the direct iteration at any
    size: qs_ppo_critic_tiles (forward, value head, backward in 16-row tiles
    over every CU; the value loss into acc[1]) and the split-K weight gradients
    qs_wgrad_t from its transposed activations.  The partial rows are the
    _M3Work critic's (qs_mlp_sum_adam tasks); the step's W2ᵀ copy is the
    segment's pack (QS_PACK_W2T), so Adam keeps it current."""

    def __init__(self, agent, mb, D):
        lib = L.load()
        mlp = agent.ac.critic.v_net
        f0, f1, f2 = mlp.fcs
        self.mlp, self.mb, self.D, self.I = mlp, mb, D, f0.in_features
        off = (ctypes.c_int64 * L.QS_PPO_SMALL_LAYOUT_N)()
        L.check(lib.qs_ppo_small_layout(mb, D, 0, self.I, 1, off, len(off)), "qs_ppo_small_layout")
        self.nC, KcP, ld = int(off[17]), int(off[19]), int(off[22])
        dev = agent.device
        self.work = torch.zeros(int(off[20]), dtype=torch.uint8, device=dev)
        view = lambda i, *shape: self.work[off[i]:off[i] + 4 * math.prod(shape)].view(torch.float32).view(*shape)
        self.xT, self.h1T, self.dz2T, self.dz1T = (view(4, self.I, ld), view(5, 256, ld), view(6, 256, ld),
                                                   view(7, 256, ld))
        self.ld = ld
        self.part_a, self.part_b = view(10, self.nC, 513), view(11, self.nC, 256)
        self.S = next(d for d in (8, 4, 2, 1) if self.nC % d == 0)
        self.pw1 = torch.empty((self.S, 256, self.I), device=dev)
        self.pw2 = torch.empty((self.S, 256, 256), device=dev)
        self.w2t = torch.empty((256, 256), device=dev)
        self.net = _mlp256(agent.critic_opt, mlp, None, self.w2t, L.QsMlp256)
        self.KcP = KcP
        self.repack()

    def repack(self):
        self.w2t.copy_(self.mlp.fcs[1].weight.t())

    def pack_segment(self, fb):
        ids = [id(p) for p in fb.params]
        f0, f1, _ = self.mlp.fcs
        return (self.w2t, fb.offsets[ids.index(id(f0.weight))][0], fb.offsets[ids.index(id(f1.weight))][0],
                self.I | L.QS_PACK_W2T)

    def step(self, rollouts, idx, acc, tasks):
        lib, st = L.load(), _stream()
        f0, f1, f2 = self.mlp.fcs
        L.check(lib.qs_ppo_critic_tiles(self.mb, self.D, L.ptr(rollouts.obs), L.ptr(idx), L.ptr(rollouts.ret_env),
                                        ctypes.byref(self.net), L.ptr(acc), L.ptr(self.work), st), "qs_ppo_critic_tiles")
        L.check(lib.qs_wgrad_t(self.KcP, self.ld, 256, self.I, L.ptr(self.dz1T), L.ptr(self.xT), self.S,
                               L.ptr(self.pw1), st), "qs_wgrad_t")
        L.check(lib.qs_wgrad_t(self.KcP, self.ld, 256, 256, L.ptr(self.dz2T), L.ptr(self.h1T), self.S,
                               L.ptr(self.pw2), st), "qs_wgrad_t")
        tasks.append((self.nC, 513, self.part_a, f1.bias.grad, 256, f2.weight.grad, 256, f2.bias.grad))
        tasks.append((self.nC, 256, self.part_b, f0.bias.grad, 256, None, 0, None))
        tasks.append((self.S, self.pw1[0].numel(), self.pw1, f0.weight.grad, f0.weight.numel(), None, 0, None))
        tasks.append((self.S, self.pw2[0].numel(), self.pw2, f1.weight.grad, f1.weight.numel(), None, 0, None))


def _f16_ok(mlp):
    """The fused actor step takes actors with inputs <= 128 wide and 1 ..
    _F16_MAX_A outputs (the ONE_D_* actors, Spiral's VEL actor); other widths
    keep the two-kernel path."""
    f0, _, f2 = mlp.fcs
    return 1 <= f2.out_features <= _F16_MAX_A and f0.in_features <= 128


def _m3_shape_ok(K, I):
    """The qs_mlp3_* launchers' row limits: at least one row, [256][K] activations
    and the [K][I] input addressed in 32 bits (larger batches take the GEMM path)."""
    return 0 < K and K * 1024 < 2 ** 31 and K * I * 4 < 2 ** 31


def _m3_ok(mlp, max_in=1024):
    f0, f1, f2 = mlp.fcs
    return (mlp._tanh3 and f0.out_features == 256 and f1.out_features == 256 and f2.out_features <= 4
            and f0.in_features <= max_in and all(p.grad is not None and p.grad.is_contiguous() for p in mlp.parameters()))


class MLP(nn.Module):
    """neural_networks.py:18-54 (nn.Linear default init; init_weights=False there).
    Under autograd with >= 2048 rows the layers take the split-K weight gradient;
    on the GPU with the learner's .grad buffers in place, the two-hidden-layer tanh
    MLP runs as _TanhMLP3."""

    def __init__(self, input_dim, output_dim, hidden_dims=(), act='relu', output_act=None, **kwargs):
        super().__init__()
        dims = [input_dim] + list(hidden_dims) + [output_dim]
        self.fcs = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(dims) - 1)])
        self.act = get_activation(act)
        self.output_act = get_activation(output_act)
        self._tanh3 = act == 'tanh' and output_act is None and len(dims) == 4

    def _fused_ok(self, x):
        if not (self._tanh3 and x.is_cuda and x.dim() == 2 and x.shape[0] >= 2048 and torch.is_grad_enabled()
                and x.dtype == torch.float32):
            return False
        n1, n2, a = self.fcs[0].out_features, self.fcs[1].out_features, self.fcs[2].out_features
        ok_n = (64, 128, 256, 512)
        return (n1 in ok_n and n2 in ok_n and a <= (1 if n2 == 512 else 4)
                and all(p.grad is not None and p.grad.is_contiguous() for p in self.parameters()))

    def _infer_fused(self, x, repack=True):
        """Inference forward (the rollout's batched actor, AG:389-415) through
        qs_mlp3_fwd without the saved activations.  repack=False reuses the
        pack image of the previous call (the rollout graph packs the weights at
        its first control step only: they change between rollouts, not inside
        one)."""
        lib, st = L.load(), _stream()
        f0, f1, f2 = self.fcs
        K, I, A = x.shape[0], x.shape[1], f2.out_features
        pack = getattr(self, '_inf_pack', None)
        if pack is None or pack.device != x.device or pack.numel() != int(lib.qs_mlp3_pack_floats(I)):
            pack = self._inf_pack = torch.empty(int(lib.qs_mlp3_pack_floats(I)), device=x.device, dtype=torch.float32)
            repack = True
        if repack:
            L.check(lib.qs_mlp3_pack(I, 256, L.ptr(f0.weight), L.ptr(f1.weight), L.ptr(pack), st), "qs_mlp3_pack")
        out = torch.empty((K, A), device=x.device, dtype=x.dtype)
        L.check(lib.qs_mlp3_fwd(K, I, 256, A, L.ptr(x), L.ptr(pack), L.ptr(f0.bias), L.ptr(f1.bias), L.ptr(f2.weight),
                                L.ptr(f2.bias), None, None, L.ptr(out), st), "qs_mlp3_fwd")
        return out

    def _infer_ok(self, x):
        return (not torch.is_grad_enabled() and self._tanh3 and x.is_cuda and x.dim() == 2
                and x.dtype == torch.float32 and x.shape[1] <= 1024 and self.fcs[0].out_features == 256
                and self.fcs[1].out_features == 256 and self.fcs[2].out_features <= 4
                and _m3_shape_ok(x.shape[0], x.shape[1]))

    def forward(self, x, repack=True):
        if self._infer_ok(x):
            return self._infer_fused(x.contiguous(), repack)
        if self._fused_ok(x):
            f0, f1, f2 = self.fcs
            return _TanhMLP3.apply(x.contiguous(), f0.weight, f0.bias, f1.weight, f1.bias, f2.weight, f2.bias)
        out = x
        splits = _splitk_chunks(x.shape[0]) if (torch.is_grad_enabled() and x.dim() == 2) else 1
        for i, fc in enumerate(self.fcs):
            out = _LinearSplitK.apply(out, fc.weight, fc.bias, splits) if splits > 1 else fc(out)
            out = self.act(out) if i < len(self.fcs) - 1 else self.output_act(out)
        return out


class Normal(torch.distributions.Normal):
    """distributions.py:9-33: log_prob summed over the last axis (keepdim), entropy summed, mode = mean."""

    def __init__(self, loc, scale):
        super().__init__(loc, scale, validate_args=False)   # validation would force host syncs

    def log_prob(self, actions):
        return super().log_prob(actions).sum(-1, keepdim=True)

    def entropy(self):
        return super().entropy().sum(-1)

    def mode(self):
        return self.mean

    def sample(self, sample_shape=torch.Size()):
        # torch.normal(loc, scale) validates scale >= 0 with a device→host read, which
        # cannot be captured in a graph; loc + scale·ε is the same distribution
        shape = self._extended_shape(sample_shape)
        with torch.no_grad():
            return self.loc.expand(shape) + self.scale.expand(shape) * torch.randn(shape, dtype=self.loc.dtype,
                                                                                 device=self.loc.device)


class MLPActor(nn.Module):
    def __init__(self, obs_dim, act_dim, hidden_dims, activation, discrete=False, action_scale=1.0):
        super().__init__()
        if discrete:
            raise NotImplementedError("discrete actions are not used by the drone tasks")
        self.pi_net = MLP(obs_dim, act_dim, hidden_dims, activation)
        self.discrete = discrete
        self.action_scale = action_scale
        self.logstd = nn.Parameter(-0.5 * torch.ones(act_dim))

    def dist(self, obs):
        return Normal(self.pi_net(obs) * self.action_scale, self.logstd.exp())

    def forward(self, obs, act=None):
        dist = self.dist(obs)
        return dist, (dist.log_prob(act) if act is not None else None)

    def get_scaled_action(self, obs, deterministic=False):
        dist = self.dist(obs)
        return dist.mode() if deterministic else dist.sample()


class CentralizedCritic(nn.Module):
    def __init__(self, global_obs_dim, hidden_dims, activation, include_actions=False, action_dim=0):
        super().__init__()
        self.include_actions = include_actions
        self.v_net = MLP(global_obs_dim + (action_dim if include_actions else 0), 1, hidden_dims, activation)

    def forward(self, global_obs, actions=None):
        x = global_obs.reshape(global_obs.shape[0], -1) if global_obs.dim() == 3 else global_obs
        if self.include_actions and actions is not None:
            x = torch.cat([x, actions.reshape(x.shape[0], -1)], dim=-1)
        return self.v_net(x)


class MAPPOActorCritic(nn.Module):
    def __init__(self, obs_space, act_space, hidden_dims=(64, 64), activation='tanh', share_actor_weights=True,
                 centralized_critic=True, include_actions_in_critic=False, global_state_dim=None, action_scale=1.0):
        super().__init__()
        obs_shape, act_shape = tuple(obs_space.shape), tuple(act_space.shape)
        if len(obs_shape) == 1:
            num_agents, obs_dim = 1, obs_shape[0]
        else:
            num_agents, obs_dim = obs_shape
        act_dim = act_shape[-1]
        if len(act_shape) == 2 and num_agents == 1:
            num_agents = act_shape[0]
        if not share_actor_weights or not centralized_critic:
            raise NotImplementedError("only share_actor_weights=True with centralized_critic=True (the configuration "
                                      "of both reference MAPPO scripts) is implemented")
        self.num_agents, self.obs_dim, self.act_dim = num_agents, obs_dim, act_dim
        self.share_actor_weights, self.centralized_critic = share_actor_weights, centralized_critic
        self.include_actions_in_critic = include_actions_in_critic
        self.action_scale = action_scale
        self.actor = MLPActor(obs_dim, act_dim, list(hidden_dims), activation, False, action_scale)
        gdim = global_state_dim if global_state_dim is not None else num_agents * obs_dim
        self.critic = CentralizedCritic(gdim, list(hidden_dims), activation, include_actions_in_critic,
                                        num_agents * act_dim if include_actions_in_critic else 0)

    def get_actor(self, agent_idx=None):
        return self.actor

    @torch.no_grad()
    def step(self, obs, get_global_obs_fn=None, out=None, repack=True):
        """Batched branch of AG:389-415 on device tensors: obs (E, D, O) or (E·D, O).
        On the GPU with the fused inference MLP: the actor's forward, then one
        qs_policy_sample launch for the sample and its log-probability (the
        same torch.randn draws as the torch path); out = (act, logp) buffers of
        shapes (E, D, A), (E, D, 1) receive them in place (the rollout slot).
        repack: see MLP._infer_fused."""
        shape = obs.shape
        flat = obs.reshape(-1, self.obs_dim)
        if len(shape) == 3:
            E, D = shape[0], shape[1]
        else:
            D = self.num_agents
            E = flat.shape[0] // D
        pi = self.actor.pi_net
        if pi._infer_ok(flat) and self.act_dim <= 4:
            mean = pi(flat.contiguous(), repack)
            K, A = mean.shape
            eps = torch.randn((K, A), dtype=mean.dtype, device=mean.device)
            if out is not None:
                act, logp = out
                if not (act.is_contiguous() and logp.is_contiguous() and act.numel() == K * A and logp.numel() == K
                        and act.dtype == torch.float32 and logp.dtype == torch.float32):
                    raise ValueError("step: out buffers must be contiguous float32 of (E, D, A) and (E, D, 1)")
            else:
                act = torch.empty((E, D, A), dtype=torch.float32, device=mean.device)
                logp = torch.empty((E, D, 1), dtype=torch.float32, device=mean.device)
            L.check(L.load().qs_policy_sample(K, A, L.ptr(mean), L.ptr(self.actor.logstd), float(self.actor.action_scale),
                                              float(self.action_scale), int(self.action_scale != 1.0), L.ptr(eps),
                                              L.ptr(act), L.ptr(logp), _stream()), "qs_policy_sample")
            return act, self._zero_values(E, D, obs.device), logp
        dist = self.actor.dist(flat)
        act = dist.sample()
        if self.action_scale != 1.0:
            act = act * self.action_scale
        logp = dist.log_prob(act)
        act, logp = act.reshape(E, D, -1), logp.reshape(E, D, 1)
        if out is not None:
            out[0].copy_(act)
            out[1].copy_(logp)
        return act, torch.zeros(E, D, 1, device=obs.device), logp

    def _zero_values(self, E, D, device):
        """The per-agent value placeholder of step() (zeros, as the reference's),
        one shared read-only tensor per shape: no fill launch per control step.
        Not cached while a graph is being captured (its memory would belong to
        the graph's pool)."""
        key = (E, D, str(device))
        z = getattr(self, '_zv', None)
        if z is not None and z[0] == key:
            return z[1]
        v = torch.zeros(E, D, 1, device=device)
        if not (v.is_cuda and torch.cuda.is_current_stream_capturing()):
            self._zv = (key, v)
        return v

    @torch.no_grad()
    def act(self, obs):
        """Deterministic actions (dist.mode) for evaluation (AG:425-449)."""
        return self.actor.dist(obs.reshape(-1, self.obs_dim)).mode().reshape(*obs.shape[:-1], self.act_dim)

    def get_value(self, global_obs, actions=None, agent_idx=None):
        return self.critic(global_obs, actions)

    def get_actor_logp(self, obs, act, agent_idx=None):
        return self.actor(obs, act)[1]

    def get_entropy(self, obs, agent_idx=None):
        return self.actor(obs)[0].entropy()


def _flat_len(module):
    """Elements of a module's FlatBuffers: every parameter starts on a 16-byte
    boundary (the MFMA kernels read weight rows as float4), the pads are zeros
    that Adam leaves at zero."""
    return sum((p.numel() + 3) & ~3 for p in module.parameters())


class FlatBuffers:
    """Parameters, gradients and Adam moments of one module in flat fp32 buffers
    (each parameter 16-byte aligned: _flat_len)."""

    def __init__(self, module, lr, betas=(0.9, 0.999), eps=1e-8, grad=None):
        """grad: optional external flat gradient view (MAPPOAgent packs the actor and
        critic gradients plus approx_kl into one buffer, so one all-reduce serves all)."""
        self.params = [p for p in module.parameters()]
        dev = self.params[0].device
        n = _flat_len(module)
        self.n = n
        self.flat = torch.zeros(n, device=dev)
        self.grad = torch.zeros(n, device=dev) if grad is None else grad
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.step = torch.zeros(1, device=dev)
        self._adam_work = torch.zeros(1, dtype=torch.int32, device=dev)   # qs_adam_step's block counter
        self.offsets = []
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            self.offsets.append((off, k))
            off += (k + 3) & ~3
        self.lr, self.betas, self.eps = lr, betas, eps

    def adam(self, gate_val=None, gate_thr=0.0):
        """One gated Adam step and its step-count commit (qs_adam_step, one launch)."""
        if self.flat.device.type != 'cuda':
            raise RuntimeError("FlatBuffers.adam is the HIP qs_adam_step kernel: the parameters must be on the GPU")
        lib = L.load()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(lib.qs_adam_step(self.n, L.ptr(self.flat), L.ptr(self.grad), L.ptr(self.exp_avg),
                                 L.ptr(self.exp_avg_sq), L.ptr(self.step), self.lr, self.betas[0], self.betas[1],
                                 self.eps, L.ptr(gate_val), float(gate_thr), L.ptr(self._adam_work), st),
                "qs_adam_step")

    @staticmethod
    def adam_multi(segs, work, packs=None, zero_grads=False):
        """One gated Adam step of several FlatBuffers in one launch (qs_adam_multi).
        segs: [(buffers, gate_val tensor or None, gate_thr)]; work: device int32[4].
        packs: per segment None or (pack image, W1 offset, W2 offset, I) of a
        256-wide tanh MLP kept current by the step; zero_grads: the gradients are
        zeroed after they are read (qs_adam_multi_pack)."""
        fb0 = segs[0][0]
        if fb0.flat.device.type != 'cuda':
            raise RuntimeError("FlatBuffers.adam_multi is the HIP qs_adam_multi kernel: the parameters must be on the GPU")
        n = len(segs)
        vp = ctypes.c_void_p
        arr = lambda ct, vals: (ct * n)(*vals)
        ptrs = lambda f: arr(vp, [f(s) for s in segs])
        common = (ptrs(lambda s: s[0].flat.data_ptr()), ptrs(lambda s: s[0].grad.data_ptr()),
                  ptrs(lambda s: s[0].exp_avg.data_ptr()), ptrs(lambda s: s[0].exp_avg_sq.data_ptr()),
                  ptrs(lambda s: s[0].step.data_ptr()), arr(ctypes.c_int64, [s[0].n for s in segs]),
                  arr(ctypes.c_float, [s[0].lr for s in segs]), arr(ctypes.c_float, [s[0].betas[0] for s in segs]),
                  arr(ctypes.c_float, [s[0].betas[1] for s in segs]), arr(ctypes.c_float, [s[0].eps for s in segs]),
                  ptrs(lambda s: s[1].data_ptr() if s[1] is not None else None),
                  arr(ctypes.c_float, [s[2] for s in segs]))
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        if packs is None and not zero_grads:
            L.check(L.load().qs_adam_multi(n, *common, L.ptr(work), st), "qs_adam_multi")
            return
        packs = packs or [None] * n
        L.check(L.load().qs_adam_multi_pack(
            n, *common, arr(vp, [p[0].data_ptr() if p else None for p in packs]),
            arr(ctypes.c_int64, [p[1] if p else 0 for p in packs]), arr(ctypes.c_int64, [p[2] if p else 0 for p in packs]),
            arr(ctypes.c_int32, [p[3] if p else 0 for p in packs]), int(bool(zero_grads)), L.ptr(work), st),
            "qs_adam_multi_pack")

    @staticmethod
    def sum_adam(tasks, task_seg, segs, packs, work):
        """The partial-sum tasks (see _flush_sums) and the gated Adam step of segs
        in one launch (qs_mlp_sum_adam): every gradient element of the segments is
        one task column, reduced straight into its Adam update."""
        lib = L.load()
        n, ns = len(tasks), len(segs)
        if n > 16:
            raise ValueError("qs_mlp_sum_adam takes at most 16 tasks")
        vp = ctypes.c_void_p
        arr = lambda ct, vals: (ct * len(vals))(*vals)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(lib.qs_mlp_sum_adam(
            n, arr(ctypes.c_int32, [t[0] for t in tasks]), arr(ctypes.c_int64, [t[1] for t in tasks]),
            arr(vp, [t[2].data_ptr() for t in tasks]), arr(vp, [t[3].data_ptr() for t in tasks]),
            arr(ctypes.c_int64, [t[4] for t in tasks]),
            arr(vp, [t[5].data_ptr() if t[5] is not None else None for t in tasks]),
            arr(ctypes.c_int64, [t[6] for t in tasks]),
            arr(vp, [t[7].data_ptr() if t[7] is not None else None for t in tasks]),
            arr(ctypes.c_int32, task_seg), ns,
            arr(vp, [s[0].flat.data_ptr() for s in segs]), arr(vp, [s[0].grad.data_ptr() for s in segs]),
            arr(vp, [s[0].exp_avg.data_ptr() for s in segs]), arr(vp, [s[0].exp_avg_sq.data_ptr() for s in segs]),
            arr(vp, [s[0].step.data_ptr() for s in segs]), arr(ctypes.c_int64, [s[0].n for s in segs]),
            arr(ctypes.c_float, [s[0].lr for s in segs]), arr(ctypes.c_float, [s[0].betas[0] for s in segs]),
            arr(ctypes.c_float, [s[0].betas[1] for s in segs]), arr(ctypes.c_float, [s[0].eps for s in segs]),
            arr(vp, [s[1].data_ptr() if s[1] is not None else None for s in segs]),
            arr(ctypes.c_float, [s[2] for s in segs]),
            arr(vp, [p[0].data_ptr() if p else None for p in packs]),
            arr(ctypes.c_int64, [p[1] if p else 0 for p in packs]), arr(ctypes.c_int64, [p[2] if p else 0 for p in packs]),
            arr(ctypes.c_int32, [p[3] if p else 0 for p in packs]), L.ptr(work), st), "qs_mlp_sum_adam")

    # torch.optim.Adam state_dict format (checkpoint compatibility, MP:203-229)
    def state_dict(self):
        state = {}
        for i, (off, k) in enumerate(self.offsets):
            if float(self.step.item()) > 0:
                state[i] = {'step': self.step.detach().cpu().reshape(()).clone(),
                            'exp_avg': self.exp_avg[off:off + k].view_as(self.params[i]).detach().clone(),
                            'exp_avg_sq': self.exp_avg_sq[off:off + k].view_as(self.params[i]).detach().clone()}
        group = {'lr': self.lr, 'betas': self.betas, 'eps': self.eps, 'weight_decay': 0, 'amsgrad': False,
                 'maximize': False, 'foreach': None, 'capturable': False, 'differentiable': False, 'fused': None,
                 'params': list(range(len(self.params)))}
        return {'state': state, 'param_groups': [group]}

    def load_state_dict(self, sd):
        g = sd['param_groups'][0]
        self.lr, self.betas, self.eps = g['lr'], tuple(g['betas']), g['eps']
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        self.step.zero_()
        for i, s in sd['state'].items():
            off, k = self.offsets[int(i)]
            self.exp_avg[off:off + k].copy_(s['exp_avg'].reshape(-1))
            self.exp_avg_sq[off:off + k].copy_(s['exp_avg_sq'].reshape(-1))
            self.step.fill_(float(s['step']))


def _dist_world():
    return tdist.get_world_size() if (tdist.is_available() and tdist.is_initialized()) else 1


class MAPPOAgent:
    """AG:501-772 with the update on device (flat buffers, gated HIP Adam, optional graph)."""

    def __init__(self, obs_space, act_space, hidden_dim=256, use_clipped_value=False, clip_param=0.2, target_kl=0.01,
                 entropy_coef=0.01, actor_lr=0.0003, critic_lr=0.001, opt_epochs=10, mini_batch_size=64,
                 activation='tanh', share_actor_weights=True, centralized_critic=True, include_actions_in_critic=False,
                 global_state_dim=None, action_scale=1.0, use_graphs=True, fused_heads=True, device='cuda', **kwargs):
        self.obs_space, self.act_space = obs_space, act_space
        self.use_clipped_value, self.clip_param, self.target_kl = use_clipped_value, clip_param, target_kl
        self.entropy_coef, self.opt_epochs, self.mini_batch_size = entropy_coef, opt_epochs, mini_batch_size
        self.activation = activation
        self.share_actor_weights, self.centralized_critic = share_actor_weights, centralized_critic
        self.include_actions_in_critic = include_actions_in_critic
        self.action_scale = action_scale
        self.use_graphs = use_graphs
        # with several ranks the per-minibatch all-reduce is captured into the update
        # graph too (RCCL collectives are graph-capturable); False: eager iterations
        self.graph_collectives = kwargs.get('graph_collectives', True)
        self._force_allreduce = False   # tests: take the all-reduce path with one rank
        self._kl_div = 1   # what the approx_kl slot holds ÷ the mean (the tile path's exchange: the ranks' sum)
        self.fused_heads = fused_heads   # qs_ppo_heads (False: the loss heads as plain torch ops)
        self.direct = kwargs.get('direct', True)   # the fused MLP kernels without autograd (_iteration_direct)
        # the direct iteration's actor on qs_mlp3f_actor (forward + loss head + backward in one launch)
        self.fused_actor = kwargs.get('fused_actor', True)
        self.side_stream = kwargs.get('side_stream', True)   # critic backward beside the actor's (_iteration_direct)
        # one rank, fused actor: the critic's sums + Adam on the side stream too (its own
        # launch).  Opt-in: measured slower (update 2 077 vs 1 961 ms)
        self.critic_adam_side = kwargs.get('critic_adam_side', False)
        self.side_priority = kwargs.get('side_priority', 0)
        # the critic's value head folded into its forward launch (qs_mlp3_fwd_rows_value)
        self.fused_value_head = kwargs.get('fused_value_head', False)
        # (opt-in) with the fused actor, the critic's step on qs_ppo_critic_tiles +
        # qs_wgrad_t instead of the qs_mlp3w kernels and hipBLASLt weight-gradient
        # GEMMs (measured slower at the C3 shape)
        self.critic_tiles = kwargs.get('critic_tiles', False)
        # ... after the fused actor kernel, beside its weight gradients (False: beside the actor kernel)
        # the critic's chain forked behind the fused actor launch (beside its
        # weight-gradient GEMMs) rather than beside it; None: for the critic tiles
        self.critic_after_actor = kwargs.get('critic_after_actor', None)
        # minibatches of at most _SMALL_MAX_ROWS actor rows on qs_ppo_small_step (one
        # rank); False: always the split-K direct iteration
        self.small = kwargs.get('small', True)
        self.device = torch.device(device)
        self.ac = MAPPOActorCritic(obs_space, act_space, hidden_dims=[hidden_dim] * 2, activation=activation,
                                   share_actor_weights=share_actor_weights, centralized_critic=centralized_critic,
                                   include_actions_in_critic=include_actions_in_critic,
                                   global_state_dim=global_state_dim, action_scale=action_scale)
        self.actor_lr, self.critic_lr = actor_lr, critic_lr
        self._opt_ready = False
        self._graph = None
        self._g_k = 0
        self.to(self.device)

    # ------------------------------------------------------------ plumbing
    def to(self, device):
        self.device = torch.device(device)
        self.ac.to(self.device)
        # The flat buffers exist on any device (the gloo tests drive the multi-rank
        # update on CPU tensors); the optimizer step itself is the HIP kernel.
        na, nc = _flat_len(self.ac.actor), _flat_len(self.ac.critic)
        # [critic grads | actor grads | approx_kl]: the buffer the ranks all-reduce, in
        # one piece (autograd paths) or as two buckets (the direct iteration): the
        # critic's [:nc], reduced while the actor backward still runs, then the
        # actor's with approx_kl [nc:]
        self._reduce_buf = torch.zeros(na + nc + 1, device=self.device)
        self.critic_opt = FlatBuffers(self.ac.critic, self.critic_lr, grad=self._reduce_buf[:nc])
        self.actor_opt = FlatBuffers(self.ac.actor, self.actor_lr, grad=self._reduce_buf[nc:nc + na])
        self._kl = self._reduce_buf[nc + na:]
        self._critic_bucket, self._actor_bucket = self._reduce_buf[:nc], self._reduce_buf[nc:]
        # qs_adam_multi's block counters / qs_mlp_sum_adam's arrival counts (one area per stream)
        nw = max(4, int(L.load().qs_mlp_sum_adam_work_bytes()) // 4) if self.device.type == 'cuda' else 4
        self._adam_work = torch.zeros(nw, dtype=torch.int32, device=self.device)
        self._adam_work_c = torch.zeros(nw, dtype=torch.int32, device=self.device)
        if _dist_world() > 1:   # identical initial weights on every rank
            collectives.broadcast(self.actor_opt.flat, 0)
            collectives.broadcast(self.critic_opt.flat, 0)
        self._opt_ready = True
        self._graph = None

    def release_graphs(self):
        """Free the captured update graph — with several ranks it holds the RCCL
        all-reduces of every minibatch — and its static index / accumulator
        buffers.  Call before the process group is destroyed: tearing the
        communicator down under a live graph that holds its kernels aborted a
        process once (exit 134).  The next update captures again."""
        g, self._graph = self._graph, None
        if g is not None:
            if self.device.type == 'cuda':
                torch.cuda.synchronize(self.device)
            g.reset()
        self._g_perm = self._g_idx = self._g_acc = self._g_rollouts = None
        self._g_k = 0

    def train(self):
        self.ac.train()

    def eval(self):
        self.ac.eval()

    def state_dict(self):
        return {'ac': self.ac.state_dict(), 'actor_opt': self.actor_opt.state_dict(),
                'critic_opt': self.critic_opt.state_dict()}

    def load_state_dict(self, state_dict):
        self.ac.load_state_dict(state_dict['ac'])   # copies into the flat-buffer views in place
        self.actor_opt.load_state_dict(state_dict['actor_opt'])
        self.critic_opt.load_state_dict(state_dict['critic_opt'])
        # a captured update graph has lr / betas / eps baked in as kernel arguments
        self._graph = None
        self._sm_key = None

    # ------------------------------------------------------------- losses
    def compute_policy_loss(self, batch, agent_idx=None):
        """AG:602-640."""
        obs, act, logp_old, adv = batch['obs'], batch['act'], batch['logp'], batch['adv']
        dist = self.ac.actor.dist(obs)
        logp = dist.log_prob(act)
        ratio = torch.exp(logp - logp_old)
        clip_adv = torch.clamp(ratio, 1 - self.clip_param, 1 + self.clip_param) * adv
        policy_loss = -torch.min(ratio * adv, clip_adv).mean()
        entropy_loss = -dist.entropy().mean()   # the reference re-runs the actor; same value
        approx_kl = (logp_old - logp).mean()
        return policy_loss, entropy_loss, approx_kl

    def compute_value_loss(self, batch, agent_idx=None):
        """AG:642-683 (centralized critic, ret averaged over agents)."""
        global_obs, ret = batch['global_obs'], batch['ret']
        v_cur = self.ac.get_value(global_obs, batch.get('act') if self.include_actions_in_critic else None)
        if ret.dim() == 3:
            ret = ret.mean(dim=1, keepdim=True)
        if v_cur.shape != ret.shape:
            ret = ret.reshape(v_cur.shape)
        if self.use_clipped_value:
            v_old = batch.get('v', torch.zeros_like(v_cur)).mean(dim=1) if batch.get('v') is not None else 0 * v_cur
            v_old = v_old.reshape(v_cur.shape)
            v_old_clipped = v_old + (v_cur - v_old).clamp(-self.clip_param, self.clip_param)
            return 0.5 * torch.max((v_cur - ret).pow(2), (v_old_clipped - ret).pow(2)).mean()
        return 0.5 * (v_cur - ret).pow(2).mean()

    # ------------------------------------------------------------- update
    def _fused_heads_ok(self, rollouts):
        """The fused loss heads cover the configuration of both reference MAPPO
        scripts: unclipped value loss, critic on the concatenated obs only."""
        return (self.device.type == 'cuda' and not self.use_clipped_value and not self.include_actions_in_critic
                and getattr(rollouts, 'include_global_state', False) and self.ac.act_dim <= 4)

    def _iteration_fused(self, rollouts, idx, acc):
        """One minibatch with the loss heads in one HIP launch (qs_ppo_heads): the
        same losses and gradients as _iteration; autograd only runs the MLPs."""
        world = _dist_world()
        D, O, A = rollouts.num_agents, rollouts.obs_dim, self.ac.act_dim
        mb = idx.shape[0]
        obs = rollouts.sample_obs(idx)
        mean = self.ac.actor.pi_net(obs.reshape(mb * D, O))
        v = self.ac.critic(obs.reshape(mb, D * O))
        lib = L.load()
        if getattr(self, '_heads_mb', None) != (mb, D, A):
            self._dmean = torch.empty(mb * D, A, device=self.device)
            self._dv = torch.empty(mb, 1, device=self.device)
            self._heads_work = torch.zeros(int(lib.qs_ppo_heads_work_bytes(mb, D)), dtype=torch.uint8,
                                           device=self.device)
            self._heads_mb = (mb, D, A)
        self._reduce_buf.zero_()
        logstd = self.ac.actor.logstd
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.check(lib.qs_ppo_heads(mb, D, A, L.ptr(idx), L.ptr(mean), L.ptr(logstd), float(self.action_scale),
                                 L.ptr(rollouts.act), L.ptr(rollouts.logp), L.ptr(rollouts.adv_env),
                                 L.ptr(rollouts.ret_env), L.ptr(v), float(self.clip_param), float(self.entropy_coef),
                                 L.ptr(self._dmean), L.ptr(logstd.grad), L.ptr(self._dv), L.ptr(self._kl), L.ptr(acc),
                                 L.ptr(self._heads_work), st), "qs_ppo_heads")
        with deferred_sums():
            torch.autograd.backward([mean, v], [self._dmean, self._dv])
        self._exchange_and_step(world)

    def _direct_ok(self):
        return self.direct and _m3_ok(self.ac.actor.pi_net) and _m3_ok(self.ac.critic.v_net)

    def _direct_setup(self, mb, D, O, A):
        lib = L.load()
        if getattr(self, '_ws_key', None) == (mb, D, O, A):
            return
        # the fused actor's own row limit (K·1024 < 2^31, qs_mlp3f_actor) as well as the widths
        f16 = self.fused_actor and _f16_ok(self.ac.actor.pi_net) and _m3_shape_ok(mb * D, O)
        self._ws_actor = (_F16Work if f16 else _M3Work)(self.ac.actor.pi_net, mb * D, self.device)
        pc = self.ac.critic.v_net
        # with the fused actor the critic runs in 16-row tiles over every CU (qs_ppo_critic_tiles);
        # the two-kernel actor path shares qs_ppo_heads' value head with the _M3Work critic
        tiles = f16 and self.critic_tiles and pc.fcs[0].in_features <= 256 and pc.fcs[2].out_features == 1
        self._ws_critic = _CriticTiles(self, mb, D) if tiles else _M3Work(pc, mb, self.device)
        self._vh_work = torch.zeros(int(lib.qs_ppo_heads_work_bytes(mb, D)), dtype=torch.uint8, device=self.device)
        self._fv_work = torch.zeros(int(lib.qs_mlp3_value_work_bytes(mb)), dtype=torch.uint8, device=self.device)
        self._xg = torch.empty((mb, D * O), device=self.device)
        self._dmean = torch.empty(mb * D, A, device=self.device)
        self._dv = torch.empty(mb, 1, device=self.device)
        self._heads_work = torch.zeros(int(lib.qs_ppo_heads_work_bytes(mb, D)), dtype=torch.uint8, device=self.device)
        self._ws_key = (mb, D, O, A)
        self._repack()

    def _repack(self):
        """Pack images from the current weights, and zeroed gradients: the direct
        iteration's Adam keeps both from then on (call after any weight change
        outside the update, e.g. load_state_dict, and before each update)."""
        if getattr(self, '_ws_key', None) is not None:
            self._ws_actor.repack()
            self._ws_critic.repack()
        if getattr(self, '_sm_key', None) is not None:
            self._sm_refresh()
        self._reduce_buf.zero_()

    def _iteration_direct(self, rollouts, idx, acc):
        """One minibatch on the 256-wide fused MLP kernels without autograd, in
        the fewest launches.  With the fused actor (_F16Work): the actor's
        forward, policy loss head and backward in one qs_mlp3f_actor launch plus
        its weight-gradient GEMMs, beside the critic's forward (which gathers the
        minibatch rows itself, qs_mlp3_fwd_rows), value head and backward on the
        second stream; otherwise the two-kernel actor (qs_mlp3_fwd_group_rows /
        qs_mlp3_bwd) around qs_ppo_heads.  Then one launch reduces every partial
        sum straight into the KL-gated Adam step (one rank), or the two-bucket
        exchange and the zeroing Adam (several ranks)."""
        world = _dist_world()
        D, O, A = rollouts.num_agents, rollouts.obs_dim, self.ac.act_dim
        mb = idx.shape[0]
        lib = L.load()
        self._direct_setup(mb, D, O, A)
        T, E = rollouts.max_length, rollouts.batch_size
        xc, xa = self._xg, self._xg.view(mb * D, O)
        logstd = self.ac.actor.logstd
        multi = world > 1 or self._force_allreduce
        ta, tc, wa, wc = [], [], [], []
        cur = torch.cuda.current_stream()
        if self.side_stream and (getattr(self, '_side', None) is None or self._side.device != cur.device):
            # side_priority -1: the critic's stream outranks the actor's, so its next
            # launch is dispatched ahead of the fused actor's queued workgroups
            self._side = torch.cuda.Stream(device=cur.device, priority=self.side_priority)
        fused = isinstance(self._ws_actor, _F16Work)

        def critic_fwd():
            # also writes the gathered copy the weight gradients read
            return self._ws_critic.forward(rollouts.obs.reshape(T * E, D * O), rows=idx, xg=self._xg)

        def critic_bwd(exchange):
            self._ws_critic.backward(xc, self._dv, tc, wc)
            if exchange:   # the critic bucket: its sums and all-reduce
                _flush_sums(tc)
                self._exchange_bucket(self._critic_bucket, world)

        if fused:
            def critic_all(exchange, own_adam=False):
                if isinstance(self._ws_critic, _CriticTiles):
                    self._ws_critic.step(rollouts, idx, acc, tc)
                    if exchange:
                        _flush_sums(tc)
                        self._exchange_bucket(self._critic_bucket, world)
                else:
                    if self.fused_value_head:
                        # the value head inside the critic forward: one launch fewer on the critic's chain
                        self._ws_critic.forward_value(rollouts.obs.reshape(T * E, D * O), idx, self._xg, rollouts.ret_env,
                                                      D, self._dv, acc, self._fv_work)
                    else:
                        v = critic_fwd()
                        L.check(lib.qs_value_head(mb, D, L.ptr(idx), L.ptr(rollouts.ret_env), L.ptr(v),
                                                  L.ptr(self._dv), L.ptr(acc), L.ptr(self._vh_work), _stream()),
                                "qs_value_head")
                    critic_bwd(exchange)
                if own_adam:
                    # the critic's Adam is ungated: its sums and step run here, beside
                    # the actor's weight-gradient GEMMs, not after the join
                    tc.extend((1, g.numel(), g, g, g.numel(), None, 0, None) for g in wc)
                    FlatBuffers.sum_adam(tc, [0] * len(tc), [(self.critic_opt, None, 0.0)],
                                         [self._ws_critic.pack_segment(self.critic_opt)], self._adam_work_c)
                    tc.clear()
                    wc.clear()

            def actor_all(exchange, after_actor=None):
                self._ws_actor.step(rollouts.obs.reshape(T * E * D, O), idx, D, self.ac.actor, rollouts,
                                    self.clip_param, self.entropy_coef, self._kl, acc, ta, wa, after_actor=after_actor)
                if exchange:
                    _flush_sums(ta)
                    self._exchange_bucket(self._actor_bucket, world)

            if self.side_stream:
                own = not multi and self.critic_adam_side
                self._side.wait_stream(cur)
                after = self.critic_after_actor
                if after is None:
                    after = isinstance(self._ws_critic, _CriticTiles)
                if after:
                    # the fused actor holds every CU's whole register file: a critic
                    # running beside it delays its workgroups.  The critic's tiles
                    # follow it instead, beside the actor's weight-gradient GEMMs
                    def fork():
                        self._side.wait_stream(cur)
                        with torch.cuda.stream(self._side):
                            critic_all(multi, own)
                    actor_all(multi, after_actor=fork)
                else:
                    with torch.cuda.stream(self._side):
                        critic_all(multi, own)
                    actor_all(multi)
                cur.wait_stream(self._side)
                if own:
                    for g in [logstd.grad] + wa:
                        ta.append((1, g.numel(), g, g, g.numel(), None, 0, None))
                    gate = self._kl if self.target_kl > 0 else None
                    FlatBuffers.sum_adam(ta, [0] * len(ta), [(self.actor_opt, gate, 1.5 * self.target_kl)],
                                         [self._ws_actor.pack_segment(self.actor_opt)], self._adam_work)
                    return
            else:
                actor_all(False)
                critic_all(False)
                if multi:
                    _flush_sums(ta + tc)
                    self._exchange_bucket(self._critic_bucket, world)
                    self._exchange_bucket(self._actor_bucket, world)
        else:
            if self.side_stream:
                # the critic forward (which also writes the gathered copy the weight
                # gradients read) on the second stream, beside the actor forward, which
                # reads its agent rows straight from the rollout table
                self._side.wait_stream(cur)
                with torch.cuda.stream(self._side):
                    v = critic_fwd()
                mean = self._ws_actor.forward(rollouts.obs.reshape(T * E * D, O), rows=idx, group=D)
                cur.wait_stream(self._side)
            else:
                v = critic_fwd()
                mean = self._ws_actor.forward(xa)
            L.check(lib.qs_ppo_heads(mb, D, A, L.ptr(idx), L.ptr(mean), L.ptr(logstd), float(self.action_scale),
                                     L.ptr(rollouts.act), L.ptr(rollouts.logp), L.ptr(rollouts.adv_env),
                                     L.ptr(rollouts.ret_env), L.ptr(v), float(self.clip_param),
                                     float(self.entropy_coef), L.ptr(self._dmean), L.ptr(logstd.grad),
                                     L.ptr(self._dv), L.ptr(self._kl), L.ptr(acc), L.ptr(self._heads_work), _stream()),
                    "qs_ppo_heads")
            if self.side_stream:
                # the critic's backward (a 128-workgroup kernel at 4 096 rows: half the
                # CUs) and its weight-gradient GEMMs on a second stream, beside the
                # actor's; with several ranks the critic bucket's partial sums and
                # all-reduce follow on that stream, hidden behind the actor backward.
                # Joined before Adam (graph capture records the fork and the join as
                # dependency edges)
                self._side.wait_stream(cur)
                with torch.cuda.stream(self._side):
                    critic_bwd(multi)
                self._ws_actor.backward(xa, self._dmean, ta, wa)
                if multi:
                    _flush_sums(ta)
                    self._exchange_bucket(self._actor_bucket, world)
                cur.wait_stream(self._side)
            else:
                self._ws_actor.backward(xa, self._dmean, ta, wa)
                critic_bwd(False)
                if multi:
                    _flush_sums(ta + tc)
                    self._exchange_bucket(self._critic_bucket, world)
                    self._exchange_bucket(self._actor_bucket, world)
        gate = self._kl if self.target_kl > 0 else None
        segs = [(self.actor_opt, gate, 1.5 * self.target_kl), (self.critic_opt, None, 0.0)]
        packs = [self._ws_actor.pack_segment(self.actor_opt), self._ws_critic.pack_segment(self.critic_opt)]
        if not multi:
            # nothing to exchange: the reductions feed Adam in the same launch; logstd's
            # gradient (written by the loss head) rides along as a one-row task
            # (as do the weight gradients formed by one GEMM straight into .grad)
            for g in [logstd.grad] + wa:
                ta.append((1, g.numel(), g, g, g.numel(), None, 0, None))
            tc += [(1, g.numel(), g, g, g.numel(), None, 0, None) for g in wc]
            FlatBuffers.sum_adam(ta + tc, [0] * len(ta) + [1] * len(tc), segs, packs, self._adam_work)
            return
        FlatBuffers.adam_multi(segs, self._adam_work, packs=packs, zero_grads=True)

    def _small_ok(self, rollouts, mb):
        """The tile path takes the minibatch: both nets 256-wide tanh MLPs with
        <= _SMALL_MAX_IN inputs, <= 4 actor outputs, mb·D <= _SMALL_MAX_ROWS (any
        number of ranks: qs_ppo_small_grads + the all-reduce + qs_ppo_small_adam)."""
        if not (self.small and self.device.type == 'cuda'):
            return False
        pa, pc = self.ac.actor.pi_net, self.ac.critic.v_net
        if not (_m3_ok(pa, _SMALL_MAX_IN) and _m3_ok(pc, _SMALL_MAX_IN) and pc.fcs[2].out_features == 1):
            return False
        rows = mb * rollouts.num_agents
        return 0 < rows <= min(_SMALL_MAX_ROWS, L.QS_PPO_SMALL_MAX_ROWS) and rollouts.obs.is_contiguous()

    def _small_setup(self, mb, D):
        if getattr(self, '_sm_key', None) == (mb, D):
            return
        lib = L.load()
        pa, pc = self.ac.actor.pi_net, self.ac.critic.v_net
        n = int(lib.qs_ppo_small_work_bytes(mb, D, pa.fcs[0].in_features, pc.fcs[0].in_features,
                                            pa.fcs[2].out_features))
        self._sm_work = torch.zeros(n, dtype=torch.uint8, device=self.device)
        self._sm_w2t = [torch.empty((256, 256), device=self.device) for _ in range(2)]
        # W1 padded to whole 16-column quads (zeros past the input width): layer 1's
        # rows read as float4s (scalar clamped loads took ~4x as long)
        self._sm_w1p = [torch.zeros((256, (m.fcs[0].in_features + 15) // 16 * 16), device=self.device)
                        for m in (pa, pc)]
        self._sm_nets = (_mlp256(self.actor_opt, pa, self.ac.actor.logstd, self._sm_w2t[0], L.QsMlp256,
                                 self._sm_w1p[0]),
                         _mlp256(self.critic_opt, pc, None, self._sm_w2t[1], L.QsMlp256, self._sm_w1p[1]))
        self._sm_key = (mb, D)
        self._sm_refresh()

    def _sm_refresh(self):
        """The small path's W2ᵀ and padded W1 copies from the current weights."""
        for w2t, w1p, mlp in zip(self._sm_w2t, self._sm_w1p, (self.ac.actor.pi_net, self.ac.critic.v_net)):
            w2t.copy_(mlp.fcs[1].weight.t())
            w1p[:, :mlp.fcs[0].in_features].copy_(mlp.fcs[0].weight)

    def _iteration_small(self, rollouts, idx, acc):
        """One minibatch on the tile kernels: the actor's forward, policy loss
        head and backward and the critic's forward, value head and backward in
        16-row tiles, then every gradient summed over the minibatch and applied
        by the KL-gated Adam (actor) / Adam (critic) in place (qs_ppo_small_step).
        With several ranks: this rank's gradients and approx_kl
        written into `_reduce_buf` (qs_ppo_small_grads), ONE all-reduce of it
        (critic | actor | approx_kl), and the Adam steps from the sums ÷ the
        world size, gated on the global approx_kl (qs_ppo_small_adam)."""
        D, mb = rollouts.num_agents, idx.shape[0]
        self._small_setup(mb, D)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        na, nc = self._sm_nets
        lib = L.load()
        world = _dist_world()
        head = (mb, D, L.ptr(rollouts.obs), L.ptr(idx), L.ptr(rollouts.act), L.ptr(rollouts.logp),
                L.ptr(rollouts.adv_env), L.ptr(rollouts.ret_env), float(self.action_scale), float(self.clip_param),
                float(self.entropy_coef))
        gate, thr = int(self.target_kl > 0), float(1.5 * self.target_kl)
        if not (world > 1 or self._force_allreduce):
            L.check(lib.qs_ppo_small_step(*head, gate, thr, ctypes.byref(na), ctypes.byref(nc), L.ptr(self._kl),
                                          L.ptr(acc), L.ptr(self._sm_work), st), "qs_ppo_small_step")
            return
        self._kl_div = world   # (the all-reduced approx_kl slot is the ranks' sum: _actor_gate_open)
        L.check(lib.qs_ppo_small_grads(*head, ctypes.byref(na), ctypes.byref(nc), L.ptr(self.actor_opt.grad),
                                       L.ptr(self.critic_opt.grad), L.ptr(self._kl), L.ptr(acc), L.ptr(self._sm_work),
                                       st), "qs_ppo_small_grads")
        collectives.all_reduce(self._reduce_buf)   # one collective: [critic | actor | approx_kl]
        L.check(lib.qs_ppo_small_adam(mb, D, ctypes.byref(na), ctypes.byref(nc), L.ptr(self.actor_opt.grad),
                                      L.ptr(self.critic_opt.grad), float(world), gate, thr, L.ptr(self._kl),
                                      L.ptr(self._sm_work), st), "qs_ppo_small_adam")

    def _iteration(self, batch, acc):
        """One minibatch: actor step (KL-gated on device), critic step, stat accumulation.

        The reference steps the actor, then computes the value loss and steps the
        critic (AG:717-760).  The value loss does not depend on the actor's
        parameters, so both losses are formed first and one backward fills both
        gradient buffers; with several ranks the actor gradient, the critic
        gradient and approx_kl then travel in ONE all-reduce (gradient mean and
        the KL mean every rank gates on, AG:731)."""
        self._local_grads(batch, acc)
        self._exchange_and_step(_dist_world())

    def _local_grads(self, batch, acc):
        """This rank's minibatch: both losses, one backward into `_reduce_buf`'s
        gradient views, approx_kl into its last slot, loss stats into acc."""
        policy_loss, entropy_loss, approx_kl = self.compute_policy_loss(batch)
        value_loss = self.compute_value_loss(batch)
        self._reduce_buf.zero_()
        (policy_loss + self.entropy_coef * entropy_loss + value_loss).backward()
        self._kl.copy_(approx_kl.detach().float().reshape(1))
        acc += torch.stack([policy_loss.detach().double(), value_loss.detach().double(),
                            entropy_loss.detach().double(), approx_kl.detach().double()])

    def _exchange(self, world):
        """The rank exchange of one minibatch iteration.  `_reduce_buf` holds
        [actor grads | critic grads | approx_kl] of this rank's minibatch; one
        all-reduce (sum) and a division by the world size turn it into the
        global-minibatch gradient and the global approx_kl mean (AG:731), so every
        rank evaluates the same KL gate on the same value.  Runs on any device
        (tests/test_distributed_cpu.py drives it on CPU tensors with gloo)."""
        if world > 1 or self._force_allreduce:
            collectives.all_reduce(self._reduce_buf)
            self._reduce_buf.div_(world)

    def _exchange_bucket(self, bucket, world):
        """One bucket of the direct iteration's exchange (critic gradients, or actor
        gradients + approx_kl): all-reduce (sum) and divide by the world size on
        the current stream — the same values as the one-piece `_exchange`."""
        collectives.all_reduce(bucket)
        bucket.div_(world)

    def _actor_gate_open(self):
        """AG:731-734: the actor steps only if approx_kl <= 1.5·target_kl (a device
        tensor; the HIP Adam reads it on the device, this is the host view)."""
        # (after the tile path's exchange the slot holds the ranks' SUM: qs_ppo_small_adam
        # divides it on the device, this host view by _kl_div)
        return self.target_kl <= 0 or bool(self._kl.item() / self._kl_div <= 1.5 * self.target_kl)

    def _optimizer_steps(self):
        """Actor Adam gated by the KL value on the device, critic Adam always
        (AG:731-760): both in one qs_adam_multi launch."""
        gate = self._kl if self.target_kl > 0 else None
        FlatBuffers.adam_multi([(self.actor_opt, gate, 1.5 * self.target_kl), (self.critic_opt, None, 0.0)],
                               self._adam_work)

    def _exchange_and_step(self, world):
        self._exchange(world)
        self._optimizer_steps()

    def _step_minibatch(self, rollouts, idx, acc):
        self._kl_div = 1
        if self.fused_heads and self._fused_heads_ok(rollouts):
            if self._small_ok(rollouts, idx.shape[0]):
                self._iteration_small(rollouts, idx, acc)
            elif self._direct_ok():
                self._iteration_direct(rollouts, idx, acc)
            else:
                self._iteration_fused(rollouts, idx, acc)
        else:
            self._iteration(rollouts.sample(idx), acc)

    @staticmethod
    def _chunk(nmb, cap=128):
        """Minibatch iterations per captured graph: the largest divisor of nmb <= cap."""
        return max(k for k in range(1, min(nmb, cap) + 1) if nmb % k == 0)

    def _capture(self, rollouts, k=1):
        """Capture k consecutive update iterations as one HIP graph over a static
        index buffer (k minibatch slices) and accumulator."""
        mb = self.mini_batch_size
        self._g_perm = torch.zeros(k * mb, dtype=torch.long, device=self.device)
        self._g_idx = self._g_perm[:mb]
        self._g_acc = torch.zeros(4, dtype=torch.float64, device=self.device)
        self._g_rollouts, self._g_k = rollouts, k
        # warm-up on a side stream (torch.cuda.graph requirement), with a snapshot/restore of
        # the parameters and optimizer state so the warm-up leaves no trace
        snap = [t.clone() for t in (self.actor_opt.flat, self.actor_opt.exp_avg, self.actor_opt.exp_avg_sq,
                                    self.actor_opt.step, self.critic_opt.flat, self.critic_opt.exp_avg,
                                    self.critic_opt.exp_avg_sq, self.critic_opt.step)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._step_minibatch(rollouts, self._g_idx, self._g_acc)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local: the RCCL watchdog thread may run during the capture; the
        # captured all-reduces on their own group (capture_collectives)
        with capture_collectives(), torch.cuda.graph(g, capture_error_mode="thread_local"):
            for i in range(k):
                self._step_minibatch(rollouts, self._g_perm[i * mb:(i + 1) * mb], self._g_acc)
        for t, v in zip((self.actor_opt.flat, self.actor_opt.exp_avg, self.actor_opt.exp_avg_sq, self.actor_opt.step,
                         self.critic_opt.flat, self.critic_opt.exp_avg, self.critic_opt.exp_avg_sq,
                         self.critic_opt.step), snap):
            t.copy_(v)
        self._graph = g

    def update(self, rollouts, device='cuda', generator=None):
        """AG:702-772: opt_epochs × minibatches; per-epoch means of the loss stats.
        With graphs, a replay runs k minibatch iterations (one index copy and one
        graph launch per k minibatches)."""
        results = defaultdict(list)
        total_steps = rollouts.max_length * rollouts.batch_size
        mb = self.mini_batch_size
        num_mini_batch = total_steps // mb
        assert num_mini_batch != 0, 'num_mini_batch is 0'
        graphs = self.use_graphs and self.device.type == 'cuda' and (_dist_world() == 1 or self.graph_collectives)
        k = self._chunk(num_mini_batch)
        if graphs and (self._graph is None or self._g_rollouts is not rollouts or self._g_k != k):
            self._capture(rollouts, k)
        self._repack()   # the direct iteration's pack images and zeroed gradients
        per_epoch = []
        for epoch in range(self.opt_epochs):
            perm = torch.randperm(total_steps, device=self.device, generator=generator)
            if graphs:
                self._g_acc.zero_()
                for c in range(num_mini_batch // k):
                    self._g_perm.copy_(perm[c * k * mb:(c + 1) * k * mb])
                    self._graph.replay()
                per_epoch.append(self._g_acc.clone())
            else:
                acc = torch.zeros(4, dtype=torch.float64, device=self.device)
                for i in range(num_mini_batch):
                    self._step_minibatch(rollouts, perm[i * mb:(i + 1) * mb], acc)
                per_epoch.append(acc)
        stats = (torch.stack(per_epoch) / num_mini_batch).cpu()   # one host sync per update
        for j, k in enumerate(['policy_loss', 'value_loss', 'entropy_loss', 'approx_kl']):
            results[k] = float(stats[:, j].mean())
        return dict(results)
