"""Dev: isolated device times (graph replays, HIP events) of the learner's
per-minibatch kernels at the bench's shapes (actor K = 32 768 rows × 27, critic
K = 4 096 × 216, hidden 256): the fused actor step, the weight-gradient
variants for dW1 / dW2, their partial sums, and the critic kernels."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402

lib = L.load()
dev = "cuda"
f32 = dict(device=dev, dtype=torch.float32)


def st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def timed(fn, reps=40, inner=1):
    """Device time per fn() call: reps replays of a graph holding inner calls (a
    graph of one short kernel mostly measures the graph launch: use inner > 1)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / inner * 1e3


def report(name, us, flop=None, byts=None):
    extra = ""
    if flop:
        extra += f"  {flop / us / 1e6:8.1f} TFLOP/s"
    if byts:
        extra += f"  {byts / us / 1e3:8.1f} GB/s"
    print(f"{name:58s} {us:9.2f} us{extra}", flush=True)


def sumadam():
    """The minibatch's qs_mlp_sum_adam launch alone, with the task list the bench's
    direct iteration builds (captured from one update at mb = 4 096, D = 8)."""
    import numpy as np
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent, FlatBuffers
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    D, O, A, T, E = 8, 27, 1, 16, 512
    osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
    agent = MAPPOAgent(osp, asp, hidden_dim=256, opt_epochs=1, mini_batch_size=4096, use_graphs=False, device=dev,
                       critic_adam_side=False)
    buf = MAPPOBuffer(osp, asp, T, E, device=dev, include_global_state=True)
    buf.next_obs_slots.normal_()
    buf.act.normal_()
    buf.logp.normal_()
    buf.ret_env.normal_()
    buf.adv_env.normal_()
    buf.t, buf.full = 0, True
    got = []
    orig = FlatBuffers.sum_adam
    FlatBuffers.sum_adam = staticmethod(lambda *a: (got.append(a), orig(*a))[1])
    agent.update(buf)
    FlatBuffers.sum_adam = staticmethod(orig)
    args = got[0]
    nbytes = sum(t[0] * t[1] * 4 for t in args[0]) + sum(s[0].n for s in args[2]) * 28
    print("tasks (G, P):", [(t[0], t[1]) for t in args[0]])
    report("qs_mlp_sum_adam (minibatch tasks), 1 per graph", timed(lambda: orig(*args)), None, nbytes)
    report("qs_mlp_sum_adam (minibatch tasks), 20 per graph", timed(lambda: orig(*args), 10, 20), None, nbytes)
    empty = torch.empty(1, **f32)
    report("an empty-ish launch (fill_ of one float), 20 per graph", timed(lambda: empty.fill_(1.0), 10, 20))


def main():
    if "sumadam" in sys.argv[1:]:
        return sumadam()
    torch.manual_seed(0)
    K, I, D, A, mb = 32768, 27, 8, 1, 4096
    TE = 256 * 16384 // 64   # a rollout table of 65 536 env-timesteps
    table = torch.randn(TE, D, I, **f32)
    act = torch.randn(TE, D, A, **f32)
    logp = torch.randn(TE, D, **f32) - 1
    adv = torch.randn(TE, device=dev, dtype=torch.float64)
    idx = torch.randperm(TE, device=dev)[:mb]
    W1, b1 = torch.randn(256, I, **f32) * 0.1, torch.zeros(256, **f32)
    W2, b2 = torch.randn(256, 256, **f32) * 0.06, torch.zeros(256, **f32)
    W3, b3 = torch.randn(A, 256, **f32) * 0.06, torch.zeros(A, **f32)
    logstd = torch.full((A,), -0.5, **f32)
    pack = torch.empty(int(lib.qs_mlp3f_pack_floats(I)), **f32)
    L.check(lib.qs_mlp3f_pack(I, L.ptr(W1), L.ptr(W2), L.ptr(pack), st()), "pack")
    G = int(lib.qs_mlp3f_tiles(K))
    xa = torch.empty(K, I, **f32)
    H1, dZ2, dZ1 = (torch.empty(K, 256, **f32) for _ in range(3))   # row-major (qs_mlp3f_actor)
    pA, pB = torch.empty(G, 512 + 1, **f32), torch.empty(G, 256, **f32)
    dls, klo = torch.empty(A, **f32), torch.empty(1, **f32)
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    work = torch.zeros(int(lib.qs_mlp3f_work_bytes(K)), dtype=torch.uint8, device=dev)

    def fused():
        L.check(lib.qs_mlp3f_actor(K, I, D, A, L.ptr(table), L.ptr(idx), L.ptr(pack), L.ptr(b1), L.ptr(b2), L.ptr(W3),
                                   L.ptr(b3), L.ptr(logstd), 1.0, L.ptr(act), L.ptr(logp), L.ptr(adv), 0.2, 0.01,
                                   L.ptr(xa), L.ptr(H1), L.ptr(dZ2), L.ptr(dZ1), L.ptr(pA), L.ptr(pB), L.ptr(dls),
                                   L.ptr(klo), L.ptr(acc), L.ptr(work), None, st()), "fused")
    fl_fused = 2 * K * (32 * 256 + 2 * 256 * 256 + 256)
    report("qs_mlp3f_actor (fwd+head+bwd)", timed(fused), fl_fused)
    fused()
    if hasattr(lib, "qs_mlp3f_stamps"):   # dev stamp build: phase durations of one launch (cycles)
        import numpy as np
        torch.cuda.synchronize()
        fused()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (G * 8 * 8))()
        lib.qs_mlp3f_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        assert lib.qs_mlp3f_stamps(buf, G * 8 * 8) == 0
        st_ = np.frombuffer(buf, dtype=np.uint64).reshape(G * 8, 8).astype(np.int64)
        t0 = st_[:, 0].min()
        names = ["start->L1 done", "epi1", "L2", "head+dZ2", "bwd", "sums+partials"]
        for k, nm in enumerate(names):
            d = st_[:, k + 1] - st_[:, k]
            print(f"  phase {nm:16s} median {np.median(d):9.0f}  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}")
        print(f"  wave start spread {np.percentile(st_[:, 0] - t0, 90):.0f}, end spread (p10..p90 of last stamp) "
              f"{np.percentile(st_[:, 6] - t0, 10):.0f} .. {np.percentile(st_[:, 6] - t0, 90):.0f}")
    if "fused" in sys.argv[1:]:   # PMC passes: the fused kernel only
        return
    # dW1 = dZ1ᵀ·Xa
    dw1 = torch.empty(256, I, **f32)
    for S in (8, 16, 32, 64):
        part = torch.empty(S, 256, I, **f32)
        a3 = dZ1.view(S, K // S, 256).transpose(1, 2)
        b3_ = xa.view(S, K // S, I)

        def bmm_dw1():
            torch.bmm(a3, b3_, out=part)
        report(f"dW1 split-K bmm S={S}", timed(bmm_dw1), 2 * K * 256 * I, 4 * K * (256 + I))

        def sum_dw1():
            L.check(lib.qs_mlp_sum_partials(S, 256 * I, L.ptr(part), L.ptr(dw1), 256 * I, None, 0, None, st()), "sum")
        report(f"   its partial sum (S={S})", timed(sum_dw1))
    for S in (16, 32, 64):
        part = torch.empty(S, 256, 256, **f32)
        a3 = dZ2.view(S, K // S, 256).transpose(1, 2)
        b3_ = H1.view(S, K // S, 256)

        def bmm_dw2():
            torch.bmm(a3, b3_, out=part)
        report(f"dW2 split-K bmm S={S}", timed(bmm_dw2), 2 * K * 256 * 256, 8 * K * 256)
    dZ1 = dZ1.t().contiguous()   # [256][K] for the qs_mlp_wgrad* variants below
    H1 = H1.t().contiguous()
    dZ2 = dZ2.t().contiguous()
    Cx = int(lib.qs_mlp_wgrad_x_chunks(K, I))
    partx = torch.empty(Cx, 256, I, **f32)

    def wgx_dw1():
        L.check(lib.qs_mlp_wgrad_x(K, 256, I, L.ptr(dZ1), 0, L.ptr(xa), L.ptr(partx), st()), "wgrad_x")
    report(f"dW1 qs_mlp_wgrad_x C={Cx}", timed(wgx_dw1), 2 * K * 256 * I, 4 * K * (256 + I))

    def sum_x():
        L.check(lib.qs_mlp_sum_partials(Cx, 256 * I, L.ptr(partx), L.ptr(dw1), 256 * I, None, 0, None, st()), "sum")
    report(f"   its partial sum (C={Cx})", timed(sum_x))
    for C in (32, 64, 128, 256):
        if K % (64 * C):
            continue
        part = torch.empty(C, 256, I, **f32)

        def wg_dw1():
            L.check(lib.qs_mlp_wgrad(K, 256, I, L.ptr(dZ1), L.ptr(xa), 0, C, L.ptr(part), st()), "wgrad")
        report(f"dW1 qs_mlp_wgrad C={C}", timed(wg_dw1), 2 * K * 256 * I, 4 * K * (256 + I))
    # dW2 = dZ2ᵀ·H1
    for C in (16, 32, 64):
        part = torch.empty(C, 256, 256, **f32)

        def wg_dw2():
            L.check(lib.qs_mlp_wgrad(K, 256, 256, L.ptr(dZ2), L.ptr(H1), 1, C, L.ptr(part), st()), "wgrad")
        report(f"dW2 qs_mlp_wgrad C={C}", timed(wg_dw2), 2 * K * 256 * 256, 8 * K * 256)
    # critic: forward (gathering its rows), backward, its weight gradients
    Kc, Ic = mb, D * I
    W1c = torch.randn(256, Ic, **f32) * 0.05
    packc = torch.empty(int(lib.qs_mlp3_pack_floats(Ic)), **f32)
    L.check(lib.qs_mlp3_pack(Ic, 256, L.ptr(W1c), L.ptr(W2), L.ptr(packc), st()), "pack")
    xg = torch.empty(Kc, Ic, **f32)
    h1c, h2c, z1c, z2c = (torch.empty(256, Kc, **f32) for _ in range(4))
    outc = torch.empty(Kc, 1, **f32)
    tab = table.view(TE, D * I)

    def cfwd():
        L.check(lib.qs_mlp3_fwd_rows(Kc, Ic, 256, 1, L.ptr(tab), L.ptr(idx), L.ptr(xg), L.ptr(packc), L.ptr(b1),
                                     L.ptr(b2), L.ptr(W3[:1]), L.ptr(b3[:1]), L.ptr(h1c), L.ptr(h2c), L.ptr(outc),
                                     st()), "cfwd")
    fl_c = 2 * Kc * (Ic * 256 + 256 * 256 + 256)
    report("critic qs_mlp3_fwd_rows (4096 x 216)", timed(cfwd), fl_c)
    cfwd()
    Gc = int(lib.qs_mlp3_tiles(Kc, Ic))
    pAc, pBc = torch.empty(Gc, 513, **f32), torch.empty(Gc, 256, **f32)
    dv = torch.randn(Kc, 1, **f32) / Kc

    def cbwd():
        L.check(lib.qs_mlp3_bwd(Kc, Ic, 256, 1, L.ptr(dv), L.ptr(h1c), L.ptr(h2c), L.ptr(packc), L.ptr(W3[:1]),
                                L.ptr(z2c), L.ptr(z1c), L.ptr(pAc), L.ptr(pBc), st()), "cbwd")
    report("critic qs_mlp3_bwd", timed(cbwd), 2 * Kc * 256 * 256)
    for S in (4, 8):
        part2 = torch.empty(S, 256, 256, **f32)
        a3 = z2c.view(256, S, Kc // S).transpose(0, 1)
        b3_ = h1c.view(256, S, Kc // S).permute(1, 2, 0)
        report(f"critic dW2 split-K bmm S={S}", timed(lambda: torch.bmm(a3, b3_, out=part2)), 2 * Kc * 256 * 256)
        part1 = torch.empty(S, 256, Ic, **f32)
        a1 = z1c.view(256, S, Kc // S).transpose(0, 1)
        b1_ = xg.view(S, Kc // S, Ic)
        report(f"critic dW1 split-K bmm S={S}", timed(lambda: torch.bmm(a1, b1_, out=part1)), 2 * Kc * 256 * Ic)
    Cc = int(lib.qs_mlp_wgrad_x_chunks(Kc, Ic))
    pxc = torch.empty(Cc, 256, Ic, **f32)
    report(f"critic dW1 qs_mlp_wgrad_x C={Cc}",
           timed(lambda: L.check(lib.qs_mlp_wgrad_x(Kc, 256, Ic, L.ptr(z1c), 0, L.ptr(xg), L.ptr(pxc), st()), "wx")),
           2 * Kc * 256 * Ic)


if __name__ == "__main__":
    main()
