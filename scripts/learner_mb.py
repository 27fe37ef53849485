"""Dev: device time per PPO minibatch of MAPPOAgent.update (graph replays, HIP
events) for learner variants at the bench's shapes, in one process so the
variants are compared on the same box:
  C3   D=8,  O=27,  A=1, mini_batch_size 4096 (32 768 actor rows, 4 096 critic rows)
  ref  D=8,  O=27,  A=1, mini_batch_size 32   (learn_mappo.py:199: 256 actor rows)
  C4   D=5,  O=119, A=4, mini_batch_size 4096 (Spiral VEL)
plus the critic-tile kernels alone at the C3 shape.
plus `ablate`: the C3 minibatch with one piece at a time made a no-op (the
numbers are meaningless then, the time is what the rest costs: the piece's
share of the critical path).
plus `ranks`: SURVEY §8(e)'s per-rank shapes (C3 at G = 2/4/8, C4 at 4, C5 at 8)
through the exchange path on a world-1 process group.
  python scripts/learner_mb.py [C3|ref|C4|kernels|scale|ablate|ranks ...]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-gym-pybullet-drones_amd"))
from gym_pybullet_drones_amd import _lib as L  # noqa: E402
from gym_pybullet_drones_amd.mappo import agent as agent_mod  # noqa: E402
from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent  # noqa: E402
from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer  # noqa: E402
from gym_pybullet_drones_amd.utils.spaces import Box  # noqa: E402

dev = "cuda"
SHAPES = {"C3": (8, 27, 1, 4096, 16, 4096), "ref": (8, 27, 1, 32, 16, 256), "C4": (5, 119, 4, 4096, 16, 4096)}


def per_minibatch_us(shape, reps=3, **variant):
    D, O, A, mb, T, E = SHAPES[shape]
    osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
    torch.manual_seed(0)
    variant.setdefault("use_graphs", True)
    force = variant.pop("force", False)
    agent = MAPPOAgent(osp, asp, hidden_dim=256, opt_epochs=1, mini_batch_size=mb, entropy_coef=0.005,
                       target_kl=1e9, device=dev, **variant)
    agent._force_allreduce = force
    buf = MAPPOBuffer(osp, asp, T, E, include_global_state=True, device=dev)
    buf.next_obs_slots.normal_()
    buf.act.normal_()
    buf.logp.normal_()
    buf.ret_env.normal_()
    buf.adv_env.normal_()
    buf.t, buf.full = 0, True
    agent.update(buf)   # capture + warm
    torch.cuda.synchronize()
    nmb = T * E // mb
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        agent.update(buf)
    e1.record()
    torch.cuda.synchronize()
    path = ("small" if getattr(agent, "_sm_key", None) else
            type(getattr(agent, "_ws_actor", None)).__name__ + "+" + type(getattr(agent, "_ws_critic", None)).__name__)
    agent.release_graphs()
    return e0.elapsed_time(e1) * 1e3 / (reps * nmb), path


# SURVEY §8(e)'s per-rank shapes (bench.py STRONG_LEGS at G ranks): D, O, A, per-rank
# mini_batch_size, T, per-rank envs
RANK_SHAPES = {"C3/2": (8, 27, 1, 2048, 16, 8192), "C3/4": (8, 27, 1, 1024, 16, 4096),
               "C3/8": (8, 27, 1, 512, 16, 2048), "C4/4": (5, 119, 4, 1024, 16, 2048),
               "C5/8": (16, 27, 1, 512, 16, 1024)}
SHAPES.update(RANK_SHAPES)


def world1():
    """A world-1 RCCL process group, so _force_allreduce runs the exchange path."""
    import socket
    import torch.distributed as dist
    if not dist.is_initialized():
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))


def ranks():
    """Per-minibatch device time of each per-rank shape through the exchange path
    (world 1, the all-reduce captured in the graph): the tile path and the split-K
    direct iteration, and the tile path without the exchange."""
    world1()
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
    for shape in RANK_SHAPES:
        for v in (dict(small=True, force=True), dict(small=False, force=True), dict(small=True, force=False)):
            us, path = per_minibatch_us(shape, **v)
            print(f"{shape:5s} {str(v):40s} {us:8.1f} us/minibatch  [{path}]", flush=True)


def timed(fn, reps=40):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 10 * 1e3


def kernels(mb=None):
    """The critic-tile launch and its split-K weight gradients at the C3 shape
    (mb: another minibatch size, to see how the launch scales with its tiles)."""
    D, O, A, mb0, T, E = SHAPES["C3"]
    mb = mb or mb0
    osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
    agent = MAPPOAgent(osp, asp, hidden_dim=256, opt_epochs=1, mini_batch_size=mb, use_graphs=False, device=dev)
    buf = MAPPOBuffer(osp, asp, T, E, include_global_state=True, device=dev)
    buf.next_obs_slots.normal_()
    buf.ret_env.normal_()
    ct = agent_mod._CriticTiles(agent, mb, D)
    idx = torch.randperm(T * E, device=dev)[:mb]
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    lib = L.load()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fl = 2 * mb * (D * O * 256 + 2 * 256 * 256 + 256)
    us = timed(lambda: L.check(lib.qs_ppo_critic_tiles(mb, D, L.ptr(buf.obs), L.ptr(idx), L.ptr(buf.ret_env),
                                                       ctypes.byref(ct.net), L.ptr(acc), L.ptr(ct.work), st()), "t"))
    print(f"qs_ppo_critic_tiles ({mb:5d} x 216)          {us:8.2f} us  {fl / us / 1e6:6.1f} TFLOP/s", flush=True)
    for name, a, b, M, part in (("W1", ct.dz1T, ct.xT, ct.I, ct.pw1), ("W2", ct.dz2T, ct.h1T, 256, ct.pw2)):
        us = timed(lambda: L.check(lib.qs_wgrad_t(ct.KcP, ct.ld, 256, M, L.ptr(a), L.ptr(b), ct.S, L.ptr(part), st()),
                                   "w"))
        print(f"qs_wgrad_t critic {name} S={ct.S}                  {us:8.2f} us  "
              f"{2 * mb * 256 * M / us / 1e6:6.1f} TFLOP/s", flush=True)


def ablate(shape="C3"):
    """Per-minibatch time with each piece removed (a no-op launch)."""
    lib = L.load()
    noop = lambda *a: 0
    M3, F16, FB = agent_mod._M3Work, agent_mod._F16Work, agent_mod.FlatBuffers
    pieces = {
        "actor kernel": [(lib, "qs_mlp3f_actor", noop), (lib, "qs_mlp3f_actor_w1", noop)],
        "actor dW2": [(F16, "_splitk_rm", lambda self, dst, dy, x, part, S:
                       None if dst is self.mlp.fcs[1].weight.grad else ORIG_RM(self, dst, dy, x, part, S))],
        "actor dW1": [(F16, "_splitk_rm", lambda self, dst, dy, x, part, S:
                       None if dst is self.mlp.fcs[0].weight.grad else ORIG_RM(self, dst, dy, x, part, S))],
        "critic (all)": [(lib, "qs_mlp3_fwd_rows", noop), (lib, "qs_value_head", noop), (lib, "qs_mlp3_bwd", noop),
                         (M3, "_splitk", lambda *a: None)],
        "critic GEMMs": [(M3, "_splitk", lambda *a: None)],
        "sum+adam": [(FB, "sum_adam", staticmethod(lambda *a: None))],
        "sums (pre-adam)": [(agent_mod, "_flush_sums", lambda *a: None)],
    }
    global ORIG_RM
    ORIG_RM = F16._splitk_rm
    base, path = per_minibatch_us(shape, critic_tiles=False)
    print(f"ablate {shape} full                       {base:8.1f} us/minibatch  [{path}]", flush=True)
    for name, patches in pieces.items():
        saved = [(o, a, o.__dict__[a] if isinstance(o, type) else getattr(o, a)) for o, a, _ in patches]
        for o, a, f in patches:
            setattr(o, a, f)
        try:
            us, _ = per_minibatch_us(shape, critic_tiles=False)
        finally:
            for o, a, f in saved:
                setattr(o, a, f)
        print(f"ablate {shape} without {name:18s} {us:8.1f} us/minibatch  (share {base - us:6.1f})", flush=True)


def gemms():
    """The fused actor's weight-gradient GEMMs alone (graph-timed), as _F16Work._splitk_rm
    issues them: dW2 = dZ2ᵀ·H1 and dW1 = dZ1ᵀ·Xa over row chunks, at C3's and C4's
    actor rows."""
    for name, K, I in (("C3", 32768, 27), ("C4", 20480, 119)):
        dz = torch.randn((K, 256), device=dev)
        h1 = torch.randn((K, 256), device=dev)
        xa = torch.randn((K, I), device=dev)
        for what, b, m in (("dW2", h1, 2048), ("dW1", xa, 1024)):
            S = agent_mod._splitk_chunks(K, m)
            part = torch.empty((S, 256, b.shape[1]), device=dev)
            fn = lambda: torch.bmm(dz.view(S, K // S, -1).transpose(1, 2), b.view(S, K // S, -1), out=part)
            us = timed(fn)
            print(f"{name} {what} bmm S={S:2d} ({K} x 256 x {b.shape[1]})   {us:8.2f} us  "
                  f"{2 * K * 256 * b.shape[1] / us / 1e6:6.1f} TFLOP/s", flush=True)


def main():
    which = sys.argv[1:] or ["kernels", "C3", "ref", "C4"]
    if "kernels" in which:
        kernels()
    if "base" in which:   # the defaults at C3 and C4 (e.g. to compare two builds via QS_DEV_LIB)
        for shape in ("C3", "C4"):
            us, path = per_minibatch_us(shape)
            print(f"{os.environ.get('QS_DEV_LIB', 'default'):>24s} {shape} default {us:8.1f} us/minibatch  [{path}]",
                  flush=True)
    if "gemms" in which:
        gemms()
    if "scale" in which:
        for mb in (256, 1024, 2048):
            kernels(mb)
    if "C3" in which:
        for v in (dict(critic_tiles=False), dict(critic_tiles=False, side_priority=-1),
                  dict(critic_tiles=False, side_priority=-1, critic_adam_side=True),
                  dict(critic_tiles=False, side_priority=-1, critic_after_actor=True),
                  dict(critic_tiles=False, use_graphs=False), dict(critic_tiles=False, use_graphs=False, side_priority=-1),
                  dict(critic_tiles=False, side_stream=False)):
            us, path = per_minibatch_us("C3", **v)
            print(f"C3  {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "ref" in which:
        for v in (dict(small=True), dict(small=False)):
            us, path = per_minibatch_us("ref", reps=2, **v)
            print(f"ref {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "dw1" in which:
        # dW1's row-chunk GEMMs: rows per chunk (the default: 1 024)
        for m in (256, 512, 1024, 2048):
            agent_mod._SPLITK_MIN_ROWS[(32768, 27)] = m
            us, path = per_minibatch_us("C3", critic_tiles=False)
            print(f"C3  dW1 chunk rows {m:<37d} {us:8.1f} us/minibatch  [{path}]", flush=True)
        agent_mod._SPLITK_MIN_ROWS.pop((32768, 27))
    if "prio" in which:   # the default and side_priority=-1 interleaved (the first variant of a process runs cold)
        for shape in ("C3", "C4"):
            for v in (dict(), dict(side_priority=-1), dict(), dict(side_priority=-1), dict(critic_adam_side=True),
                      dict(side_priority=-1, critic_adam_side=True), dict()):
                us, path = per_minibatch_us(shape, **v)
                print(f"{shape}  {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "ranks" in which:
        ranks()
    if "tiles" in which:   # the tile path alone at the per-rank shapes (QS_SHAPES): exchange path, fused step
        world1()
        agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
        tag = os.path.basename(os.environ.get("QS_DEV_LIB", "default"))
        for shape in os.environ.get("QS_SHAPES", " ".join(RANK_SHAPES)).split():
            for v in (dict(small=True, force=True), dict(small=True, force=False)):
                us, path = per_minibatch_us(shape, **v)
                print(f"{tag:>12s} {shape:5s} {str(v):36s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    for w in which:   # "shape:NAME[:direct|:force]": one shape's tile (or direct) path alone, e.g. under a
        if w.startswith("shape:"):   # kernel trace; force: the tile path's exchange launches (world-1 RCCL group)
            _, name, *rest = w.split(":")
            agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
            force = rest == ["force"]
            if force:
                world1()
            us, path = per_minibatch_us(name, small=rest != ["direct"], force=force)
            mode = "direct" if rest == ["direct"] else ("tile+exchange" if force else "tile")
            print(f"{name:5s} {mode} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "one" in which:   # the default C3 iteration alone (for a kernel trace: scripts/learner_timeline.py)
        us, path = per_minibatch_us("C3")
        print(f"C3  default {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "w1" in which:   # the actor's dW1 beside dW2 on a third stream (default) vs after it, interleaved
        for shape in ("C3", "C4"):
            for w1s in (True, False, True, False, True):
                agent_mod._F16Work.w1_stream = w1s
                us, path = per_minibatch_us(shape)
                print(f"{shape}  w1_stream={w1s!s:48s} {us:8.1f} us/minibatch  [{path}]", flush=True)
        agent_mod._F16Work.w1_stream = True
    if "fold" in which:   # dW1 folded into the fused actor vs the split-K GEMMs (default), interleaved
        for shape in ("C3", "C4"):
            for f in (True, False, True, False):
                agent_mod._F16Work.fold_w1 = f
                us, path = per_minibatch_us(shape)
                print(f"{shape}  fold_w1={f!s:50s} {us:8.1f} us/minibatch  [{path}]", flush=True)
        agent_mod._F16Work.fold_w1 = False
    if "vh" in which:   # the critic's value head folded into its forward vs the separate launch, interleaved
        for shape in ("C3", "C4"):
            for v in (dict(), dict(fused_value_head=True), dict(), dict(fused_value_head=True), dict()):
                us, path = per_minibatch_us(shape, **v)
                print(f"{shape}  {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "C4v" in which:   # learner variants at C4 (critic I = 595)
        for v in (dict(critic_tiles=False), dict(critic_tiles=False, critic_adam_side=True),
                  dict(critic_tiles=False, side_priority=-1), dict(critic_tiles=False, side_stream=False),
                  dict(critic_tiles=False, critic_after_actor=True)):
            us, path = per_minibatch_us("C4", **v)
            print(f"C4  {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "ct" in which:   # the critic on the tile launch (qs_ppo_critic_tiles) vs the 8-wave kernels, interleaved
        for shape in ("C3", "C4"):
            for v in (dict(critic_tiles=False), dict(critic_tiles=True), dict(critic_tiles=False),
                      dict(critic_tiles=True)):
                us, path = per_minibatch_us(shape, **v)
                print(f"{shape}  {str(v):55s} {us:8.1f} us/minibatch  [{path}]", flush=True)
    if "ablate" in which:
        ablate()
    if "ablate4" in which:
        ablate("C4")
    if "C4" in which:
        for a in (1, 4):
            agent_mod._F16_MAX_A = a
            us, path = per_minibatch_us("C4")
            print(f"C4  fused_max_a={a:<43d} {us:8.1f} us/minibatch  [{path}]", flush=True)
        agent_mod._F16_MAX_A = 4


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"({time.time() - t0:.0f} s)")
