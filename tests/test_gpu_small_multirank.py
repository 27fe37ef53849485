"""The tile path across ranks: each rank's
share of a minibatch through qs_ppo_small_grads, the gradient / approx_kl
all-reduce, and qs_ppo_small_adam.

* Two ranks (gloo, both on cuda:0, tests/small_multirank_worker.py) end with
  the same parameters as one rank stepping the union of their minibatches
  through qs_ppo_small_step: the same losses and gradients up to the order of
  the row sums (the global minibatch's mean is the mean of the two halves'
  means), so within Adam's step tolerance, the step counts exact, and both
  ranks bit-identical to each other.  Two sizes: 256 actor rows per rank (one
  K-chunk: launches 1-2) and 2 048 (K-chunks: launches 1-3).
* One rank forced through the exchange (world 1, RCCL all-reduce, captured in
  the update graph or eager) gives qs_ppo_small_step's bits.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, world, E, T, D, MB, gate_closed=False):
    port = _port()
    outs = [str(tmp_path / f"r{r}.pt") for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "small_multirank_worker.py"), str(r), str(world),
                               str(port), outs[r], str(E), str(T), str(D), str(MB), str(int(gate_closed))], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    return [torch.load(o, weights_only=True) for o in outs]


@pytest.mark.parametrize("E,T,MB", [(16, 8, 64), (64, 16, 512)])
def test_two_ranks_match_one_rank_on_the_global_minibatch(tmp_path, E, T, MB):
    import small_multirank_case as case
    D, world = 8, 2
    got = _run_ranks(tmp_path, world, E, T, D, MB)
    for k in got[0]:
        if k != "acc":
            assert torch.equal(got[0][k], got[1][k]), k   # every rank applies the same all-reduced step
    # one rank on the union of the ranks' minibatches (rank 0's rows, then rank 1's)
    El = E // world
    agent, buf = case.build(E, T, D)
    acc = torch.zeros(4, dtype=torch.float64, device="cuda")
    for idx in case.local_minibatches(El, T, MB // world):
        g = torch.cat([case.to_global(idx, r, El, E) for r in range(world)])
        agent._step_minibatch(buf, g.cuda(), acc)
    torch.cuda.synchronize()
    assert agent._sm_key is not None
    want = {k: v.cpu() for k, v in case.snapshot(agent).items()}
    n = case.EPOCHS * case.MB_PER_EPOCH
    assert float(got[0]["actor_step"]) == float(want["actor_step"]) == n
    assert float(got[0]["critic_step"]) == float(want["critic_step"]) == n
    # ulp-level gradient differences (row-sum order) carried by Adam's normalised steps: ~lr/60 per step
    from test_gpu_learner import adam_close
    adam_close(got[0]["actor"], want["actor"], 3e-4, n)
    adam_close(got[0]["critic"], want["critic"], 1e-3, n)
    # the W2ᵀ / padded W1 copies the tile kernels read stayed current on the ranks
    assert bool(got[0]["copies_current"]) and bool(want["copies_current"])
    # per-rank loss statistics are this rank's: their mean over the ranks is the global one
    acc_mean = (got[0]["acc"] + got[1]["acc"]) / world
    for j in (0, 1, 3):   # policy, value, approx_kl (sums of per-minibatch means)
        assert float(acc_mean[j]) == pytest.approx(float(acc[j].cpu()), rel=1e-4, abs=1e-6)


@pytest.mark.parametrize("E,T", [(8, 8), (64, 16)])
@pytest.mark.parametrize("graphs", [False, True])
def test_small_allreduce_path_bit_identical(graphs, E, T):
    """World 1 forced through qs_ppo_small_grads + the RCCL all-reduce +
    qs_ppo_small_adam (÷ 1) gives the bits of qs_ppo_small_step, eagerly and
    with the all-reduce captured in the update graph; at the reference shape
    (256 actor rows, one K-chunk) and at 4 096 actor rows (K-chunks)."""
    import torch.distributed as dist
    from gym_pybullet_drones_amd import _lib as L
    from gym_pybullet_drones_amd.mappo import agent as agent_mod
    from test_gpu_learner import _hidden256_update
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
    keep = agent_mod._SMALL_MAX_ROWS
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
    agents = []
    try:
        a_one, r_one = _hidden256_update(graphs, E, T, small=True)
        a_ar, r_ar = _hidden256_update(graphs, E, T, small=True, force_allreduce=True)
        agents += [a_one, a_ar]
        assert a_one._sm_key is not None and a_ar._sm_key is not None
        for k in ("flat", "exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(getattr(a_one.actor_opt, k), getattr(a_ar.actor_opt, k)), ("actor", k)
            assert torch.equal(getattr(a_one.critic_opt, k), getattr(a_ar.critic_opt, k)), ("critic", k)
        for x, y in zip(a_one._sm_w2t + a_one._sm_w1p, a_ar._sm_w2t + a_ar._sm_w1p):
            assert torch.equal(x, y)
        assert r_one == r_ar
    finally:
        agent_mod._SMALL_MAX_ROWS = keep
        for a in agents:
            a.release_graphs()
        torch.cuda.synchronize()
        if own:
            dist.destroy_process_group()


@pytest.mark.parametrize("E,T,MB", [(16, 8, 64), (64, 16, 512)])
def test_two_ranks_kl_gate_closed(tmp_path, E, T, MB):
    """the multi-rank KL gate with a divisor above 1.  approx_kl ≈
    0.05 on every minibatch against a threshold of 1.5e-4: qs_ppo_small_adam
    reads the two ranks' all-reduced SUM ÷ 2, so a wrong divisor (or a gate
    read off one rank's value) would still close it only by luck of the
    margin — the actor must not step on either rank (parameters, moments and
    step count unchanged), the critic must step every minibatch, both ranks
    bit-identical, and one rank on the union of their minibatches likewise."""
    import small_multirank_case as case
    D, world = 8, 2
    got = _run_ranks(tmp_path, world, E, T, D, MB, gate_closed=True)
    for k in got[0]:
        if k != "acc":
            assert torch.equal(got[0][k], got[1][k]), k
    fresh, _ = case.build(E, T, D, gate_closed=True)   # the seeded initial parameters
    init_actor = fresh.actor_opt.flat.cpu()
    n = case.EPOCHS * case.MB_PER_EPOCH
    assert float(got[0]["actor_step"]) == 0.0 and float(got[0]["critic_step"]) == n
    assert torch.equal(got[0]["actor"], init_actor)
    assert float(got[0]["actor_m"].abs().max()) == 0.0
    assert not torch.equal(got[0]["critic"], fresh.critic_opt.flat.cpu())
    # the per-rank approx_kl (acc[3]: a sum of per-minibatch means) sits at the shift
    for r in range(world):
        assert float(got[r]["acc"][3]) == pytest.approx(n * case.KL_SHIFT, rel=0.05)
    # one rank on the union: the same gate, the same actor (untouched), the critic within Adam's tolerance
    El = E // world
    agent, buf = case.build(E, T, D, gate_closed=True)
    acc = torch.zeros(4, dtype=torch.float64, device="cuda")
    for idx in case.local_minibatches(El, T, MB // world):
        g = torch.cat([case.to_global(idx, r, El, E) for r in range(world)])
        agent._step_minibatch(buf, g.cuda(), acc)
    torch.cuda.synchronize()
    want = {k: v.cpu() for k, v in case.snapshot(agent).items()}
    assert float(want["actor_step"]) == 0.0 and torch.equal(want["actor"], init_actor)
    from test_gpu_learner import adam_close
    adam_close(got[0]["critic"], want["critic"], 1e-3, n)


def test_capture_right_after_eager_allreduce():
    """the update graph (its all-reduce captured) is captured
    immediately after eager all-reduces on a world-1 RCCL group — no
    synchronize, no sleep — three times over, and replays.  The captured
    all-reduce runs on the dedicated capture group (mappo/collectives.py), so
    the RCCL watchdog has no eager work of that group to poll during a capture."""
    import numpy as np
    import torch.distributed as dist
    from gym_pybullet_drones_amd import _lib as L
    from gym_pybullet_drones_amd.mappo import agent as agent_mod
    from gym_pybullet_drones_amd.mappo import collectives
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
    keep = agent_mod._SMALL_MAX_ROWS
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS
    agent = None
    try:
        D, O, A, T, E = 8, 27, 1, 8, 64
        osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
        torch.manual_seed(0)
        agent = MAPPOAgent(osp, asp, hidden_dim=256, opt_epochs=1, mini_batch_size=64, entropy_coef=0.005,
                           target_kl=1e9, device="cuda", small=True)
        agent._force_allreduce = True
        buf = MAPPOBuffer(osp, asp, T, E, include_global_state=True, device="cuda")
        for t in (buf.next_obs_slots, buf.act, buf.logp, buf.ret_env, buf.adv_env):
            t.normal_()
        buf.t, buf.full = 0, True
        x = torch.ones(1 << 16, device="cuda")
        for _ in range(3):
            for _ in range(4):
                dist.all_reduce(x)   # eager, on the default group: still pending in its watchdog
            agent._capture(buf, 1)   # (no synchronize, no sleep)
            assert agent._graph is not None
            agent._graph.replay()
        torch.cuda.synchronize()
        assert agent._sm_key is not None, "the tile path did not take the minibatch"
        assert collectives._CAPTURE_GROUPS, "the capture group was not created"
        assert float(x[0]) == 1.0   # (world 1: the sum of one rank)
    finally:
        agent_mod._SMALL_MAX_ROWS = keep
        if agent is not None:
            agent.release_graphs()
        torch.cuda.synchronize()
        if own:
            dist.destroy_process_group()
