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


@pytest.mark.parametrize("E,T,MB", [(16, 8, 64), (64, 16, 512)])
def test_two_ranks_match_one_rank_on_the_global_minibatch(tmp_path, E, T, MB):
    import small_multirank_case as case
    D, world = 8, 2
    port = _port()
    outs = [str(tmp_path / f"r{r}.pt") for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "small_multirank_worker.py"), str(r), str(world),
                               str(port), outs[r], str(E), str(T), str(D), str(MB)], env=env,
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
    got = [torch.load(o, weights_only=True) for o in outs]
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
