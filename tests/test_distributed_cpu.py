"""N>1 paths on CPU with gloo (world_size 2, 127.0.0.1).

* Simulator sharding contract: rank r owns envs [r·E, (r+1)·E) with global env ids
  (env_offset); the union of the shards equals the unsharded run bit for bit, so
  the data path needs no collective (checked with the oracle, which keys its
  Philox streams exactly like the kernel — tests/test_gpu_parity.py shows the
  kernel honours the same contract).
* Learner collectives: global advantage normalisation and the running obs
  moments merged across ranks equal the single-process result on the
  concatenated data; approx_kl / gradient averaging (all_reduce / world) equals
  the gradient of the mean over the global minibatch.
* MAPPOAgent's own update exchange (agent.py _local_grads → _exchange → KL gate,
  the code the GPU path runs, here on CPU tensors): identical initial weights on
  every rank (broadcast), ONE all-reduce of the packed [critic grads | actor
  grads | approx_kl] buffer — or, as the direct iteration exchanges it, two
  buckets (critic, then actor + approx_kl) — whose result is the single-process
  gradient of the global minibatch, and the same KL-gate decision on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


# ------------------------------------------------------------------ workers
def _shard_worker(rank, world):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "oracle")]
    import qs_oracle
    E = 6
    s = qs_oracle.OracleSim(task="multihover", num_envs=E, num_drones=4, act="rpm", precision=8, env_offset=rank * E)
    obs = [s.reset(9)]
    for _ in range(30):
        obs.append(s.step(None)["obs"])
    local = torch.as_tensor(np.stack(obs))
    gathered = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(gathered, local)
    return torch.cat(gathered, dim=1).numpy()


def _adv_worker(rank, world):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "marl-gym-pybullet-drones_amd")]
    from gym_pybullet_drones_amd.mappo.buffer import normalize_advantages
    from gym_pybullet_drones_amd.mappo.normalization import RunningMeanStd
    g = torch.Generator().manual_seed(5)
    full = torch.randn(2 * 40, 3, generator=g, dtype=torch.float64) * 3 + 1
    mine = full[rank * 40:(rank + 1) * 40]
    adv = normalize_advantages(mine)
    rms = RunningMeanStd(shape=(3,))
    rms.update(mine)
    rms.update(mine * 2 + 1)
    return adv.numpy(), rms.mean.numpy(), rms.var.numpy(), float(rms.count)


def _grad_worker(rank, world):
    torch.manual_seed(0)
    net = torch.nn.Linear(5, 2).double()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 5, generator=g, dtype=torch.float64)
    mine = x[rank * 4:(rank + 1) * 4]
    (net(mine) ** 2).mean().backward()
    grad = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    dist.all_reduce(grad)
    grad /= world
    return grad.numpy()


D_, O_, A_, MB_ = 3, 10, 2, 6


def _agent(seed, target_kl):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "marl-gym-pybullet-drones_amd")]
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.utils.spaces import Box
    torch.manual_seed(seed)
    obs_space = Box(np.full((D_, O_), -np.inf, np.float32), np.full((D_, O_), np.inf, np.float32), dtype=np.float32)
    act_space = Box(-np.ones((D_, A_), np.float32), np.ones((D_, A_), np.float32), dtype=np.float32)
    return MAPPOAgent(obs_space, act_space, hidden_dim=16, device="cpu", use_graphs=False, fused_heads=False,
                      target_kl=target_kl, entropy_coef=0.01)


def _update_batch(n):
    g = torch.Generator().manual_seed(3)
    obs = torch.randn(n, D_, O_, generator=g)
    return {"obs": obs, "act": torch.randn(n, D_, A_, generator=g),
            "logp": torch.randn(n, D_, 1, generator=g) * 0.1 - 2.0,
            "adv": torch.randn(n, D_, 1, generator=g, dtype=torch.float64),
            "ret": torch.randn(n, D_, 1, generator=g, dtype=torch.float64),
            "v": torch.zeros(n, D_, 1), "global_obs": obs.reshape(n, D_ * O_)}


def _update_worker_for(target_kl, bucketed=False):
    def work(rank, world):
        agent = _agent(100 + rank, target_kl)   # different init per rank: the broadcast equalises it
        w0 = torch.cat([agent.actor_opt.flat, agent.critic_opt.flat]).clone()
        full = _update_batch(world * MB_)
        mine = {k: v[rank * MB_:(rank + 1) * MB_] for k, v in full.items()}
        acc = torch.zeros(4, dtype=torch.float64)
        agent._local_grads(mine, acc)
        calls = []
        orig = dist.all_reduce

        def counting(t, *a, **kw):
            calls.append(t.numel())
            return orig(t, *a, **kw)

        dist.all_reduce = counting
        try:
            if bucketed:   # _iteration_direct's order: the critic bucket, then actor + approx_kl
                agent._exchange_bucket(agent._critic_bucket, world)
                agent._exchange_bucket(agent._actor_bucket, world)
            else:
                agent._exchange(world)
        finally:
            dist.all_reduce = orig
        return w0.numpy(), agent._reduce_buf.clone().numpy(), agent._actor_gate_open(), calls
    return work


def _upd_worker_open(rank, world):
    return _update_worker_for(10.0)(rank, world)


def _upd_worker_kl(rank, world):
    return _update_worker_for(1e-4)(rank, world)


def _upd_worker_buckets(rank, world):
    return _update_worker_for(10.0, bucketed=True)(rank, world)


def _upd_worker_buckets_kl(rank, world):
    return _update_worker_for(1e-4, bucketed=True)(rank, world)


# -------------------------------------------------------------------- tests
def test_env_shards_union_equals_unsharded():
    import qs_oracle
    parts = spawn(_shard_worker)
    s = qs_oracle.OracleSim(task="multihover", num_envs=12, num_drones=4, act="rpm", precision=8)
    obs = [s.reset(9)]
    for _ in range(30):
        obs.append(s.step(None)["obs"])
    np.testing.assert_array_equal(parts[0], np.stack(obs))
    np.testing.assert_array_equal(parts[1], np.stack(obs))


def test_global_advantage_normalisation_and_obs_moments():
    from gym_pybullet_drones_amd.mappo.buffer import normalize_advantages
    from gym_pybullet_drones_amd.mappo.normalization import RunningMeanStd
    res = spawn(_adv_worker)
    g = torch.Generator().manual_seed(5)
    full = torch.randn(80, 3, generator=g, dtype=torch.float64) * 3 + 1
    want = normalize_advantages(full).numpy()
    np.testing.assert_allclose(np.concatenate([res[0][0], res[1][0]]), want, rtol=1e-12, atol=1e-12)
    rms = RunningMeanStd(shape=(3,))
    rms.update(full)
    rms.update(full * 2 + 1)
    for r in res:
        np.testing.assert_allclose(r[1], rms.mean.numpy(), rtol=1e-12)
        np.testing.assert_allclose(r[2], rms.var.numpy(), rtol=1e-10)
        assert r[3] == pytest.approx(float(rms.count))


def test_gradient_average_equals_global_minibatch_gradient():
    res = spawn(_grad_worker)
    torch.manual_seed(0)
    net = torch.nn.Linear(5, 2).double()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 5, generator=g, dtype=torch.float64)
    (net(x) ** 2).mean().backward()
    want = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).numpy()
    for r in res:
        np.testing.assert_allclose(r, want, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("worker,target_kl,bucketed", [(_upd_worker_open, 10.0, False), (_upd_worker_kl, 1e-4, False),
                                                      (_upd_worker_buckets, 10.0, True),
                                                      (_upd_worker_buckets_kl, 1e-4, True)])
def test_agent_update_exchange_two_ranks(worker, target_kl, bucketed):
    res = spawn(worker)
    single = _agent(100, target_kl)   # rank 0's weights (the broadcast source)
    acc = torch.zeros(4, dtype=torch.float64)
    single._local_grads(_update_batch(2 * MB_), acc)
    want = single._reduce_buf.numpy()
    n = want.size
    for w0, buf, gate, calls in res:
        np.testing.assert_array_equal(w0, res[0][0])   # identical initial weights on both ranks
        np.testing.assert_array_equal(w0, torch.cat([single.actor_opt.flat, single.critic_opt.flat]).numpy())
        nc = single.critic_opt.n
        # one packed all-reduce per minibatch, or the two buckets in the direct iteration's order
        assert calls == ([nc, n - nc] if bucketed else [n])
        np.testing.assert_allclose(buf, want, rtol=2e-5, atol=1e-7)   # = the global-minibatch gradient and KL
        assert gate == single._actor_gate_open()
    assert res[0][2] == res[1][2]
    np.testing.assert_array_equal(res[0][1], res[1][1])   # every rank holds the same reduced values
