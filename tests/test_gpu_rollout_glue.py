"""The rollout's per-step glue on the HIP kernels qs_policy_sample /
qs_rollout_record (csrc/rollout.hip), through the C-ABI, against the torch
expressions they replace (MAPPOActorCritic.step's batched branch,
agent.py:389-415; Normal.log_prob, distributions.py:9-33; MP:818-845's buffer
writes):

* actions from the same torch.randn draws: within 1 ulp-scale (1e-6 absolute
  on O(1) actions; the same float32 operations in the same order);
* log-probabilities: 2e-5 absolute (torch's exp / log and sum order against
  the device library's);
* done / mask / reward: exact;
* MAPPOActorCritic.step on the fused path against its torch path from the
  same generator state, and `out=` writing into a rollout slot.
"""
import ctypes
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_sample(mean, logstd, loc_scale, act_scale, eps):
    loc = mean * loc_scale
    scale = logstd.exp()
    x = loc + scale * eps
    if act_scale != 1.0:
        x = x * act_scale
    var = scale ** 2
    lp = -((x - loc) ** 2) / (2 * var) - scale.log() - math.log(math.sqrt(2 * math.pi))
    return x, lp.sum(-1)


@pytest.mark.parametrize("K,A,s", [(1, 1, 1.0), (257, 1, 0.25), (40960, 4, 0.4), (1000, 2, 1.0), (33, 3, 0.7)])
def test_policy_sample_matches_torch(K, A, s):
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(K + A)
    mean = torch.randn((K, A), device="cuda", generator=g)
    logstd = torch.randn((A,), device="cuda", generator=g) * 0.5
    eps = torch.randn((K, A), device="cuda", generator=g)
    act = torch.full((K, A), float("nan"), device="cuda")
    logp = torch.full((K,), float("nan"), device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.qs_policy_sample(K, A, L.ptr(mean), L.ptr(logstd), s, s, int(s != 1.0), L.ptr(eps), L.ptr(act),
                                 L.ptr(logp), st), "qs_policy_sample")
    ra, rl = _torch_sample(mean, logstd, s, s, eps)
    torch.cuda.synchronize()
    assert torch.allclose(act, ra, rtol=0, atol=1e-6)
    assert torch.allclose(logp, rl, rtol=0, atol=2e-5)


def test_policy_sample_rejects_wide_actions():
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    x = torch.zeros(16, device="cuda")
    rc = lib.qs_policy_sample(2, 5, L.ptr(x), L.ptr(x), 1.0, 1.0, 0, L.ptr(x), L.ptr(x), L.ptr(x), None)
    assert rc != 0 and b"A <= 4" in lib.qs_rollout_last_error()


@pytest.mark.parametrize("E", [1, 255, 16384])
def test_rollout_record_exact(E):
    from gym_pybullet_drones_amd import _lib as L
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(E)
    te = (torch.rand(E, device="cuda", generator=g) < 0.1).to(torch.uint8)
    tr = (torch.rand(E, device="cuda", generator=g) < 0.1).to(torch.uint8)
    rew = torch.randn(E, device="cuda", generator=g)
    rew_dst, mask, done = (torch.full((E,), float("nan"), device="cuda") for _ in range(3))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(lib.qs_rollout_record(E, L.ptr(te), L.ptr(tr), L.ptr(rew), L.ptr(rew_dst), L.ptr(mask), L.ptr(done), st),
            "qs_rollout_record")
    d = (te | tr).float()
    torch.cuda.synchronize()
    assert torch.equal(done, d) and torch.equal(mask, 1 - d) and torch.equal(rew_dst, rew)


@pytest.mark.parametrize("A,s", [(1, 0.25), (4, 0.4)])
def test_actor_critic_step_fused_matches_torch_path(A, s):
    import numpy as np
    from gym_pybullet_drones_amd.mappo.agent import MAPPOActorCritic
    from gym_pybullet_drones_amd.utils.spaces import Box
    E, D, O = 512, 5, 27
    torch.manual_seed(1)
    osp, asp = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O))), Box(-np.ones((D, A)), np.ones((D, A)))
    ac = MAPPOActorCritic(osp, asp, hidden_dims=(256, 256), activation='tanh', action_scale=s).cuda()
    obs = torch.randn((E, D, O), device="cuda")
    rng = torch.cuda.get_rng_state()
    act, _, logp = ac.step(obs)
    # the torch path: the same module, its MLP on the unfused layers
    torch.cuda.set_rng_state(rng)
    with torch.no_grad():
        flat = obs.reshape(-1, O)
        mean = flat
        for i, fc in enumerate(ac.actor.pi_net.fcs):
            mean = fc(mean)
            mean = torch.tanh(mean) if i < 2 else mean
        eps = torch.randn(mean.shape, device="cuda")
        ra, rl = _torch_sample(mean, ac.actor.logstd, s, s, eps)
    assert torch.allclose(act.reshape(-1, A), ra, rtol=0, atol=2e-5)
    assert torch.allclose(logp.reshape(-1), rl, rtol=0, atol=1e-3)
    # out= writes into a rollout slot, the same values from the same draws
    slot_a = torch.zeros((3, E, D, A), device="cuda")
    slot_l = torch.zeros((3, E, D, 1), device="cuda")
    torch.cuda.set_rng_state(rng)
    ac.step(obs, out=(slot_a[1], slot_l[1]), repack=False)
    assert torch.equal(slot_a[1], act) and torch.equal(slot_l[1], logp)
    assert not slot_a[0].any() and not slot_a[2].any()
