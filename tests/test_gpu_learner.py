"""On-device learner kernels and the MAPPO update, through the C-ABI.

* qs_gae vs the oracle's restatement of _compute_single_agent_returns (float32, as the
  reference evaluates it under numpy 2): bit for bit.
* qs_adam_gated vs torch.optim.Adam (the reference's optimizer): 2e-6 relative, and
  an exact no-op when the KL gate is closed.
* one PPO minibatch update of MAPPOAgent vs a pure-torch restatement of
  MAPPOAgent.update (agent.py:702-772) from identical weights and data: losses 1e-5
  relative; parameters within lr/60 absolute (Adam's first step is ≈ lr·sign(g), so
  ulp-level gradient differences on near-zero gradients move a weight by a few 1e-6).
"""
import numpy as np
import pytest
import torch

import qs_oracle

pytestmark = pytest.mark.gpu


def test_gae_kernel_matches_oracle():
    from gym_pybullet_drones_amd.mappo.buffer import gae
    rng = np.random.default_rng(3)
    T, N = 37, 1000
    rews = rng.normal(size=(T, N)).astype(np.float32)
    vals = rng.normal(size=(T, N)).astype(np.float32)
    masks = (rng.random((T, N)) > 0.05).astype(np.float32)
    tv = rng.normal(size=(T, N)).astype(np.float32) * (rng.random((T, N)) > 0.9)
    lv = rng.normal(size=N).astype(np.float32)
    for use_gae in (True, False):
        want_r, want_a = qs_oracle.gae(rews, vals, masks, tv, lv, gamma=0.99, use_gae=use_gae, lam=0.95)
        d = lambda x: torch.as_tensor(x, device="cuda")
        got_r, got_a = gae(d(rews), d(vals), d(masks), d(tv), d(lv), 0.99, use_gae, 0.95)
        np.testing.assert_array_equal(got_r.cpu().numpy(), want_r)   # the same float32 operations, bit for bit
        np.testing.assert_array_equal(got_a.cpu().numpy(), want_a)


def test_gated_adam_matches_torch_adam():
    from gym_pybullet_drones_amd.mappo.agent import FlatBuffers
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.Tanh(), torch.nn.Linear(33, 3)).cuda()
    ref = torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.Tanh(), torch.nn.Linear(33, 3)).cuda()
    ref.load_state_dict(net.state_dict())
    fb = FlatBuffers(net, lr=3e-4)
    opt = torch.optim.Adam(ref.parameters(), 3e-4)
    x = torch.randn(64, 7, device="cuda")
    for it in range(25):
        fb.grad.zero_()
        (net(x) ** 2).mean().backward()
        opt.zero_grad()
        (ref(x) ** 2).mean().backward()
        closed = it % 5 == 4
        kl = torch.tensor([0.5 if closed else 0.001], device="cuda")
        before = fb.flat.clone()
        fb.adam(kl, 0.015)
        if closed:
            assert torch.equal(before, fb.flat)
        else:
            opt.step()
    torch.cuda.synchronize()
    for p, q in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=2e-6, atol=2e-7)
    assert int(fb.step.item()) == 20
    sd = fb.state_dict()
    sd_ref = opt.state_dict()
    for i in sd_ref['state']:
        torch.testing.assert_close(sd['state'][i]['exp_avg'], sd_ref['state'][i]['exp_avg'], rtol=1e-5, atol=1e-9)


def test_adam_multi_matches_torch_adam():
    """qs_adam_multi: two flat buffers (the actor's, KL-gated, and the critic's) in one
    launch, each equal to its own torch.optim.Adam (AG:731-760)."""
    from gym_pybullet_drones_amd.mappo.agent import FlatBuffers
    torch.manual_seed(1)
    mk = lambda i, o: torch.nn.Sequential(torch.nn.Linear(i, 300), torch.nn.Tanh(), torch.nn.Linear(300, o)).cuda()
    nets = [mk(7, 3), mk(11, 1)]
    refs = [mk(7, 3), mk(11, 1)]
    for n, r in zip(nets, refs):
        r.load_state_dict(n.state_dict())
    fbs = [FlatBuffers(nets[0], lr=3e-4), FlatBuffers(nets[1], lr=1e-3, betas=(0.8, 0.99), eps=1e-6)]
    opts = [torch.optim.Adam(refs[0].parameters(), 3e-4), torch.optim.Adam(refs[1].parameters(), 1e-3,
                                                                           betas=(0.8, 0.99), eps=1e-6)]
    work = torch.zeros(4, dtype=torch.int32, device="cuda")
    xs = [torch.randn(64, 7, device="cuda"), torch.randn(64, 11, device="cuda")]
    for it in range(25):
        for fb, n, r, o, x in zip(fbs, nets, refs, opts, xs):
            fb.grad.zero_()
            (n(x) ** 2).mean().backward()
            o.zero_grad()
            (r(x) ** 2).mean().backward()
        closed = it % 5 == 4
        kl = torch.tensor([0.5 if closed else 0.001], device="cuda")
        before = fbs[0].flat.clone()
        FlatBuffers.adam_multi([(fbs[0], kl, 0.015), (fbs[1], None, 0.0)], work)
        opts[1].step()
        if closed:
            assert torch.equal(before, fbs[0].flat)
        else:
            opts[0].step()
    torch.cuda.synchronize()
    for n, r in zip(nets, refs):
        for p, q in zip(n.parameters(), r.parameters()):
            torch.testing.assert_close(p, q, rtol=2e-6, atol=2e-7)
    assert int(fbs[0].step.item()) == 20 and int(fbs[1].step.item()) == 25
    assert int(work.abs().sum()) == 0


def _reference_update(actor, critic, logstd, batch, clip=0.2, ent=0.005, target_kl=0.01, alr=3e-4, clr=1e-3):
    """agent.py:602-772 restated with plain torch + torch.optim.Adam, one minibatch."""
    aopt = torch.optim.Adam(list(actor.parameters()) + [logstd], alr)
    copt = torch.optim.Adam(critic.parameters(), clr)
    obs, act, logp_old, adv = batch['obs'], batch['act'], batch['logp'], batch['adv']
    dist = torch.distributions.Normal(actor(obs), logstd.exp())
    logp = dist.log_prob(act).sum(-1, keepdim=True)
    ratio = torch.exp(logp - logp_old)
    clip_adv = torch.clamp(ratio, 1 - clip, 1 + clip) * adv
    policy_loss = -torch.min(ratio * adv, clip_adv).mean()
    dist2 = torch.distributions.Normal(actor(obs), logstd.exp())
    entropy_loss = -dist2.entropy().sum(-1).mean()
    approx_kl = (logp_old - logp).mean()
    if approx_kl <= 1.5 * target_kl:
        aopt.zero_grad()
        (policy_loss + ent * entropy_loss).backward()
        aopt.step()
    v = critic(batch['global_obs'])
    ret = batch['ret'].mean(dim=1, keepdim=True).view(v.shape)
    value_loss = 0.5 * (v - ret).pow(2).mean()
    copt.zero_grad()
    value_loss.backward()
    copt.step()
    return policy_loss.item(), value_loss.item(), approx_kl.item()


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("graphs", [False, True])
def test_ppo_minibatch_update_matches_reference(graphs, fused):
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    torch.manual_seed(1)
    E, D, O, A, T = 8, 3, 27, 1, 4
    obs_space = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O)))
    act_space = Box(-np.ones((D, A)), np.ones((D, A)))
    agent = MAPPOAgent(obs_space, act_space, hidden_dim=32, opt_epochs=1, mini_batch_size=T * E, entropy_coef=0.005,
                       use_graphs=graphs, fused_heads=fused, device="cuda")
    # a pure-torch copy of the initial weights
    import copy
    actor = copy.deepcopy(agent.ac.actor.pi_net)
    logstd = torch.nn.Parameter(agent.ac.actor.logstd.detach().clone())
    critic = copy.deepcopy(agent.ac.critic.v_net)
    buf = MAPPOBuffer(obs_space, act_space, T, E, include_global_state=True, device="cuda")
    buf.next_obs_slots.normal_()
    buf.act.normal_()
    with torch.no_grad():
        d = agent.ac.actor.dist(buf.obs.reshape(-1, O))
        buf.logp.copy_(d.log_prob(buf.act.reshape(-1, A)).reshape(T, E, D, 1) + 0.001 * torch.randn(T, E, D, 1,
                                                                                                     device="cuda"))
    buf.ret_env.normal_()
    buf.adv_env.normal_()
    buf.t, buf.full = 0, True
    # the reference samples a permutation; use the identity order on both sides
    batch = buf.sample(torch.arange(T * E, device="cuda"))
    want = _reference_update(actor, critic, logstd, {k: v.clone() for k, v in batch.items()})
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    res = agent.update(buf, generator=None) if not graphs else None
    if graphs:
        # graphs: replay with a fixed identity permutation through the static index
        agent._capture(buf)
        agent._g_idx.copy_(torch.arange(T * E, device="cuda"))
        agent._g_acc.zero_()
        agent._graph.replay()
        torch.cuda.synchronize()
        res = {'policy_loss': float(agent._g_acc[0]), 'value_loss': float(agent._g_acc[1]),
               'approx_kl': float(agent._g_acc[3])}
    assert res['policy_loss'] == pytest.approx(want[0], rel=1e-5, abs=1e-6)
    assert res['value_loss'] == pytest.approx(want[1], rel=1e-5, abs=1e-6)
    for p, q in zip(agent.ac.actor.pi_net.parameters(), actor.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=3e-4 / 60)
    torch.testing.assert_close(agent.ac.actor.logstd, logstd, rtol=0, atol=3e-4 / 60)
    for p, q in zip(agent.ac.critic.v_net.parameters(), critic.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=1e-3 / 60)


def adam_close(got, want, lr, steps):
    """Parameters after `steps` Adam steps from gradients that agree to fp32
    rounding (another row-sum order): within lr/60 per step, except where a
    gradient element is near zero — Adam's m/√v then turns its rounding into a
    step of up to ~lr (m and √v of comparable size at any scale) — so a handful
    of elements (≤ 1e-4 of them) may differ by up to the steps' full size."""
    d = (got - want).abs()
    assert float(d.max()) <= steps * lr * 1.01, float(d.max())
    far = int((d > steps * lr / 60).sum())
    assert far <= max(3, int(1e-4 * d.numel())), (far, d.numel())


def _hidden256_update(graphs, E=32, T=8, force_allreduce=False, D=8, A=1, logp_shift=0.0, run=True, O=27, **variant):
    """Two epochs x two minibatches of the 256-wide MAPPO update (the direct
    iteration's configuration) from fixed weights, data and permutations
    (small=False unless given: the split-K direct iteration at every size).
    logp_shift: added to every old log-probability (approx_kl of the first
    minibatch = the shift + the 0.001-scale noise's mean).  run=False: the
    agent as initialised, no update."""
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    variant.setdefault('small', False)
    obs_space = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O)))
    act_space = Box(-np.ones((D, A)), np.ones((D, A)))
    torch.manual_seed(1)
    agent = MAPPOAgent(obs_space, act_space, hidden_dim=256, opt_epochs=2, mini_batch_size=T * E // 2,
                       entropy_coef=0.005, use_graphs=graphs, device="cuda", **variant)
    agent._force_allreduce = force_allreduce
    torch.manual_seed(2)
    buf = MAPPOBuffer(obs_space, act_space, T, E, include_global_state=True, device="cuda")
    buf.next_obs_slots.normal_()
    buf.act.normal_()
    with torch.no_grad():
        d = agent.ac.actor.dist(buf.obs.reshape(-1, O))
        buf.logp.copy_(d.log_prob(buf.act.reshape(-1, A)).reshape(T, E, D, 1)
                       + 0.001 * torch.randn(T, E, D, 1, device="cuda") + logp_shift)
    buf.ret_env.normal_()
    buf.adv_env.normal_()
    buf.t, buf.full = 0, True
    if not run:
        return agent, None
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    res = agent.update(buf, generator=gen)
    torch.cuda.synchronize()
    return agent, res


@pytest.mark.parametrize("E,T", [(256, 16), (32, 8)])
@pytest.mark.parametrize("graphs", [False, True])
def test_direct_update_side_stream_bit_identical(graphs, E, T):
    """The critic forward / backward (and, opt-in with the fused actor, its sums +
    Adam) on their own stream (side_stream) change no bit of the update; the direct iteration agrees with the autograd-driven fused
    one (E=256, T=16: the same kernels at 16 384 actor / 2 048 critic rows)."""
    a_side, r_side = _hidden256_update(graphs, E, T)
    assert a_side._direct_ok()
    a_one, r_one = _hidden256_update(graphs, E, T, side_stream=False)
    assert torch.equal(a_side.actor_opt.flat, a_one.actor_opt.flat)
    assert torch.equal(a_side.critic_opt.flat, a_one.critic_opt.flat)
    assert torch.equal(a_side.actor_opt.exp_avg_sq, a_one.actor_opt.exp_avg_sq)
    assert r_side == r_one
    # the critic's sums + Adam in their own launch on the side stream (opt-in)
    a_join, r_join = _hidden256_update(graphs, E, T, critic_adam_side=True)
    assert torch.equal(a_side.actor_opt.flat, a_join.actor_opt.flat)
    assert torch.equal(a_side.critic_opt.flat, a_join.critic_opt.flat)
    assert torch.equal(a_side.critic_opt.exp_avg, a_join.critic_opt.exp_avg)
    assert r_side == r_join
    # the critic on qs_ppo_critic_tiles + qs_wgrad_t (opt-in) instead of the qs_mlp3w kernels + GEMMs,
    # after the fused actor (default) or beside it
    assert type(a_side._ws_critic).__name__ == "_M3Work"
    for after in (True, False):
        a_t, r_t = _hidden256_update(graphs, E, T, critic_tiles=True, critic_after_actor=after)
        assert type(a_t._ws_critic).__name__ == "_CriticTiles"
        torch.testing.assert_close(a_t.critic_opt.flat, a_side.critic_opt.flat, rtol=0, atol=4 * 1e-3 / 60)
        torch.testing.assert_close(a_t.actor_opt.flat, a_side.actor_opt.flat, rtol=0, atol=4 * 3e-4 / 60)
        for k in r_side:
            assert r_t[k] == pytest.approx(r_side[k], rel=1e-5, abs=1e-7)
    a_fused, r_fused = _hidden256_update(graphs, E, T, direct=False)
    # (the fused path's critic, at 128 rows, is plain torch: ulp-level gradient
    # differences, which Adam's normalised steps carry up to ~lr/60 per step; 4 steps)
    torch.testing.assert_close(a_side.actor_opt.flat, a_fused.actor_opt.flat, rtol=0, atol=4 * 3e-4 / 60)
    torch.testing.assert_close(a_side.critic_opt.flat, a_fused.critic_opt.flat, rtol=0, atol=4 * 1e-3 / 60)
    for k in r_side:
        assert r_side[k] == pytest.approx(r_fused[k], rel=1e-5, abs=1e-7)


@pytest.mark.parametrize("E,T", [(256, 16), (32, 8)])
def test_direct_update_fused_value_head_bit_identical(E, T):
    """The critic's value head folded into its forward (qs_mlp3_fwd_rows_value)
    gives the same dv, hence bit-identical weights and moments, as the separate
    qs_value_head launch; the value-loss statistic differs only in its summation
    order."""
    a_f, r_f = _hidden256_update(True, E, T, fused_value_head=True)
    assert a_f.fused_value_head and type(a_f._ws_critic).__name__ == "_M3Work"
    a_s, r_s = _hidden256_update(True, E, T, fused_value_head=False)
    assert torch.equal(a_f.actor_opt.flat, a_s.actor_opt.flat)
    assert torch.equal(a_f.critic_opt.flat, a_s.critic_opt.flat)
    assert torch.equal(a_f.critic_opt.exp_avg_sq, a_s.critic_opt.exp_avg_sq)
    for k in r_f:
        assert r_f[k] == pytest.approx(r_s[k], rel=1e-12, abs=1e-15)
    assert int(a_f._fv_work[:4].sum()) == 0   # the arrival counter is left zero for the next replay


@pytest.mark.parametrize("graphs", [False, True])
def test_direct_update_fused_actor_four_outputs(graphs):
    """The fused actor kernel on a 4-output actor (Spiral's VEL actions, the C4
    trainer config; _F16_MAX_A = 4): the direct iteration with and without the
    side stream agree bit for bit, and with the autograd-driven iteration within
    Adam's step tolerance."""
    E, T, D, A = 128, 8, 5, 4
    a_side, r_side = _hidden256_update(graphs, E, T, D=D, A=A)
    assert a_side._direct_ok() and type(a_side._ws_actor).__name__ == "_F16Work"
    a_one, r_one = _hidden256_update(graphs, E, T, D=D, A=A, side_stream=False)
    assert torch.equal(a_side.actor_opt.flat, a_one.actor_opt.flat)
    assert torch.equal(a_side.critic_opt.flat, a_one.critic_opt.flat)
    assert r_side == r_one
    a_ref, r_ref = _hidden256_update(graphs, E, T, D=D, A=A, direct=False)
    torch.testing.assert_close(a_side.actor_opt.flat, a_ref.actor_opt.flat, rtol=0, atol=4 * 3e-4 / 60)
    torch.testing.assert_close(a_side.critic_opt.flat, a_ref.critic_opt.flat, rtol=0, atol=4 * 1e-3 / 60)
    for k in r_side:
        assert r_side[k] == pytest.approx(r_ref[k], rel=1e-5, abs=1e-7)


@pytest.mark.parametrize("E,T,D,A,O", [(8, 8, 8, 1, 27), (32, 8, 8, 1, 27), (5, 6, 8, 1, 27), (16, 4, 5, 4, 27),
                                       (3, 2, 16, 1, 27), (64, 16, 8, 1, 27), (32, 8, 16, 1, 27),
                                       (16, 8, 5, 4, 119), (4, 4, 8, 4, 72), (128, 16, 8, 1, 27),
                                       (64, 16, 16, 1, 27), (128, 16, 5, 4, 119), (256, 16, 8, 1, 27)])
@pytest.mark.parametrize("graphs", [False, True])
def test_small_update_matches_autograd(graphs, E, T, D, A, O, monkeypatch):
    """The tile path (qs_ppo_small_step: two launches per minibatch, three
    when a net's weight gradients are split in K-chunks) against the
    autograd-driven fused iteration over 2 epochs x 2 minibatches:
    (8, 8, 8): the reference's mini_batch_size 32 (256 actor rows, 32 critic
    rows); (5, 6, 8): 15 env-timesteps, rows not a multiple of the 16-row tile;
    (16, 4, 5, 4): Spiral's 4-wide VEL actor; (3, 2, 16): 3 critic rows of 432
    inputs (the wide tile instance); (64, 16, 8): 4 096 actor rows (C3's
    per-rank shape at G = 8: the actor's weight gradients in 4 K-chunks);
    (32, 8, 16): C5's drones, a 432-wide critic on 128 rows and 2 048 actor rows;
    (128, 16, 8): 8 192 actor rows (C3 at G = 4: 48-row actor tiles, 16-row
    critic tiles, one round of the CUs); (64, 16, 16): C5 at G = 8, 8 192 actor
    rows beside a 432-wide critic at 16 rows; (128, 16, 5, 4, 119): C4 at G = 4
    (5 120 four-output actor rows, a 595-wide critic); (256, 16, 8): 16 384 actor rows (C3 at G = 2: 48-row tiles in
    two rounds, the actor's weight gradients in K-chunks summed by launch 3);
    (16, 8, 5, 4, 119): Spiral's obs, a 595-wide critic; (4, 4, 8, 4, 72): a
    576-wide critic (C3 with VEL actions), past 640 nothing."""
    from gym_pybullet_drones_amd import _lib as L
    from gym_pybullet_drones_amd.mappo import agent as agent_mod
    monkeypatch.setattr(agent_mod, "_SMALL_MAX_ROWS", L.QS_PPO_SMALL_MAX_ROWS)
    a_small, r_small = _hidden256_update(graphs, E, T, D=D, A=A, O=O, small=True)
    mb = T * E // 2
    took_small = getattr(a_small, '_sm_key', None) is not None
    assert took_small == (D * O <= 640), (D, O, took_small)
    a_ref, r_ref = _hidden256_update(graphs, E, T, D=D, A=A, O=O, direct=False)
    # Adam's normalised steps carry ulp-level gradient differences up to ~lr/60 per step; 4 steps
    adam_close(a_small.actor_opt.flat, a_ref.actor_opt.flat, 3e-4, 4)
    adam_close(a_small.critic_opt.flat, a_ref.critic_opt.flat, 1e-3, 4)
    assert float(a_small.actor_opt.step) == float(a_ref.actor_opt.step)
    assert float(a_small.critic_opt.step) == float(a_ref.critic_opt.step) == 4.0
    for k in r_small:
        # approx_kl: a mean of log-probability differences ~1e-3 formed from float32
        # log-densities ~5 (cancellation), so an absolute bound
        assert r_small[k] == pytest.approx(r_ref[k], rel=1e-5, abs=1e-6 if k == 'approx_kl' else 1e-7), k
    if took_small:
        _assert_small_copies_current(a_small)
    assert mb > 0


def _assert_small_copies_current(agent):
    """The small path's transposed W2 copies and padded W1 copies equal the
    weights after the Adam steps (the pad columns stay zero)."""
    for w2t, w1p, mlp in zip(agent._sm_w2t, agent._sm_w1p, (agent.ac.actor.pi_net, agent.ac.critic.v_net)):
        I = mlp.fcs[0].in_features
        assert torch.equal(w2t, mlp.fcs[1].weight.t())
        assert torch.equal(w1p[:, :I], mlp.fcs[0].weight)
        assert not w1p[:, I:].any()


@pytest.mark.parametrize("graphs", [False, True])
def test_small_update_kl_gate_closed(graphs):
    """qs_ppo_small_step with the actor's KL gate closed (AG:731-734): old
    log-probabilities 0.02 above the current ones put approx_kl above
    1.5·target_kl = 0.015 on every minibatch, so the actor's weight tiles,
    vector parameters and logstd are skipped and its step count is not
    committed, while the critic steps every time — as the autograd-driven
    iteration's gated Adam does."""
    a_small, r_small = _hidden256_update(graphs, 8, 8, small=True, logp_shift=0.02)
    assert a_small._sm_key is not None
    a_init, _ = _hidden256_update(graphs, 8, 8, small=True, run=False)
    a_ref, r_ref = _hidden256_update(graphs, 8, 8, direct=False, logp_shift=0.02)
    assert float(a_small.actor_opt.step) == float(a_ref.actor_opt.step) == 0.0
    assert float(a_small.critic_opt.step) == float(a_ref.critic_opt.step) == 4.0
    assert torch.equal(a_small.actor_opt.flat, a_init.actor_opt.flat)   # not one actor element moved
    assert not a_small.actor_opt.exp_avg.any() and not a_small.actor_opt.exp_avg_sq.any()
    torch.testing.assert_close(a_small.critic_opt.flat, a_ref.critic_opt.flat, rtol=0, atol=4 * 1e-3 / 60)
    assert r_small['approx_kl'] > 0.015 and r_small['approx_kl'] == pytest.approx(r_ref['approx_kl'], rel=1e-5)
    _assert_small_copies_current(a_small)


def test_small_update_replay_deterministic():
    """Fixed reduction orders: two runs of the small path give the same bits."""
    a1, r1 = _hidden256_update(True, 8, 8, small=True)
    a2, r2 = _hidden256_update(True, 8, 8, small=True)
    assert torch.equal(a1.actor_opt.flat, a2.actor_opt.flat) and torch.equal(a1.critic_opt.flat, a2.critic_opt.flat)
    assert r1 == r2


@pytest.mark.parametrize("graphs", [True, False])
def test_mappo_train_step_and_checkpoint(graphs, tmp_path):
    from gym_pybullet_drones_amd.envs import MultiHoverAviary
    from gym_pybullet_drones_amd.mappo import MAPPO
    from gym_pybullet_drones_amd.utils.enums import ActionType
    env_func = lambda seed=None, **kw: MultiHoverAviary(num_drones=3, act=ActionType.ONE_D_PID)
    m = MAPPO(env_func, output_dir=str(tmp_path), checkpoint_path=str(tmp_path / "m.pt"), use_gpu=True, seed=0,
              hidden_dim=64, rollout_batch_size=32, rollout_steps=40, mini_batch_size=64, opt_epochs=2,
              max_env_steps=32 * 40 * 2, eval_interval=0, log_interval=0, use_graphs=graphs)
    m.reset()
    r1 = m.train_step()
    r2 = m.train_step()
    for r in (r1, r2):
        for k in ('policy_loss', 'value_loss', 'entropy_loss', 'approx_kl'):
            assert np.isfinite(r[k]), k
    assert m.total_steps == 2 * 32 * 40
    m.save(str(tmp_path / "ck.pt"))
    w = m.agent.actor_opt.flat.clone()
    m.agent.actor_opt.flat.zero_()
    m.load(str(tmp_path / "ck.pt"))
    assert torch.equal(m.agent.actor_opt.flat, w)
    ev = m.run(n_episodes=1)
    assert len(ev['ep_returns']) == 1
    m.close()


def test_close_releases_graphs(tmp_path):
    """MAPPO.close() frees the rollout graph and the agent's update graph (with
    several ranks they hold captured RCCL all-reduces, which must not outlive the
    process group): no CUDAGraph of the trainer is alive after close()."""
    import gc
    import weakref
    from gym_pybullet_drones_amd.envs import MultiHoverAviary
    from gym_pybullet_drones_amd.mappo import MAPPO
    from gym_pybullet_drones_amd.utils.enums import ActionType
    env_func = lambda seed=None, **kw: MultiHoverAviary(num_drones=2, act=ActionType.ONE_D_PID)
    m = MAPPO(env_func, output_dir=str(tmp_path), use_gpu=True, seed=0, hidden_dim=64, rollout_batch_size=16,
              rollout_steps=8, mini_batch_size=32, opt_epochs=1, eval_interval=0, log_interval=0, use_graphs=True)
    m.reset()
    m.train_step()
    assert m._rollout_graph is not None and m.agent._graph is not None
    refs = [weakref.ref(m._rollout_graph), weakref.ref(m.agent._graph)]
    m.close()
    gc.collect()   # only to rule out reference cycles: close() itself dropped the graphs
    assert m._rollout_graph is None and m.agent._graph is None
    assert all(r() is None for r in refs)


@pytest.mark.parametrize("A", [1, 4])
def test_ppo_heads_kernel_matches_autograd(A):
    """qs_ppo_heads (one launch) against autograd through compute_policy_loss +
    compute_value_loss, with log-prob offsets large enough that both clip
    branches and ties occur."""
    import ctypes
    from gym_pybullet_drones_amd import _lib as L
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    torch.manual_seed(3)
    E, D, O, T = 32, 4, 12 + 15 * A, 4
    obs_space = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O)))
    act_space = Box(-np.ones((D, A)), np.ones((D, A)))
    agent = MAPPOAgent(obs_space, act_space, hidden_dim=32, entropy_coef=0.01, device="cuda")
    with torch.no_grad():
        agent.ac.actor.logstd.copy_(torch.linspace(-0.7, -0.3, A))
    buf = MAPPOBuffer(obs_space, act_space, T, E, include_global_state=True, device="cuda")
    buf.next_obs_slots.normal_()
    buf.act.normal_()
    with torch.no_grad():
        d = agent.ac.actor.dist(buf.obs.reshape(-1, O))
        lp = d.log_prob(buf.act.reshape(-1, A)).reshape(T, E, D, 1)
        buf.logp.copy_(lp + 0.4 * torch.randn_like(lp))
    buf.ret_env.normal_()
    buf.adv_env.normal_()
    idx = torch.randperm(T * E, device="cuda")[:100]   # 400 rows: two workgroups
    # autograd reference
    batch = buf.sample(idx)
    obs_flat = batch['obs'].reshape(-1, O)
    mean = agent.ac.actor.pi_net(obs_flat).detach().requires_grad_(True)
    v = agent.ac.critic(batch['global_obs']).detach().requires_grad_(True)
    logstd = agent.ac.actor.logstd.detach().clone().requires_grad_(True)
    from gym_pybullet_drones_amd.mappo.agent import Normal
    dist = Normal(mean, logstd.exp())
    logp = dist.log_prob(batch['act'].reshape(-1, A))
    ratio = torch.exp(logp - batch['logp'].reshape(-1, 1))
    adv = batch['adv'].reshape(-1, 1)
    pl = -torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv).mean()
    el = -dist.entropy().mean()
    ret = batch['ret'].mean(dim=1, keepdim=True).reshape(v.shape)
    vl = 0.5 * (v - ret).pow(2).mean()
    kl = (batch['logp'].reshape(-1, 1) - logp).mean()
    (pl + 0.01 * el + vl).backward()
    # fused kernel
    mb = idx.shape[0]
    dmean = torch.empty(mb * D, A, device="cuda")
    dv = torch.empty(mb, 1, device="cuda")
    dls = torch.empty(A, device="cuda")
    klo = torch.empty(1, device="cuda")
    acc = torch.zeros(4, dtype=torch.float64, device="cuda")
    lib = L.load()
    work = torch.zeros(int(lib.qs_ppo_heads_work_bytes(mb, D)), dtype=torch.uint8, device="cuda")
    for rep in range(2):   # the second call checks the workspace was left ready
        acc.zero_()
        L.check(lib.qs_ppo_heads(mb, D, A, L.ptr(idx), L.ptr(mean.detach().contiguous()), L.ptr(logstd.detach()), 1.0,
                                 L.ptr(buf.act), L.ptr(buf.logp), L.ptr(buf.adv_env), L.ptr(buf.ret_env),
                                 L.ptr(v.detach().contiguous()), 0.2, 0.01, L.ptr(dmean), L.ptr(dls), L.ptr(dv),
                                 L.ptr(klo), L.ptr(acc), L.ptr(work),
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "qs_ppo_heads")
    torch.cuda.synchronize()
    clipped = ((ratio < 0.8) | (ratio > 1.2)).sum().item()
    assert 0 < clipped < ratio.numel()   # both branches exercised
    torch.testing.assert_close(dmean, mean.grad, rtol=2e-6, atol=1e-9)
    torch.testing.assert_close(dv, v.grad, rtol=1e-6, atol=1e-12)
    torch.testing.assert_close(dls, logstd.grad, rtol=1e-5, atol=1e-7)
    assert acc[0].item() == pytest.approx(pl.item(), rel=1e-6)   # fp32 log-prob sums over A (order)
    assert acc[1].item() == pytest.approx(vl.item(), rel=1e-12)
    assert acc[2].item() == pytest.approx(el.item(), rel=1e-6)
    assert klo.item() == pytest.approx(kl.item(), rel=1e-5, abs=1e-7)


def test_update_graph_captures_the_allreduce():
    """The multi-rank update: the gradient/approx_kl all-reduce (RCCL) captured into
    the minibatch HIP graph.  One rank (world 1, nccl backend) forced through the
    all-reduce path: graph replays must equal eager iterations exactly."""
    import socket
    import torch.distributed as dist
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    own = not dist.is_initialized()
    if own:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
    agents, res = [], []
    try:
        E, D, O, A, T = 64, 3, 27, 1, 8
        obs_space = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O)))
        act_space = Box(-np.ones((D, A)), np.ones((D, A)))
        for graphs in (False, True):
            torch.manual_seed(5)
            ag = MAPPOAgent(obs_space, act_space, hidden_dim=64, opt_epochs=2, mini_batch_size=128,
                            entropy_coef=0.005, use_graphs=graphs, device="cuda")
            ag._force_allreduce = True
            agents.append(ag)
        torch.manual_seed(6)
        buf = MAPPOBuffer(obs_space, act_space, T, E, include_global_state=True, device="cuda")
        buf.next_obs_slots.normal_()
        buf.act.normal_()
        buf.logp.normal_()
        buf.ret_env.normal_()
        buf.adv_env.normal_()
        buf.t, buf.full = 0, True
        for ag in agents:
            gen = torch.Generator(device="cuda")
            gen.manual_seed(0)
            res.append(ag.update(buf, generator=gen))
        torch.cuda.synchronize()
        assert agents[1]._graph is not None
        assert torch.equal(agents[0].actor_opt.flat, agents[1].actor_opt.flat)
        assert torch.equal(agents[0].critic_opt.flat, agents[1].critic_opt.flat)
        for k in ('policy_loss', 'value_loss', 'approx_kl'):
            assert res[0][k] == res[1][k]
    finally:
        for ag in agents:
            ag.release_graphs()
        agents.clear()
        res.clear()
        if own:
            dist.destroy_process_group()


@pytest.mark.parametrize("graphs", [False, True])
def test_direct_update_allreduce_path_bit_identical(graphs):
    """The multi-rank form of the 256-wide direct iteration (what every rank of
    `bench.py --gpus N` runs): partial sums into .grad, the exchange as two RCCL
    all-reduce buckets (one rank; captured in the graph when graphs=True) — the
    critic's on the second stream right after its backward, overlapping the actor
    backward, then the actor's with approx_kl — and the zeroing Adam: bit-identical
    to the one-rank fused sum+Adam launch, at 16 384 / 256 actor rows, with the
    critic on the second stream and on one stream."""
    import socket
    import torch.distributed as dist
    own = not dist.is_initialized()
    if own:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
    def case(E, T, side):
        a_one, r_one = _hidden256_update(graphs, E, T)
        a_ar, r_ar = _hidden256_update(graphs, E, T, force_allreduce=True, side_stream=side)
        try:
            assert torch.equal(a_one.actor_opt.flat, a_ar.actor_opt.flat)
            assert torch.equal(a_one.critic_opt.flat, a_ar.critic_opt.flat)
            assert torch.equal(a_one.critic_opt.exp_avg_sq, a_ar.critic_opt.exp_avg_sq)
            assert r_one == r_ar
        finally:
            # the graph holding the captured all-reduces goes before the communicator
            a_one.release_graphs()
            a_ar.release_graphs()

    try:
        for E, T, side in ((256, 16, True), (32, 8, True), (256, 16, False)):
            case(E, T, side)
    finally:
        torch.cuda.synchronize()
        if own:
            dist.destroy_process_group()
