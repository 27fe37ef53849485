"""The shared case of tests/test_gpu_small_multirank.py and its rank workers:
a 256-wide MAPPO agent (seeded init, identical on every rank) and one rank's
env slice of a global rollout drawn from a seeded CPU generator."""
import numpy as np
import torch

O, A = 27, 1
EPOCHS, MB_PER_EPOCH = 2, 2


# the KL gate closed far from its threshold: logp_old shifted by +KL_SHIFT makes every
# minibatch's approx_kl ≈ KL_SHIFT (the actor never steps, so it stays there) against
# a threshold of 1.5·GATE_TARGET_KL
KL_SHIFT, GATE_TARGET_KL = 0.05, 1e-4


def build(E, T, D, rank=0, world=1, gate_closed=False):
    """Agent + this rank's MAPPOBuffer (envs [rank·E/world, (rank+1)·E/world)).
    gate_closed: the actor's KL gate shut on every minibatch (AG:731-734)."""
    from gym_pybullet_drones_amd.mappo import agent as agent_mod
    from gym_pybullet_drones_amd.mappo.agent import MAPPOAgent
    from gym_pybullet_drones_amd.mappo.buffer import MAPPOBuffer
    from gym_pybullet_drones_amd.utils.spaces import Box
    from gym_pybullet_drones_amd import _lib as L
    agent_mod._SMALL_MAX_ROWS = L.QS_PPO_SMALL_MAX_ROWS   # the tile path at every size of the case
    obs_space = Box(-np.inf * np.ones((D, O)), np.inf * np.ones((D, O)))
    act_space = Box(-np.ones((D, A)), np.ones((D, A)))
    torch.manual_seed(1)
    # target_kl: no KL gate (the gate's global approx_kl may sit at the threshold, where the
    # ranks' and the single rank's row-sum orders could branch differently; the gated
    # branch has its own tests in tests/test_gpu_learner.py)
    agent = MAPPOAgent(obs_space, act_space, hidden_dim=256, opt_epochs=EPOCHS, mini_batch_size=1,
                       entropy_coef=0.005, target_kl=GATE_TARGET_KL if gate_closed else 1e9, use_graphs=False,
                       device="cuda", small=True)
    g = torch.Generator().manual_seed(2)
    obs = torch.randn((T, E, D, O), generator=g)
    act = torch.randn((T, E, D, A), generator=g)
    noise = 1e-3 * torch.randn((T, E, D, 1), generator=g)
    ret = torch.randn((T, E), generator=g, dtype=torch.float64)
    adv = torch.randn((T, E), generator=g, dtype=torch.float64)
    El = E // world
    sl = slice(rank * El, (rank + 1) * El)
    buf = MAPPOBuffer(obs_space, act_space, T, El, include_global_state=True, device="cuda")
    buf.next_obs_slots[:T].copy_(obs[:, sl])
    buf.act.copy_(act[:, sl])
    with torch.no_grad():
        d = agent.ac.actor.dist(buf.obs.reshape(-1, O))
        buf.logp.copy_(d.log_prob(buf.act.reshape(-1, A)).reshape(T, El, D, 1) + noise[:, sl].cuda()
                       + (KL_SHIFT if gate_closed else 0.0))
    buf.ret_env.copy_(ret[:, sl])
    buf.adv_env.copy_(adv[:, sl])
    buf.t, buf.full = 0, True
    return agent, buf


def local_minibatches(El, T, mb):
    """Every rank's minibatch index sets (env-timestep t·El + e of its own buffer):
    EPOCHS × MB_PER_EPOCH slices of seeded permutations."""
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(EPOCHS):
        perm = torch.randperm(T * El, generator=g)
        out += [perm[i * mb:(i + 1) * mb] for i in range(MB_PER_EPOCH)]
    return out


def to_global(idx, rank, El, E):
    """A rank's local env-timestep indices as indices of the global (T, E) rollout."""
    t, e = idx // El, idx % El
    return t * E + rank * El + e


def snapshot(agent):
    ok = True
    for w2t, w1p, mlp in zip(agent._sm_w2t, agent._sm_w1p, (agent.ac.actor.pi_net, agent.ac.critic.v_net)):
        I = mlp.fcs[0].in_features
        ok = ok and torch.equal(w2t, mlp.fcs[1].weight.t()) and torch.equal(w1p[:, :I], mlp.fcs[0].weight)
    return {"actor": agent.actor_opt.flat.clone(), "critic": agent.critic_opt.flat.clone(),
            "actor_m": agent.actor_opt.exp_avg.clone(), "critic_v": agent.critic_opt.exp_avg_sq.clone(),
            "actor_step": agent.actor_opt.step.clone(), "critic_step": agent.critic_opt.step.clone(),
            "copies_current": torch.tensor(bool(ok))}
