"""Device-resident MAPPO rollout storage, GAE and advantage normalisation.

Mirrors gym_pybullet_drones/mappo/buffer.py (MAPPOBuffer BUF:10-306,
compute_returns_and_advantages BUF:428-614, normalize_advantages BUF:666-695)
with all storage in HBM:

* obs/act/logp live in (T, E, D, ·) tensors the simulator and the actor write
  into directly (no per-step deepcopy + host→device push);
* per-env quantities the reference tiles over agents (reward, mask, returns,
  advantages — MP:740-817, 1118-1133) are stored once per env and exposed as
  stride-0 expanded (T, E, D, 1) views, which is value-identical;
* `global_obs` (the concatenated per-env obs, MP:583-617) is a reshape view of
  `obs`, not a second copy;
* GAE runs as one HIP kernel (qs_gae) instead of an E·D·T Python loop.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as tdist

from .. import _lib as L
from . import collectives


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def gae(rews, vals, masks, terminal_vals, last_val, gamma=0.99, use_gae=True, gae_lambda=0.95):
    """compute_returns_and_advantages for sequences laid out (T, N...) on the GPU.

    rews/masks (T, *S) float32, vals/terminal_vals (T, *S) float32 or None (zeros),
    last_val (*S) float32 → (rets, advs) float64 (T, *S), like the reference."""
    T = rews.shape[0]
    N = rews[0].numel()
    cont = lambda x: None if x is None else x.to(torch.float32).contiguous()
    rews, vals, masks, terminal_vals, last_val = map(cont, (rews, vals, masks, terminal_vals, last_val))
    rets = torch.empty(rews.shape, dtype=torch.float64, device=rews.device)
    advs = torch.empty_like(rets)
    lib = L.load()
    L.check(lib.qs_gae(T, N, L.ptr(rews), L.ptr(vals), L.ptr(masks), L.ptr(terminal_vals), L.ptr(last_val),
                       float(gamma), float(gae_lambda), int(bool(use_gae)), L.ptr(rets), L.ptr(advs), _stream()),
            "qs_gae")
    return rets, advs


compute_returns_and_advantages = gae


def normalize_advantages(advs, epsilon=1e-8):
    """BUF:666-695 (torch branch: unbiased std).  Under torch.distributed the
    moments are global over all ranks' buffers."""
    if advs.numel() == 0:
        return advs
    if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
        x = advs.to(torch.float64)
        s = torch.stack([x.sum(), (x * x).sum(), torch.tensor(float(x.numel()), dtype=torch.float64,
                                                                device=x.device)])
        collectives.all_reduce(s)
        n = s[2]
        mean = s[0] / n
        var = (s[1] - n * mean * mean) / (n - 1)
        std = torch.sqrt(torch.clamp(var, min=0))
    else:
        mean = advs.mean()
        std = advs.std()
    # reference: `if adv_std < epsilon: return advs - adv_mean` (host branch) — computed on device
    scaled = (advs - mean) / (std + epsilon)
    return torch.where(std < epsilon, advs - mean, scaled)


class MAPPOBuffer:
    """(T, E, D, ·) rollout storage on the GPU (BUF:10-306)."""

    def __init__(self, obs_space, act_space, max_length, batch_size, include_global_state=False,
                 global_state_dim=None, include_actions_in_critic=False, device='cuda', use_gpu_storage=True):
        self.max_length = T = max_length
        self.batch_size = E = batch_size
        self.include_global_state = include_global_state
        self.include_actions_in_critic = include_actions_in_critic
        self.device = torch.device(device)
        obs_shape, act_shape = tuple(obs_space.shape), tuple(act_space.shape)
        if len(obs_shape) == 1:
            D, O = 1, obs_shape[0]
        else:
            D, O = obs_shape
        A = act_shape[-1]
        self.num_agents, self.obs_dim, self.act_dim = D, O, A
        self.global_obs_dim = (global_state_dim or D * O) if include_global_state else None
        if include_global_state and self.global_obs_dim != D * O:
            raise NotImplementedError("a true global state (global_state_dim != D*O) is not provided by these envs")
        kw = dict(device=self.device)
        # obs has T+1 slots: slot t+1 receives the env's next obs in place
        self._obs_all = torch.zeros((T + 1, E, D, O), dtype=torch.float32, **kw)
        self.act = torch.zeros((T, E, D, A), dtype=torch.float32, **kw)
        self.logp = torch.zeros((T, E, D, 1), dtype=torch.float32, **kw)
        self.v = torch.zeros((T, E, D, 1), dtype=torch.float32, **kw)
        self.rew_env = torch.zeros((T, E), dtype=torch.float32, **kw)
        self.mask_env = torch.ones((T, E), dtype=torch.float32, **kw)
        self.terminal_v_env = torch.zeros((T, E), dtype=torch.float32, **kw)
        self.ret_env = torch.zeros((T, E), dtype=torch.float64, **kw)
        self.adv_env = torch.zeros((T, E), dtype=torch.float64, **kw)
        self.keys = ['obs', 'act', 'rew', 'mask', 'v', 'logp', 'ret', 'adv', 'terminal_v'] + \
            (['global_obs'] if include_global_state else [])
        self.t = 0
        self.full = False

    # ------------------------------------------------------------ views
    @property
    def obs(self):
        return self._obs_all[:self.max_length]

    @property
    def next_obs_slots(self):
        return self._obs_all

    @property
    def global_obs(self):
        T, E, D, O = self.obs.shape
        return self.obs.reshape(T, E, D * O)

    def _agents(self, x):
        return x.unsqueeze(-1).unsqueeze(-1).expand(*x.shape, self.num_agents, 1)

    rew = property(lambda self: self._agents(self.rew_env))
    mask = property(lambda self: self._agents(self.mask_env))
    terminal_v = property(lambda self: self._agents(self.terminal_v_env))
    ret = property(lambda self: self._agents(self.ret_env))

    @property
    def adv(self):
        return self._agents(self.adv_env)

    @adv.setter
    def adv(self, value):
        # normalize_advantages result: per-env values broadcast over agents; copied in
        # place so captured update graphs keep reading the same storage
        self.adv_env.copy_(value[..., 0, 0] if value.dim() == 4 else value)

    def reset(self):
        self.t = 0
        self.full = False

    def push(self, batch):
        """Compatibility path of BUF:157-220 (the rollout loop writes in place instead)."""
        t = self.t
        for k, v in batch.items():
            if k not in self.keys or k == 'global_obs':
                continue
            v = torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v, device=self.device)
            if k in ('rew', 'mask', 'terminal_v'):
                getattr(self, k + '_env')[t].copy_(v.reshape(self.batch_size, -1)[:, 0])
            elif k == 'obs':
                self._obs_all[t].copy_(v.reshape(self._obs_all[t].shape))
            else:
                getattr(self, k)[t].copy_(v.reshape(getattr(self, k)[t].shape))
        self.t = (self.t + 1) % self.max_length
        if self.t == 0:
            self.full = True

    def advance(self):
        self.t = (self.t + 1) % self.max_length
        if self.t == 0:
            self.full = True

    def get(self, device=None):
        T, E = self.max_length, self.batch_size
        out = {k: getattr(self, k) for k in self.keys}
        return {k: v.reshape(T * E, *v.shape[2:]) for k, v in out.items()}

    def sample(self, indices):
        """Gather env-timestep rows (BUF:251-276) → dict of (mb, D, ·) tensors."""
        T, E, D = self.max_length, self.batch_size, self.num_agents
        idx = indices
        batch = {
            'obs': self.obs.reshape(T * E, D, self.obs_dim).index_select(0, idx),
            'act': self.act.reshape(T * E, D, self.act_dim).index_select(0, idx),
            'logp': self.logp.reshape(T * E, D, 1).index_select(0, idx),
            'v': self.v.reshape(T * E, D, 1).index_select(0, idx),
        }
        for k in ('rew', 'mask', 'terminal_v', 'ret', 'adv'):
            env = getattr(self, k + '_env').reshape(T * E).index_select(0, idx)
            batch[k] = env.view(-1, 1, 1).expand(-1, D, 1)
        if self.include_global_state:
            batch['global_obs'] = batch['obs'].reshape(-1, D * self.obs_dim)
        return batch

    def sample_obs(self, indices):
        """The obs rows of env-timesteps `indices` only, (mb, D, O): what the fused
        loss heads (qs_ppo_heads) need gathered; they read act/logp/adv/ret by index."""
        T, E, D = self.max_length, self.batch_size, self.num_agents
        return self.obs.reshape(T * E, D, self.obs_dim).index_select(0, indices)

    def sampler(self, mini_batch_size, device=None, drop_last=True, generator=None):
        """random_sample (BUF:399-425): a permutation of the env-timesteps, in
        mini-batches of whole env-timesteps (all D agents together)."""
        total = (self.max_length if self.full or self.t == 0 else self.t) * self.batch_size
        perm = torch.randperm(total, device=self.device, generator=generator)
        full = total // mini_batch_size
        for i in range(full):
            yield self.sample(perm[i * mini_batch_size:(i + 1) * mini_batch_size])
        if not drop_last and total % mini_batch_size:
            yield self.sample(perm[full * mini_batch_size:])

    def compute_returns_and_advantages(self, last_val, gamma=0.99, use_gae=False, gae_lambda=0.95):
        """BUF:328-396.  The reference's values are zero placeholders and last_val is
        tiled over agents (MP:821-841, 1050-1067), so the recurrence is per env;
        a per-agent last_val/v falls back to the per-agent kernel launch."""
        T, E, D = self.max_length, self.batch_size, self.num_agents
        last_val = torch.as_tensor(last_val, device=self.device, dtype=torch.float32)
        per_env = (last_val.numel() == E or bool((last_val.reshape(E, -1) == last_val.reshape(E, -1)[:, :1]).all())) \
            and not bool(self.v.abs().max() > 0)
        if not per_env:
            raise NotImplementedError("per-agent values are not produced by this trainer (v is a zero placeholder)")
        lv = last_val.reshape(E, -1)[:, 0]
        rets, advs = gae(self.rew_env, None, self.mask_env, self.terminal_v_env, lv, gamma, use_gae, gae_lambda)
        self.ret_env.copy_(rets)
        self.adv_env.copy_(advs)
        return self.ret, self.adv
