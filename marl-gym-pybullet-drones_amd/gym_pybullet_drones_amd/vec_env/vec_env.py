"""Baselines-style VecEnv surface backed by the HIP QuadSwarm.

Keeps the contract the reference's MAPPO calls:
  VecEnv               safe_control_gym/envs/env_wrappers/vectorized_env/vec_env.py:13-141
  SubprocVecEnv        .../vectorized_env/subproc_vec_env.py:20-109 (pool removed)
  worker.step_env      .../vectorized_env/subproc_vec_env.py:188-206 (auto-reset kept)
  VecRecordEpisodeStatistics  .../env_wrappers/record_episode_statistics.py:97-172

`reset()` → (obs (E,D,O), {'n': infos}); `step(actions)` → (obs, rews (E,) float64,
dones (E,) bool, {'n': infos}) with 'terminal_observation'/'terminal_info' on done.
The numpy path materialises Python infos (as the reference does); `step_t`
is the zero-copy device path the on-device trainer uses.
"""
from collections import deque
from copy import deepcopy

import numpy as np
import torch

from .. import _lib as L
from ..envs.swarm import QuadSwarm
from ..utils.enums import ActionType, Physics
from ..utils.spaces import Box


class VecEnv:
    """Abstract vectorised env (vec_env.py:13-141)."""

    closed = False
    viewer = None

    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space

    def reset(self):
        raise NotImplementedError

    def step_async(self, actions):
        raise NotImplementedError

    def step_wait(self):
        raise NotImplementedError

    def close_extras(self):
        pass

    def close(self):
        if self.closed:
            return
        self.close_extras()
        self.closed = True

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    @property
    def unwrapped(self):
        return self


def observation_space_for(swarm: QuadSwarm) -> Box:
    """BaseRLAviary._observationSpace (BRL:256-277) / SpiralAviary (SP:103-114)."""
    D, O, H, A = swarm.num_drones, swarm.obs_dim, swarm.hist_len, swarm.act_dim
    if swarm.task == "spiral":
        return Box(np.full((D, O), -np.inf, np.float32), np.full((D, O), np.inf, np.float32), dtype=np.float32)
    lo = np.full((D, O), -np.inf, np.float32)
    hi = np.full((D, O), np.inf, np.float32)
    lo[:, 2] = 0
    lo[:, 12:12 + H * A] = -1
    hi[:, 12:12 + H * A] = 1
    return Box(lo, hi, dtype=np.float32)


def action_space_for(swarm: QuadSwarm) -> Box:
    """BaseRLAviary._actionSpace (BRL:132-156)."""
    shape = (swarm.num_drones, swarm.act_dim)
    return Box(-np.ones(shape, np.float32), np.ones(shape, np.float32), dtype=np.float32)


def _reasons_strings(bits, tobs):
    """MultiHoverAviary._computeTerminated reason strings (MH:225-238)."""
    out = []
    for i, b in enumerate(bits):
        x, y, z, roll, pitch = tobs[i, 0], tobs[i, 1], tobs[i, 2], tobs[i, 3], tobs[i, 4]
        if b & L.REASON_CRASH:
            out.append(f"Drone {i} crashed (z={z:.2f})")
        if b & L.REASON_FLIP:
            out.append(f"Drone {i} flipped (roll={roll:.2f}, pitch={pitch:.2f})")
        if b & L.REASON_OOB:
            out.append(f"Drone {i} out of bounds (pos=[{x:.2f}, {y:.2f}, {z:.2f}])")
    return out


class SwarmVecEnv(VecEnv):
    """GPU-backed replacement of make_vec_envs(...) → SubprocVecEnv (no worker pool)."""

    def __init__(self, task="multihover", num_envs=1, num_drones=2, act=ActionType.RPM, physics=Physics.DYN,
                 seed=0, device=None, precision=4, env_offset=0, initial_xyzs=None, **kw):
        self.swarm = QuadSwarm(task=task, num_envs=num_envs, num_drones=num_drones, act=act, physics=physics,
                               precision=precision, device=device, env_offset=env_offset,
                               initial_xyzs=initial_xyzs, **kw)
        self.seed = int(seed)
        super().__init__(num_envs, observation_space_for(self.swarm), action_space_for(self.swarm))
        self._actions = None
        self.NUM_DRONES = self.swarm.num_drones
        self.CTRL_FREQ = self.swarm.ctrl_freq
        self.CTRL_TIMESTEP = 1.0 / self.CTRL_FREQ
        self.PYB_FREQ = self.swarm.pyb_freq
        self.EPISODE_LEN_SEC = self.swarm.episode_len_sec

    @property
    def device(self):
        return self.swarm.device

    # ---------------------------------------------------------- info dicts
    def _info(self, step_counter, reasons=()):
        if self.swarm.task == "spiral":   # SpiralAviary._computeInfo (SP:200-205)
            sp = self.swarm.spec
            return {"time": step_counter / self.PYB_FREQ, "omega": 2 * np.pi / sp.spiral_period,
                    "radius": sp.spiral_radius}
        if self.swarm.task != "multihover":   # Flock/Meetup/LeaderFollower._computeInfo
            return {"answer": 42}
        return {"answer": 42, "termination_reasons": list(reasons)}   # MH:274-285

    # ----------------------------------------------------------- numpy API
    def reset(self):
        obs = self.swarm.reset(self.seed)
        infos = tuple(self._info(0) for _ in range(self.num_envs))
        return obs.cpu().numpy(), {"n": infos}

    def step_async(self, actions):
        a = torch.as_tensor(np.asarray(actions, np.float32)).reshape(
            self.num_envs, self.swarm.num_drones, self.swarm.act_dim)
        self._actions = a.to(self.device).contiguous()

    def step_wait(self):
        sc_before = self.swarm.get_state(L.STATE_ENV)[L.E_STEP_COUNTER].cpu().numpy()
        r = self.swarm.step(self._actions, want_terminal=True, want_reasons=True)
        obs = r.obs.cpu().numpy()
        rews = r.reward.double().cpu().numpy()
        te = r.terminated.cpu().numpy().astype(bool)
        tr = r.truncated.cpu().numpy().astype(bool)
        dones = te | tr
        tobs = r.terminal_obs.cpu().numpy() if dones.any() else None
        bits = r.reasons.cpu().numpy()
        infos = []
        for i in range(self.num_envs):
            if dones[i]:
                reasons = _reasons_strings(bits[i], tobs[i]) if self.swarm.task == "multihover" else []
                info = self._info(0)
                info["terminal_observation"] = tobs[i].copy()
                info["terminal_info"] = self._info(int(sc_before[i]), reasons)
            else:
                info = self._info(int(sc_before[i]))
            infos.append(info)
        return obs, rews, dones, {"n": tuple(infos)}

    # ------------------------------------------------- zero-copy device API
    def reset_t(self):
        return self.swarm.reset(self.seed)

    def step_t(self, actions=None, **kw):
        return self.swarm.step(actions, **kw)

    # -------------------------------------------- checkpoint RNG (MP:203-270)
    def get_env_random_state(self):
        """Counter-based RNG: the stream state is (seed, per-env counters)."""
        return {"seed": self.seed, "env_state": self.swarm.get_state(L.STATE_ENV).cpu()}

    def set_env_random_state(self, state):
        self.seed = int(state["seed"])
        self.swarm.set_state(L.STATE_ENV, state["env_state"])

    def close_extras(self):
        self.swarm.close()


class VecEnvWrapper(VecEnv):
    """vec_env.py:144-206: forwards unknown attributes to the wrapped venv."""

    def __init__(self, venv):
        self.venv = venv
        super().__init__(venv.num_envs, venv.observation_space, venv.action_space)

    def step_async(self, actions):
        self.venv.step_async(actions)

    def reset(self):
        return self.venv.reset()

    def step_wait(self):
        return self.venv.step_wait()

    def close(self):
        return self.venv.close()

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.venv, name)


class VecRecordEpisodeStatistics(VecEnvWrapper):
    """record_episode_statistics.py:97-172 with the same attributes and semantics."""

    def __init__(self, venv, deque_size=None, **kwargs):
        super().__init__(venv)
        self.deque_size = deque_size
        self.episode_return = np.zeros(self.num_envs)
        self.episode_length = np.zeros(self.num_envs)
        self.return_queue = deque(maxlen=deque_size)
        self.length_queue = deque(maxlen=deque_size)
        self.episode_stats = {}
        self.accumulated_stats = {}
        self.queued_stats = {}

    def add_tracker(self, name, init_value, mode="accumulate"):
        self.episode_stats[name] = [init_value for _ in range(self.num_envs)]
        if mode == "accumulate":
            self.accumulated_stats[name] = init_value
        elif mode == "queue":
            self.queued_stats[name] = deque(maxlen=self.deque_size)
        else:
            raise Exception("Tracker mode not implemented.")

    def reset(self, **kwargs):
        self.episode_return = np.zeros(self.num_envs)
        self.episode_length = np.zeros(self.num_envs)
        self._synced, self._synced_seq = 0, -1   # the reset restarts the device episode counters
        for key in self.episode_stats:
            for i in range(self.num_envs):
                self.episode_stats[key][i] *= 0
        return self.venv.reset(**kwargs)

    def step_wait(self):
        """Same bookkeeping as record_episode_statistics.py:144-172: the return
        grows by the env's mean reward, the length by one; trackers read the
        env's info (its terminal_info on done); a finished episode is written to
        info['n'][i]['episode'], queued, and its per-env counters restart."""
        obs, reward, done, info = self.venv.step_wait()
        infos = info["n"]
        # vectorised over envs: mean over agents of each env's reward
        self.episode_return += np.asarray(reward, np.float64).reshape(self.num_envs, -1).mean(axis=1)
        self.episode_length += 1
        ended = np.flatnonzero(np.asarray(done, bool))
        if self.episode_stats:
            ended_set = set(ended.tolist())
            for i in range(self.num_envs):
                src = infos[i]["terminal_info"] if i in ended_set else infos[i]
                for key, vals in self.episode_stats.items():
                    if key in src:
                        vals[i] += src[key]
        for i in ended:
            ep_r, ep_l = float(self.episode_return[i]), float(self.episode_length[i])
            summary = {"r": ep_r, "l": ep_l}
            self.return_queue.append(ep_r)
            self.length_queue.append(ep_l)
            for key, vals in self.episode_stats.items():
                value = deepcopy(vals[i])
                summary[key] = value
                if key in self.accumulated_stats:
                    self.accumulated_stats[key] += deepcopy(value)
                if key in self.queued_stats:
                    self.queued_stats[key].append(deepcopy(value))
                vals[i] *= 0
            infos[i]["episode"] = summary
        self.episode_return[ended] = 0
        self.episode_length[ended] = 0
        return obs, reward, done, info

    def sync_from_device(self):
        """Fast-path equivalent for step_t users: pull the episodes the kernel
        logged since the last sync (device ring, env order per step).  Returns
        how many episodes ended since then; queues the newest of them that the
        rings still hold (at most deque_size), each exactly once: a record is
        new iff its seq (the step it ended at) is past the last synced one."""
        sw = self.venv.swarm
        _, total = sw.episode_log(cap=0)
        last = getattr(self, "_synced", 0)
        gen = getattr(sw, "reset_generation", 0)
        if gen != getattr(self, "_synced_gen", gen) or total < last:
            # the swarm was reset (by any path) since the last sync: its episode
            # counters and record seqs restarted at 0
            last, self._synced_seq = 0, -1
        self._synced_gen = gen
        new = total - last
        self._synced = total
        if new <= 0:
            return 0
        recs, _ = sw.episode_log(cap=new if self.deque_size is None else min(new, self.deque_size))
        recs = recs[recs["seq"] > getattr(self, "_synced_seq", -1)]
        if len(recs):
            self._synced_seq = int(recs["seq"].max())
        for rec in recs:
            self.return_queue.append(float(rec["ret"]))
            self.length_queue.append(float(rec["len"]))
        return new
