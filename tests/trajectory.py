"""Free-running trajectory comparison of the HIP kernel against the fp64 oracle
(test infrastructure: imported by tests/ and scripts/tolerance_curves.py only).

Both sides start from the same Philox reset draws and step the same Philox
random-policy actions; nothing is injected after the reset, so the comparison
measures the accumulated trajectory error.  Per step it records
the maximum over live envs of |Δpos|, |Δquat|, |Δvel| and |Δreward|.

Threshold ties ("identical term/trunc flags except at threshold
ties (flagged, not failed)"): an env whose terminated/truncated flags differ
while its state was still inside the tolerance is a tie; it is counted and
dropped from the comparison from then on (its two copies now live different
episodes).  A MultiHover reward that differs by more than the reward bound in
an env where some drone sits within the tie window of a reward branch
threshold (MultiHoverAviary.py:140-179: |e_z| < 0.2, e_xy < 0.03, |e_z| < 0.03,
|v_z| < 0.03) is a reward tie, counted, and not a failure.  The window is 10x
the step's own max |Δpos| / |Δvel| (tie_window): a threshold can only be
straddled by as much as the state differs.

diverge(subject="oracle") runs the oracle's fp32 instantiation in the kernel's
place: the departure of an exact fp32 restatement from fp64 — the reference's
own sensitivity to fp32 rounding, against which the kernel's fp32 horizons are
measured (tests/test_gpu_tolerance.py, scripts/horizon_compare.py).
"""
import numpy as np
import torch

import qs_oracle

F_POS, F_QUAT, F_VEL, F_TARGET = 0, 3, 7, 26


def make_swarm(cfg, E, precision, env_offset=0):
    from gym_pybullet_drones_amd.envs import QuadSwarm
    from gym_pybullet_drones_amd.utils.enums import Physics
    kw = dict(cfg)
    aux = tuple(kw.pop("aux", ()))
    phys = kw.pop("physics", "dyn")
    if phys == "pyb":   # the reference's PYB / PYB_GND_DRAG_DW / PYB_DW modes
        name = {(): Physics.PYB, ("gnd", "drag", "dw"): Physics.PYB_GND_DRAG_DW, ("dw",): Physics.PYB_DW}[aux]
        return QuadSwarm(num_envs=E, precision=precision, physics=name, env_offset=env_offset, **kw)
    return QuadSwarm(num_envs=E, precision=precision, physics=Physics.DYN, aux=aux, env_offset=env_offset, **kw)


def make_oracle(cfg, E, precision, env_offset=0):
    kw = dict(cfg)
    return qs_oracle.OracleSim(num_envs=E, precision=precision, env_offset=env_offset, **kw)


def _mh_reward_tie(state, target, D, env, eps):
    """True if some drone of `env` is within eps of a MultiHover reward branch
    threshold (MH:140-179).  state: SoA [29][N] float64 (pre-reset view)."""
    sl = slice(env * D, (env + 1) * D)
    p, v, t = state[F_POS:F_POS + 3, sl], state[F_VEL:F_VEL + 3, sl], target[:, sl]
    exy = np.hypot(p[0] - t[0], p[1] - t[1])
    ez = np.abs(p[2] - t[2])
    vz = np.abs(v[2])
    near = (np.abs(ez - 0.2) < eps) | (np.abs(exy - 0.03) < eps) | (np.abs(ez - 0.03) < eps) | (np.abs(vz - 0.03) < eps)
    return bool(near.any())


class _OracleSubject:
    """The oracle at `precision` behind the swarm interface diverge() reads: the
    exact-arithmetic subject (IEEE fp32 division / sqrt, libm transcendentals,
    no contraction) whose departure from the fp64 oracle is the reference's own
    sensitivity to fp32 rounding (CPU only)."""

    class _R:
        pass

    def __init__(self, cfg, E, precision, env_offset):
        self.o = make_oracle(cfg, E, precision, env_offset)
        self.num_drones = self.o.D

    def reset(self, seed):
        self.o.reset(seed)

    def step(self, actions, want_terminal=True):
        c = self.o.step(actions)
        r = self._R()
        for k in ("terminated", "truncated", "reward"):
            setattr(r, k, torch.from_numpy(np.asarray(c[k])))
        return r

    def get_state(self, block):
        return torch.from_numpy(self.o.get_state(block))

    def close(self):
        self.o.close()


def tie_window(dpos, dvel, eps=None):
    """Width of the reward-threshold tie window at one step: a fixed eps if
    given, else 10x the step's own |Δpos| / |Δvel| (the MultiHover branches
    compare position errors and |vz| with thresholds, MH:140-179), floored at
    1e-7 so that a zero-deviation step excuses nothing."""
    if eps is not None:
        return eps
    return max(10.0 * max(dpos, dvel), 1e-7)


def diverge(cfg, E, precision, steps, seed=11, env_offset=0, rew_bound=1e-4, tie_eps=None, full_E=None,
            on_step=None, on_reset=None, subject="kernel"):
    """Run the kernel (at `precision`) and the fp64 oracle side by side for
    `steps` control steps.  Returns a dict of per-step curves and tie counts.

    full_E: run the kernel at this env count (a BASELINE config's real size) and
    compare its envs [env_offset, env_offset + E) with an E-env oracle built with
    the same env_offset (the Philox key holds the global env id, so the slice is
    the same computation).  on_step(t, sw, result) runs property checks over
    every env of the kernel after each step (on_reset(sw) after the reset).
    tie_eps: reward-threshold tie window (None: tie_window's 10x the step's own
    state deviation).  subject="oracle": the oracle at `precision` in place of
    the kernel (the exact-fp32 sensitivity reference, CPU)."""
    if subject == "oracle":
        sw = _OracleSubject(cfg, E, precision, env_offset)
        lo = 0
    elif full_E is None:
        sw = make_swarm(cfg, E, precision, env_offset)
        lo = 0
    else:
        sw = make_swarm(cfg, full_E, precision, 0)
        lo = env_offset
    truth = make_oracle(cfg, E, 8, env_offset)
    D = sw.num_drones
    esl = slice(lo, lo + E)
    asl = slice(lo * D, (lo + E) * D)
    sw.reset(seed)
    truth.reset(seed)
    if on_reset is not None:
        on_reset(sw)
    live = np.ones(E, bool)
    curves = {k: np.zeros(steps) for k in ("pos", "quat", "vel", "rew")}
    flag_ties = rew_ties = ended = 0
    mh = cfg.get("task", "multihover") == "multihover"
    st_prev = truth.get_state(0)
    for t in range(steps):
        r = sw.step(None, want_terminal=True)
        c = truth.step(None, nthreads=1 if E * D < 4096 else 8)
        if on_step is not None:
            on_step(t, sw, r)
        if subject != "oracle":
            torch.cuda.synchronize()
        term_g, trunc_g = r.terminated[esl].cpu().numpy().astype(bool), r.truncated[esl].cpu().numpy().astype(bool)
        term_c, trunc_c = c["terminated"].astype(bool), c["truncated"].astype(bool)
        mism = live & ((term_g != term_c) | (trunc_g != trunc_c))
        flag_ties += int(mism.sum())
        live &= ~mism
        ended += int((live & (term_c | trunc_c)).sum())
        g = sw.get_state(0)[:, asl].cpu().numpy().astype(np.float64)
        o = truth.get_state(0)
        cols = np.repeat(live, D)
        for name, off, n in (("pos", F_POS, 3), ("quat", F_QUAT, 4), ("vel", F_VEL, 3)):
            if cols.any():
                curves[name][t] = np.abs(g[off:off + n, cols] - o[off:off + n, cols]).max()
        drew = np.abs(r.reward[esl].cpu().numpy().astype(np.float64) - c["reward"])
        drew[~live] = 0.0
        if mh:
            done_c = term_c | trunc_c
            eps_t = tie_window(curves["pos"][t], curves["vel"][t], tie_eps)
            for e in np.flatnonzero(drew > rew_bound):
                # reward is formed from the pre-reset state: for a done env the
                # terminal obs carries pos/vel, the target is the previous step's
                if done_c[e]:
                    view = np.zeros_like(o)
                    tob = c["terminal_obs"][e]
                    view[F_POS:F_POS + 3, e * D:(e + 1) * D] = tob[:, 0:3].T
                    view[F_VEL:F_VEL + 3, e * D:(e + 1) * D] = tob[:, 6:9].T
                    tgt = st_prev[F_TARGET:F_TARGET + 3]
                else:
                    view, tgt = o, o[F_TARGET:F_TARGET + 3]
                if _mh_reward_tie(view, tgt, D, e, eps_t):
                    rew_ties += 1
                    drew[e] = 0.0
        curves["rew"][t] = drew.max() if live.any() else 0.0
        st_prev = o
    sw.close()
    truth.close()
    return dict(curves=curves, flag_ties=flag_ties, rew_ties=rew_ties, ended=ended, live=int(live.sum()), E=E)


def first_exceed(curve, bound):
    """First step index where curve > bound, or len(curve) if never."""
    idx = np.flatnonzero(curve > bound)
    return int(idx[0]) if idx.size else len(curve)


def episode_returns(log_recs):
    """(returns, lengths) of the completed episodes in an episode-log record array."""
    return np.asarray(log_recs["ret"], np.float64), np.asarray(log_recs["len"], np.float64)


def run_episodes(cfg, E, precision, steps, seed=11, oracle=False):
    """Free-running random-policy rollout; returns the episode-log records of
    every episode completed in `steps` control steps (kernel or fp64 oracle)."""
    if oracle:
        sim = make_oracle(cfg, E, precision)
        sim.reset(seed)
        for _ in range(steps):
            sim.step(None, nthreads=16)
        recs, _ = sim.episode_log()
        sim.close()
        return recs
    sw = make_swarm(cfg, E, precision)
    sw.reset(seed)
    for _ in range(steps):
        sw.step(None)
    torch.cuda.synchronize()
    recs, total = sw.episode_log(cap=1 << 20)
    assert total == len(recs)
    sw.close()
    return recs
