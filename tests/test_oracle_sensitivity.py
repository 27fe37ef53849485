"""Sensitivity of the reference's own closed loop (fp64 oracle only, CPU).

Why the fp32 tolerance of tests/test_gpu_tolerance.py has a horizon for the VEL
and downwash configs: round the fp64 oracle's state ONCE to fp32 after 20
control steps and keep stepping both copies in fp64 with the same actions.
  * C3-VEL (MultiHover 8 drones, ActionType.VEL) and C4 (Spiral VEL): the DSL
    PID attitude loop under random velocity targets (BaseRLAviary.py:208-223,
    DSLPIDControl.py:212-259) grows the ~6e-8 rounding past 1e-4 m within
    19 and 34 steps.
  * C5 (16 drones, PYB_DW): the downwash force alpha = 2267.18 (r/(4 dz))^2
    (BaseAviary.py:797-810) is singular as dz -> 0+, and the grid's drones
    cross each other's heights; the rounding passes 1e-4 m within 10 steps.
  * C2 (RPM) and C3 (ONE_D_PID) do not amplify: below 1e-6 m after 300 steps.
No fp32 implementation of these configs can therefore stay within 1e-4 of the
fp64 reference for longer than these horizons; bit-identical fp64 arithmetic
would be needed.

One rounding is the mildest perturbation: from k0 = 0 (the reset draws rounded
once) C5 takes ~55 steps to pass the bounds.  Real fp32 arithmetic rounds every
operation of every substep; the oracle's own fp32 instantiation (IEEE division
and square root, libm expf, no contraction — an exact fp32 restatement) departs
from its fp64 run within 3 (C5 velocity) to 28 (C4 position) steps.  Those are
the reference's fp32 sensitivity horizons; the GPU tests' horizon tables
(FP32_HORIZON, FREE_HORIZON_FP32) are pinned to them below, and
tests/test_gpu_tolerance.py::test_fp32_horizons_match_exact_fp32 shows the
kernel departs at the same steps.
"""
import importlib.util
import os

import numpy as np
import pytest

import qs_oracle
import trajectory as tj


def _grid(D):
    cols = int(np.ceil(np.sqrt(D)))
    rows = int(np.ceil(D / cols))
    return [[(i % cols - (cols - 1) / 2), (i // cols - (rows - 1) / 2), 0.5] for i in range(D)]


CFGS = {
    "C2": dict(task="multihover", num_drones=4, act="rpm"),
    "C3": dict(task="multihover", num_drones=8, act="one_d_pid", initial_xyzs=_grid(8)),
    "C3v": dict(task="multihover", num_drones=8, act="vel", initial_xyzs=_grid(8)),
    "C4": dict(task="spiral", num_drones=5, act="vel"),
    "C5": dict(task="multihover", num_drones=16, act="one_d_pid", initial_xyzs=_grid(16), physics="pyb",
               aux=("dw",)),
}


def rounding_growth(cfg, steps, E=64, k0=20, seed=11):
    a = qs_oracle.OracleSim(num_envs=E, precision=8, **cfg)
    b = qs_oracle.OracleSim(num_envs=E, precision=8, **cfg)
    a.reset(seed)
    b.reset(seed)
    for _ in range(k0):
        a.step(None)
        b.step(None)
    s = b.get_state(0)
    b.set_state(0, s.astype(np.float32).astype(np.float64))
    curves = {k: np.zeros(steps) for k in ("pos", "quat", "vel", "rew")}
    for t in range(steps):
        ra = a.step(None)
        rb = b.step(None)
        sa, sb = a.get_state(0), b.get_state(0)
        for k, sl in (("pos", slice(0, 3)), ("quat", slice(3, 7)), ("vel", slice(7, 10))):
            curves[k][t] = np.abs(sa[sl] - sb[sl]).max()
        curves["rew"][t] = np.abs(ra["reward"] - rb["reward"]).max()
    a.close()
    b.close()
    return curves


BOUND = dict(pos=1e-4, quat=1e-4, vel=1e-3, rew=1e-4)   # the fp32 bounds of test_gpu_tolerance.py


# control steps within which one rounding passes the bound (measured: C3v quat 12, vel 18,
# pos 19, rew 24; C4 rew 20, quat 26, vel 32, pos 34; C5 pos / vel / rew 10)
@pytest.mark.parametrize("name,field,within", [("C3v", "quat", 12), ("C3v", "pos", 19), ("C4", "rew", 20),
                                               ("C4", "pos", 34), ("C5", "pos", 10), ("C5", "vel", 10)])
def test_reference_amplifies_one_fp32_rounding(name, field, within):
    curve = rounding_growth(CFGS[name], within + 1)[field]
    assert curve.max() > BOUND[field], f"{name} {field}: {curve.max():.2e}"


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_reference_does_not_amplify(name):
    curves = rounding_growth(CFGS[name], 300)
    assert curves["pos"].max() < 1e-6, f"{name}: {curves['pos'].max():.2e}"


def _gpu_table(module, attr):
    spec = importlib.util.spec_from_file_location(module, os.path.join(os.path.dirname(__file__), module + ".py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m, getattr(m, attr)


def _exact_fp32_horizons(cfg, E, steps):
    """First-exceed steps of the oracle's fp32 instantiation against its fp64 run
    (seed 11, tests/trajectory.py diverge)."""
    res = tj.diverge(cfg, E=E, precision=4, steps=steps, seed=11, subject="oracle")
    return {k: tj.first_exceed(res["curves"][k], BOUND[k]) for k in BOUND}


def _check_table(name, table, fe):
    # once the state has departed the reward follows it: a reward horizon is only
    # required up to one step past the state's
    need = dict(fe, rew=min(fe["rew"], min(fe["pos"], fe["vel"]) + 1))
    for k, h in table.items():
        assert h <= fe[k], f"{name} {k}: table {h} claims more than the exact fp32 restatement ({fe[k]})"
        assert h >= need[k] - 2, f"{name} {k}: table {h} well short of the exact fp32 horizon {need[k]}"


@pytest.mark.parametrize("name", ["C3v_mh_vel_d8", "C4_spiral_vel_d5", "C4p_spiral_vel_d5_pyb", "meetup_vel_d4",
                                  "C5_mh_dw_d16", "C5p_mh_dw_d16_pyb", "mh_dw_d8", "pyb_dw_d4", "mh_gnd_drag_d4",
                                  "pyb_gnd_drag_dw_d4"])
def test_free_running_horizons_are_the_exact_fp32_ones(name):
    """FREE_HORIZON_FP32 (16 envs, 30 steps) is the exact fp32 restatement's
    horizon per field, or at most 2 steps short of it (never longer)."""
    m, table = _gpu_table("test_gpu_parity", "FREE_HORIZON_FP32")
    _check_table(name, table[name], _exact_fp32_horizons(m.CONFIGS[name], 16, m.FREE_STEPS))


@pytest.mark.parametrize("name", ["C3v", "C4", "C5"])
def test_tolerance_horizons_are_the_exact_fp32_ones(name):
    """FP32_HORIZON (64 envs, 60-step window) likewise."""
    m, table = _gpu_table("test_gpu_tolerance", "FP32_HORIZON")
    _check_table(name, table[name], _exact_fp32_horizons(m.CFGS[name], 64, 60))
