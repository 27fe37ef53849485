"""Known-answer tests pinning the CPU oracle to the reference *text* (SURVEY §8(c) K1–K9).

The reference ships no golden vectors and cannot be executed here,
so each expected value below is derived analytically from the cited reference
lines.  All checks run the fp64 oracle (the reference's precision).
"""
import numpy as np
import pytest

import qs_oracle as Q

C = Q.constants()
DT = 1.0 / 240
F_POS, F_QUAT, F_VEL, F_W, F_RPM, F_TGT = 0, 3, 7, 10, 13, 26


def test_philox_random123_kat():
    """Random123 philox4x32-10 known-answer vectors (kat_vectors)."""
    assert [hex(x) for x in Q.philox([0, 0, 0, 0], [0, 0])] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    assert [hex(x) for x in Q.philox([0xffffffff] * 4, [0xffffffff] * 2)] == \
        ["0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]
    assert [hex(x) for x in Q.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0])] \
        == ["0xd16cfe09", "0x94fdcceb", "0x5001e420", "0x24126ea1"]


def test_derived_constants():
    """BaseAviary.py:117-128 with cf2x.urdf values."""
    assert C["GRAVITY"] == pytest.approx(0.2646, rel=1e-15)
    assert C["HOVER_RPM"] == pytest.approx(14468.43, abs=5e-3)
    assert C["MAX_RPM"] == pytest.approx(21702.64, abs=5e-3)
    assert C["MAX_THRUST"] == pytest.approx(0.59535, rel=1e-12)
    assert C["GND_EFF_H_CLIP"] == pytest.approx(0.037764, abs=1e-6)
    assert C["SPEED_LIMIT"] == pytest.approx(0.25, rel=1e-15)   # BaseRLAviary.py:95
    assert C["INIT_Z"] == pytest.approx(0.1125, rel=1e-15)      # BaseAviary.py:197


def _sim(task="multihover", D=2, act="rpm", **kw):
    s = Q.OracleSim(task=task, num_envs=1, num_drones=D, act=act, precision=8, **kw)
    s.reset(0)
    return s


def _inject_level_rest(s, pos):
    st = s.get_state(0)
    st[:] = 0
    st[F_POS:F_POS + 3] = np.asarray(pos, np.float64).T
    st[F_QUAT + 3] = 1.0
    st[F_TGT:F_TGT + 3] = np.asarray(pos, np.float64).T
    s.set_state(0, st)
    return st


def test_K1_dyn_hover_fixed_point():
    """Level, at rest, all rpm = HOVER_RPM (RPM action a = 0, BRL:192) ⇒ F_w = 0, τ = 0 (BA:838-863)."""
    s = _sim(D=2, act="rpm", initial_xyzs=[[0, 0, 1.0], [1, 0, 1.0]])
    st0 = _inject_level_rest(s, [[0, 0, 1.0], [1, 0, 1.0]])
    for _ in range(30):
        out = s.step(np.zeros((1, 2, 4), np.float32))
    st = s.get_state(0)
    np.testing.assert_allclose(st[F_POS:F_POS + 3], st0[F_POS:F_POS + 3], atol=1e-12)
    np.testing.assert_allclose(st[F_VEL:F_VEL + 3], 0, atol=1e-12)
    np.testing.assert_allclose(st[F_QUAT:F_QUAT + 4], st0[F_QUAT:F_QUAT + 4], atol=1e-15)
    np.testing.assert_allclose(st[F_RPM:F_RPM + 4], C["HOVER_RPM"], rtol=1e-15)
    assert out["reward"][0] == pytest.approx(2.5, abs=1e-9)   # K5 at target (MH:140-179)


def test_K2_dyn_free_fall_semi_implicit():
    """rpm = 0 (ONE_D_RPM a = -20 ⇒ HOVER·(1 + 0.05·(-20)) = 0) ⇒ after k substeps
    v_z = -g·k·dt and z = z0 - g·dt²·k(k+1)/2 (semi-implicit Euler, BA:860-862)."""
    s = _sim(D=2, act="one_d_rpm")
    _inject_level_rest(s, [[0, 0, 2.0], [1, 0, 2.0]])
    s.step(np.full((1, 2, 1), -20.0, np.float32))
    st = s.get_state(0)
    k = 8
    g = C["GRAVITY"] / 0.027
    np.testing.assert_allclose(st[F_VEL + 2], -g * k * DT, rtol=1e-12)
    np.testing.assert_allclose(st[F_POS + 2], 2.0 - g * DT * DT * k * (k + 1) / 2, rtol=1e-12)
    np.testing.assert_allclose(st[F_RPM:F_RPM + 4], 0.0, atol=0)


def test_K3_pure_yaw():
    """rpm = [r0, r1, r0, r1] ⇒ τx = τy = 0, τz = 2·KM·(r1² - r0²) (BA:845-851);
    ω_z grows linearly, q = [0, 0, sin(ψ/2), cos(ψ/2)] (exp-map, BA:879-892)."""
    s = _sim(D=1, act="rpm", initial_xyzs=[[0, 0, 1.0]])
    _inject_level_rest(s, [[0, 0, 1.0]])
    a0, a1 = np.float32(0.5), np.float32(-0.3)
    s.step(np.array([[[a0, a1, a0, a1]]], np.float32))
    st = s.get_state(0)
    r0, r1 = C["HOVER_RPM"] * (1 + 0.05 * float(a0)), C["HOVER_RPM"] * (1 + 0.05 * float(a1))
    alpha = 2 * 7.94e-12 * (r1 ** 2 - r0 ** 2) / 2.17e-5
    n = 8
    np.testing.assert_allclose(st[F_W + 2], alpha * DT * n, rtol=1e-10)
    np.testing.assert_allclose(st[F_W:F_W + 2], 0, atol=1e-14)   # ((f0+f1)-f0)-f1 rounding only
    psi = DT * DT * alpha * n * (n + 1) / 2
    np.testing.assert_allclose(st[F_QUAT:F_QUAT + 4, 0], [0, 0, np.sin(psi / 2), np.cos(psi / 2)], atol=1e-14)


def test_K4_pid_hover_fixed_point():
    """Fresh DSLPIDControl, level at rest, target = current pos ⇒
    thrust_pwm = (HOVER_RPM - 4070.3)/0.2685 ⇒ rpm = HOVER_RPM on all motors (PID:188-259)."""
    rpm, st = Q.dsl_pid(np.zeros(9), [0.3, -0.2, 1.0], [0, 0, 0, 1], [0, 0, 0], [0.3, -0.2, 1.0])
    np.testing.assert_allclose(rpm, C["HOVER_RPM"], rtol=1e-12)
    np.testing.assert_array_equal(st, 0)


def test_K5_multihover_reward_offset():
    """e_z = +0.1, v = 0 ⇒ 1/(1+0) + exp(-7.5·0.1) - 1.5·0² = 1 + e^-0.75 (MH:140-179)."""
    s = _sim(D=2, act="rpm", initial_xyzs=[[0, 0, 1.0], [1, 0, 1.0]])
    st = _inject_level_rest(s, [[0, 0, 1.0], [1, 0, 1.0]])
    st[F_POS + 2] += 0.1
    s.set_state(0, st)
    out = s.step(np.zeros((1, 2, 4), np.float32))
    assert out["reward"][0] == pytest.approx(1 + np.exp(-0.75), abs=1e-9)
    assert out["reward"][0] == pytest.approx(1.47237, abs=1e-5)


@pytest.mark.parametrize("field,value,bit", [("z", 0.029, 1), ("roll", 1.21, 2), ("x", 3.01, 4), ("y", -3.01, 4)])
def test_K6_termination_thresholds(field, value, bit):
    """z < 0.03 crash, |roll| > 1.2 flip, |x|,|y| > 3 out of bounds (MH:226-236)."""
    s = _sim(D=2, act="rpm", initial_xyzs=[[0, 0, 1.0], [1, 0, 1.0]])
    st = _inject_level_rest(s, [[0, 0, 1.0], [1, 0, 1.0]])
    if field == "z":
        st[F_POS + 2, 1] = value
    elif field == "x":
        st[F_POS, 1] = value
    elif field == "y":
        st[F_POS + 1, 1] = value
    else:   # roll about x: q = [sin(r/2), 0, 0, cos(r/2)]
        st[F_QUAT, 1], st[F_QUAT + 3, 1] = np.sin(value / 2), np.cos(value / 2)
    s.set_state(0, st)
    out = s.step(np.zeros((1, 2, 4), np.float32))
    assert out["terminated"][0] == 1
    assert out["reasons"][0, 1] & bit
    assert out["reasons"][0, 0] == 0


def test_K6_truncation_at_step_242():
    """step_counter/240 > 8 evaluated before the += 8 increment (MH:268, BA:378-382) ⇒ the
    242nd control step is the first truncated one; auto-reset follows (subproc_vec_env.py:195)."""
    s = _sim(D=2, act="rpm", initial_xyzs=[[0, 0, 1.0], [1, 0, 1.0]])
    _inject_level_rest(s, [[0, 0, 1.0], [1, 0, 1.0]])
    for k in range(1, 243):
        out = s.step(np.zeros((1, 2, 4), np.float32))
        assert out["truncated"][0] == (1 if k == 242 else 0), k
        assert out["terminated"][0] == 0
    assert s.get_state(1)[0, 0] == 0        # step_counter reset
    recs, total = s.episode_log()
    assert total == 1 and recs["len"][0] == 242


def test_K6_spiral_truncation_at_step_578():
    """Spiral: step_counter/240 > 12 with 5 PYB steps per ctrl step ⇒ step 578 (SP:196)."""
    s = _sim(task="spiral", D=3, act="rpm")
    st = s.get_state(0)
    _inject_level_rest(s, st[F_POS:F_POS + 3].T)
    steps = 0
    while True:
        steps += 1
        out = s.step(np.zeros((1, 3, 4), np.float32))
        if out["truncated"][0]:
            break
        assert steps < 600
    assert steps == 578


def test_K7_spiral_reference_at_t0():
    """SpiralAviary._spiral_reference at t=0 (SP:82-99) through the reset obs (SP:120-146)."""
    D = 5
    s = Q.OracleSim(task="spiral", num_envs=1, num_drones=D, act="vel", precision=8)
    obs = s.reset(0)[0]
    R, omega = 0.4, 2 * np.pi / 10.0
    H, A = 24, 4
    assert obs.shape == (D, 12 + H * A + 11)
    for i in range(D):
        ph = 2 * np.pi * i / D
        np.testing.assert_allclose(obs[i, :3], [R * np.cos(ph), R * np.sin(ph), 0.3], atol=1e-7)
        x = obs[i, 12 + H * A:]
        vref = [-R * omega * np.sin(ph), R * omega * np.cos(ph), 0.05]
        np.testing.assert_allclose(x[0:3], 0, atol=1e-7)                    # rel_pos
        np.testing.assert_allclose(x[3:6], vref, atol=1e-7)                 # vel_ref - quat[0:3]
        np.testing.assert_allclose(x[6:8], [np.sin(ph), np.cos(ph)], atol=1e-7)
        np.testing.assert_allclose(x[8:11], vref, atol=1e-7)


def _numpy_single_agent_returns(rews, vals, masks, terminal_vals, last_val, gamma, use_gae, gae_lambda):
    """buffer.py:561-614 line by line on numpy scalars: with numpy >= 2 (the
    reference pins 2.2.6, environment.yml:63) NEP 50 keeps every float32-scalar
    expression with the Python floats γ, λ in float32."""
    T = len(rews)
    rets, advs = np.zeros(T), np.zeros(T)
    vals_extended = np.concatenate([vals, [last_val]])
    ret, adv = last_val, 0
    for i in reversed(range(T)):
        rew_adjusted = rews[i] + gamma * terminal_vals[i]
        ret = rew_adjusted + gamma * masks[i] * ret
        if not use_gae:
            adv = ret - vals[i]
        else:
            td_error = rew_adjusted + gamma * masks[i] * vals_extended[i + 1] - vals[i]
            adv = adv * gae_lambda * gamma * masks[i] + td_error
        rets[i], advs[i] = ret, adv
    return rets, advs


@pytest.mark.parametrize("use_gae", [True, False])
def test_K8_gae_oracle_equals_reference_numpy_semantics(use_gae):
    """The oracle's GAE (float32 line by line) equals the reference's numpy code
    run on float32 arrays under numpy 2 — bit for bit."""
    assert int(np.__version__.split(".")[0]) >= 2
    rng = np.random.default_rng(4)
    T, N = 41, 60
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    m = (rng.random((T, N)) > 0.1).astype(np.float32)
    tv = (rng.normal(size=(T, N)) * (rng.random((T, N)) > 0.8)).astype(np.float32)
    last = rng.normal(size=N).astype(np.float32)
    rets, advs = Q.gae(r, v, m, tv, last, gamma=0.99, use_gae=use_gae, lam=0.95)
    for n in range(N):
        want_r, want_a = _numpy_single_agent_returns(r[:, n], v[:, n], m[:, n], tv[:, n], last[n], 0.99, use_gae, 0.95)
        np.testing.assert_array_equal(rets[:, n], want_r)
        np.testing.assert_array_equal(advs[:, n], want_a)
    # and the float32 recursion is what it is: not the float64 one
    r64, _ = _numpy_single_agent_returns(r[:, 0].astype(np.float64), v[:, 0].astype(np.float64), m[:, 0].astype(np.float64),
                                         tv[:, 0].astype(np.float64), np.float64(last[0]), 0.99, use_gae, 0.95)
    assert not np.array_equal(r64, rets[:, 0])


def test_K8_gae_zero_values():
    """V ≡ 0, m ≡ 1 ⇒ ret_t = Σ_k γ^k r_{t+k} + γ^{T-t}·last (buffer.py:586-612),
    to float32 accuracy (the reference's recursion is float32)."""
    rng = np.random.default_rng(0)
    T, N, g = 17, 5, 0.99
    r = rng.normal(size=(T, N)).astype(np.float32)
    last = rng.normal(size=N).astype(np.float32)
    zeros = np.zeros((T, N), np.float32)
    rets, advs = Q.gae(r, zeros, np.ones((T, N), np.float32), zeros, last, gamma=g, use_gae=True, lam=0.95)
    for t in range(T):
        want = sum(g ** k * r[t + k].astype(np.float64) for k in range(T - t)) + g ** (T - t) * last.astype(np.float64)
        np.testing.assert_allclose(rets[t], want, rtol=2e-6, atol=1e-6)
    # GAE with V ≡ 0: δ_t = r_t (+γ·V_{t+1}=0 except the bootstrap at T-1)
    lam_g = 0.95 * g
    for t in range(T):
        want = sum(lam_g ** k * r[t + k].astype(np.float64) for k in range(T - t)) + lam_g ** (T - 1 - t) * g * last.astype(np.float64)
        np.testing.assert_allclose(advs[t], want, rtol=2e-6, atol=1e-6)


def test_K8_gae_masks_cut_bootstrap():
    T, N = 6, 3
    r = np.ones((T, N), np.float32)
    m = np.ones((T, N), np.float32)
    m[2] = 0
    rets, _ = Q.gae(r, np.zeros((T, N), np.float32), m, np.zeros((T, N), np.float32), np.full(N, 10, np.float32),
                    gamma=0.5, use_gae=False)
    np.testing.assert_allclose(rets[2], 1.0)
    np.testing.assert_allclose(rets[1], 1.5)
    np.testing.assert_allclose(rets[5], 1 + 0.5 * 10)


def test_K9_obs_layout_and_history_persistence():
    """obs = [pos, rpy, vel, ang_v, a_{t-H+1..t}] oldest first (BRL:307-319); the history
    is not cleared by env.reset() (it is filled with zeros once, BRL:153-154)."""
    D, H = 2, 15
    s = Q.OracleSim(task="multihover", num_envs=1, num_drones=D, act="one_d_rpm", precision=8)
    obs = s.reset(0)
    np.testing.assert_array_equal(obs[0, :, 12:], 0)
    acts = [np.full((1, D, 1), 0.01 * (k + 1), np.float32) for k in range(20)]
    for k in range(20):
        out = s.step(acts[k])
    hist = out["obs"][0, 0, 12:]
    np.testing.assert_array_equal(hist, np.array([acts[k][0, 0, 0] for k in range(20 - H, 20)], np.float32))
    np.testing.assert_array_equal(out["obs"][0, :, 3:6], out["obs"][0, :, 3:6])
    obs_r = s.reset_envs(np.array([1], np.uint8))
    np.testing.assert_array_equal(obs_r[0, 0, 12:], hist)           # persists across reset
    np.testing.assert_array_equal(obs_r[0, :, 3:12], 0)             # rpy, vel, ang_v zero after reset
    st = s.get_state(0)
    np.testing.assert_allclose(st[F_TGT + 2] - st[F_POS + 2], [1.0, 0.5])   # TARGET = INIT + [0,0,1/(i+1)] (MH:106)


def test_pid_state_persists_across_reset():
    """Nothing calls ctrl.reset() on env.reset() (BRL/BA/MH): integrators survive."""
    s = Q.OracleSim(task="multihover", num_envs=1, num_drones=2, act="one_d_pid", precision=8)
    s.reset(0)
    for _ in range(10):
        s.step(np.full((1, 2, 1), 0.8, np.float32))
    before = s.get_state(0)[17:26].copy()
    assert np.abs(before).max() > 0
    s.reset_envs(np.array([1], np.uint8))
    np.testing.assert_array_equal(s.get_state(0)[17:26], before)


def test_default_layout_large_d_rejected():
    """MultiHover's rejection loop cannot complete for D >= 6 with the default layout (SURVEY §7 hard-2)."""
    with pytest.raises(ValueError, match="D >= 6"):
        Q.OracleSim(task="multihover", num_envs=1, num_drones=6, act="rpm")
