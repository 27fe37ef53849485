"""Known-answer tests for the oracle's Physics.PYB restatement.

pybullet is not installed and the reference cannot run here, so the
PYB mode is "parity unpinned" against Bullet itself.  These tests pin the
restatement to the btMultiBody semantics it claims — prop forces at the prop-link
COMs of assets/cf2x.urdf:42-79, default damping 0.04 as m·v·(k + k|v|) and
I·ω·(k + k|ω|), semi-implicit Euler, world-frame exp-map orientation update with
renormalisation, the ground plane — each expected value derived by hand.
"""
import numpy as np
import pytest

import qs_oracle as Q

C = Q.constants()
DT = 1.0 / 240
K = 0.04
M, IXX, IYY, IZZ = 0.027, 1.4e-5, 1.4e-5, 2.17e-5
F_POS, F_QUAT, F_VEL, F_W, F_RPM, F_TGT = 0, 3, 7, 10, 13, 26


def _sim(D=1, act="rpm", aux=(), **kw):
    s = Q.OracleSim(task="multihover", num_envs=1, num_drones=D, act=act, precision=8, physics="pyb", aux=aux,
                    initial_xyzs=[[float(i), 0.0, 1.0] for i in range(D)], **kw)
    s.reset(0)
    return s


def _inject(s, pos, quat=(0, 0, 0, 1), vel=(0, 0, 0), w=(0, 0, 0)):
    st = s.get_state(0)
    st[:] = 0
    D = st.shape[1]
    for d in range(D):
        st[F_POS:F_POS + 3, d] = pos[d]
        st[F_QUAT:F_QUAT + 4, d] = quat
        st[F_VEL:F_VEL + 3, d] = vel
        st[F_W:F_W + 3, d] = w
        st[F_TGT:F_TGT + 3, d] = pos[d]
    s.set_state(0, st)
    return st


def test_pyb_hover_fixed_point():
    """Level, at rest, 4·KF·HOVER_RPM² = G·M ⇒ no net force or torque, no damping at rest."""
    s = _sim(D=2)
    st0 = _inject(s, [[0, 0, 1.0], [1, 0, 1.0]])
    for _ in range(30):
        s.step(np.zeros((1, 2, 4), np.float32))
    st = s.get_state(0)
    np.testing.assert_allclose(st[F_POS:F_POS + 3], st0[F_POS:F_POS + 3], atol=1e-12)
    np.testing.assert_allclose(st[F_VEL:F_VEL + 3], 0, atol=1e-12)
    np.testing.assert_allclose(st[F_QUAT:F_QUAT + 4], st0[F_QUAT:F_QUAT + 4], atol=1e-15)


def test_pyb_free_fall_with_linear_damping():
    """rpm = 0: v' = -g - k(1 + |v|)v, velocity first then position (semi-implicit)."""
    s = _sim(D=1, act="one_d_rpm")
    _inject(s, [[0, 0, 3.0]])
    s.step(np.full((1, 1, 1), -20.0, np.float32))
    st = s.get_state(0)
    g = C["GRAVITY"] / M
    v, z = 0.0, 3.0
    for _ in range(8):
        v = v + DT * (-g - (K + K * abs(v)) * v)
        z = z + DT * v
    np.testing.assert_allclose(st[F_VEL + 2, 0], v, rtol=1e-12)
    np.testing.assert_allclose(st[F_POS + 2, 0], z, rtol=1e-13)


def test_pyb_yaw_spin_with_angular_damping_and_exp_map():
    """rpm = [r0, r1, r0, r1] ⇒ only τz = KM(-r0² + r1² - r0² + r1²); ω_z' = τz/Izz - k(1+|ω|)ω_z;
    q = [0, 0, sin(ψ/2), cos(ψ/2)] with ψ += ω_z·dt each substep (new ω, exp map)."""
    s = _sim(D=1)
    _inject(s, [[0, 0, 1.0]])
    a0, a1 = np.float32(0.5), np.float32(-0.3)
    s.step(np.array([[[a0, a1, a0, a1]]], np.float32))
    st = s.get_state(0)
    r0, r1 = C["HOVER_RPM"] * (1 + 0.05 * float(a0)), C["HOVER_RPM"] * (1 + 0.05 * float(a1))
    tz = 7.94e-12 * (-r0 ** 2 + r1 ** 2 - r0 ** 2 + r1 ** 2)
    w, psi = 0.0, 0.0
    for _ in range(8):
        w = w + DT * (tz - (K + K * abs(w)) * IZZ * w) / IZZ
        psi += w * DT
    np.testing.assert_allclose(st[F_W + 2, 0], w, rtol=1e-12)
    np.testing.assert_allclose(st[F_W:F_W + 2, 0], 0, atol=1e-15)
    np.testing.assert_allclose(st[F_QUAT:F_QUAT + 4, 0], [0, 0, np.sin(psi / 2), np.cos(psi / 2)], atol=1e-14)
    # thrust of the four rotors is not balanced against gravity here: only the z motion changes
    np.testing.assert_allclose(st[F_POS:F_POS + 2, 0], 0, atol=1e-15)


def test_pyb_roll_torque_from_prop_positions():
    """Rotors 2 and 3 (y = +0.028, assets/cf2x.urdf) faster than 0 and 1 (y = -0.028) ⇒
    τx = Σ y_i f_i > 0 ⇒ positive roll rate; the DSL mixer commands this roll for +τx."""
    s = _sim(D=1)
    _inject(s, [[0, 0, 1.0]])
    da = np.float32(0.2)
    s.step(np.array([[[-da, -da, da, da]]], np.float32))
    st = s.get_state(0)
    f = 3.16e-10 * (C["HOVER_RPM"] * (1 + 0.05 * np.array([-da, -da, da, da], np.float64))) ** 2
    tx = 0.028 * (-f[0] - f[1] + f[2] + f[3])
    assert tx > 0 and st[F_W, 0] > 0
    # first substep: ω_x = dt·τx/Ixx exactly (no damping at rest, no gyroscopic term)
    s2 = _sim(D=1, ctrl_freq=240)
    _inject(s2, [[0, 0, 1.0]])
    s2.step(np.array([[[-da, -da, da, da]]], np.float32))
    np.testing.assert_allclose(s2.get_state(0)[F_W, 0], DT * tx / IXX, rtol=1e-12)


def test_pyb_quaternion_stays_normalised():
    """Renormalisation after every exp-map update (btMultiBody::stepPositionsMultiDof)."""
    s = _sim(D=1)
    q = np.array([0.3, -0.2, 0.1, 0.9])
    _inject(s, [[0, 0, 1.5]], quat=q / np.linalg.norm(q), w=(30.0, -20.0, 50.0))
    for _ in range(10):
        s.step(np.random.default_rng(1).uniform(-1, 1, (1, 1, 4)).astype(np.float32))
    qq = s.get_state(0)[F_QUAT:F_QUAT + 4, 0]
    assert abs(np.linalg.norm(qq) - 1) < 1e-14


def test_pyb_ground_plane():
    """A level drone below z = 0.0125 (cylinder half-length) is pushed up to it and its
    downward velocity removed; the episode then terminates as a crash (z < 0.03, MH:226)."""
    s = _sim(D=1, act="one_d_rpm")
    _inject(s, [[0, 0, 0.02]], vel=(0, 0, -1.0))
    out = s.step(np.full((1, 1, 1), -20.0, np.float32))
    assert out["terminated"][0] == 1
    # look at the state before the auto-reset: run without it
    s2 = Q.OracleSim(task="multihover", num_envs=1, num_drones=1, act="one_d_rpm", precision=8, physics="pyb",
                     initial_xyzs=[[0.0, 0.0, 1.0]], autoreset=False)
    s2.reset(0)
    _inject(s2, [[0, 0, 0.02]], vel=(0, 0, -1.0))
    s2.step(np.full((1, 1, 1), -20.0, np.float32))
    st = s2.get_state(0)
    np.testing.assert_allclose(st[F_POS + 2, 0], 0.0125, rtol=1e-12)
    assert st[F_VEL + 2, 0] == 0.0


def test_pyb_differs_from_dyn_only_by_bullet_terms():
    """Same start, small actions: PYB and DYN agree to first order over one step (the
    damping and the prop arm 0.028 vs L/√2 are the differences; the roll and pitch
    torque signs agree: props at (±0.028, ±0.028) give τx = −0.028(f0+f1−f2−f3), the
    sign of BaseAviary.py:849's −(f0+f1−f2−f3)·L/√2)."""
    rng = np.random.default_rng(3)
    a = rng.uniform(-0.1, 0.1, (1, 2, 1)).astype(np.float32)
    out = {}
    for phys in ("dyn", "pyb"):
        s = Q.OracleSim(task="multihover", num_envs=1, num_drones=2, act="one_d_rpm", precision=8, physics=phys,
                        initial_xyzs=[[0.0, 0, 1.0], [1.0, 0, 1.0]])
        s.reset(0)
        _inject(s, [[0, 0, 1.0], [1, 0, 1.0]])
        s.step(a)
        out[phys] = s.get_state(0)
    np.testing.assert_allclose(out["pyb"][F_POS:F_POS + 3], out["dyn"][F_POS:F_POS + 3], atol=1e-6)
    np.testing.assert_allclose(out["pyb"][F_VEL:F_VEL + 3], out["dyn"][F_VEL:F_VEL + 3], atol=1e-4)
