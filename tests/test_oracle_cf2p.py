"""DroneModel.CF2P in the CPU oracle (QS_FLAG_CF2P): known answers derived from
the reference text — BaseAviary.py:852-853 (the + configuration's torques),
cf2p.urdf:12 (inertia) and 42-79 (prop links on the body axes at L),
DSLPIDControl.py:54-60 (its mixer).  fp64 oracle, one env."""
import numpy as np
import pytest

import qs_oracle as Q

C = Q.constants()
DT = 1.0 / 240
F_POS, F_QUAT, F_VEL, F_W, F_RPM, F_TGT = 0, 3, 7, 10, 13, 26
KF, KM, L = 3.16e-10, 7.94e-12, 0.0397
IXX_X, IXX_P = 1.4e-5, 2.3951e-5


def _sim(model, act="rpm", physics="dyn", D=1):
    s = Q.OracleSim(task="multihover", num_envs=1, num_drones=D, act=act, precision=8, physics=physics,
                    initial_xyzs=[[0, 0, 1.0]] * D if D == 1 else None, drone_model=model)
    s.reset(0)
    st = s.get_state(0)
    st[:] = 0
    st[F_POS + 2] = 1.0
    st[F_QUAT + 3] = 1.0
    st[F_TGT + 2] = 1.0
    s.set_state(0, st)
    return s, st


def _roll_step(model, physics="dyn"):
    """RPM action [0, a, 0, -a]: motors 1 / 3 at HOVER·(1 ± 0.05a) (BRL:191-192)."""
    s, _ = _sim(model, physics=physics)
    a = np.float32(0.5)
    s.step(np.array([[[0, a, 0, -a]]], np.float32))
    return s.get_state(0)[:, 0], float(a)


def test_cf2p_dyn_roll_torque():
    """CF2P: τx = (f1 − f3)·L, τy = (−f0 + f2)·L = 0 (BA:852-853); from rest and level
    ω_x after the 8 substeps = 8·dt·τx / IXX (cf2p.urdf:12), the gyroscopic
    coupling with the small yaw rate below 1e-9 of it."""
    st, a = _roll_step("cf2p")
    h = C["HOVER_RPM"]
    r1, r3 = h * (1 + 0.05 * a), h * (1 - 0.05 * a)
    tx = (KF * r1 ** 2 - KF * r3 ** 2) * L
    np.testing.assert_allclose(st[F_W], 8 * DT * tx / IXX_P, rtol=1e-9)
    assert abs(st[F_W + 1]) < 1e-5 * abs(st[F_W])


def test_cf2p_against_cf2x_roll():
    """The same motor pair on CF2X: τx = −(f0 + f1 − f2 − f3)·L/√2 = −(f1 − f3)·L/√2
    (BA:849) about IXX = 1.4e-5 — opposite sign, ratio −√2·IXX_x/IXX_p (to 1e-4:
    on CF2X the diagonal pair also pitches, τy = (f1 − f3)·L/√2, and the
    gyroscopic term couples the three rates at ~1e-5)."""
    sp, _ = _roll_step("cf2p")
    sx, _ = _roll_step("cf2x")
    assert sx[F_W] < 0 < sp[F_W]
    np.testing.assert_allclose(sp[F_W] / sx[F_W], -np.sqrt(2) * IXX_X / IXX_P, rtol=1e-4)


def test_cf2p_pyb_props_on_the_axes():
    """Physics.PYB: the prop forces at (±L, 0) / (0, ±L) (cf2p.urdf:42-79) give the DYN
    torque (Bullet's damping, 0.04, the only difference: < 0.5 % over 8 substeps)."""
    sd, _ = _roll_step("cf2p", "dyn")
    sb, _ = _roll_step("cf2p", "pyb")
    np.testing.assert_allclose(sb[F_W], sd[F_W], rtol=5e-3)
    assert abs(sb[F_W + 1]) < 1e-5 * abs(sb[F_W])


def test_cf2p_pid_mixer():
    """A drone rolled by 0.1 rad, at rest, target = its position (ONE_D_PID, a = 0):
    the attitude loop's torque demand tq is the same for both models (the gains do
    not depend on them, PID:37-47), so the mixers fix the motor differences
    (DSLPIDControl.py:48-60): CF2P pwm1 − pwm3 = 2·tq0, pwm0 − pwm2 = −2·tq1;
    CF2X pwm0 − pwm2 = −tq0 − tq1 and pwm1 − pwm3 = −tq0 + tq1."""
    rpms = {}
    for model in ("cf2p", "cf2x"):
        s, st = _sim(model, act="one_d_pid")
        st[F_QUAT, 0], st[F_QUAT + 3, 0] = np.sin(0.05), np.cos(0.05)   # roll 0.1 about x
        s.set_state(0, st)
        s.step(np.zeros((1, 1, 1), np.float32))
        rpms[model] = s.get_state(0)[F_RPM:F_RPM + 4, 0]
    k = 0.2685   # rpm = 0.2685·pwm + 4070.3 (PID:255-259)
    p, x = rpms["cf2p"] / k, rpms["cf2x"] / k
    tq0, tq1 = (p[1] - p[3]) / 2, -(p[0] - p[2]) / 2
    assert tq0 < 0                                            # restoring roll torque
    np.testing.assert_allclose(x[0] - x[2], -tq0 - tq1, rtol=1e-9, atol=1e-6)
    np.testing.assert_allclose(x[1] - x[3], -tq0 + tq1, rtol=1e-9, atol=1e-6)


def test_cf2p_hover_fixed_point():
    """K4 for CF2P: level, at rest, target = position ⇒ every motor at HOVER_RPM
    (the mixer multiplies zero torques; PID:188-259)."""
    s, _ = _sim("cf2p", act="one_d_pid")
    s.step(np.zeros((1, 1, 1), np.float32))
    st = s.get_state(0)
    np.testing.assert_allclose(st[F_RPM:F_RPM + 4, 0], C["HOVER_RPM"], rtol=1e-12)
    np.testing.assert_allclose(st[F_W:F_W + 3, 0], 0, atol=1e-12)
