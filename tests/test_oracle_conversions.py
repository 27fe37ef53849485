"""Pin the oracle's third-party arithmetic against scipy (present in this container).

The reference delegates rotations to pybullet (getMatrixFromQuaternion,
getEulerFromQuaternion) and scipy.spatial.transform.Rotation (DSLPIDControl.py:4,
205, 242-244).  pybullet is absent, so its conversions are checked against scipy's
equivalent conventions; the DSL PID is re-derived here a second time, in numpy,
line by line from DSLPIDControl.py *with the scipy calls the reference makes*, and
compared to the oracle's C++ restatement (which replaces the scipy round trip by
the identity).
"""
import math

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import qs_oracle as Q

RNG = np.random.default_rng(1234)


def rand_quats(n):
    q = RNG.normal(size=(n, 4))
    return q / np.linalg.norm(q, axis=1, keepdims=True)


def test_quat_to_matrix_matches_scipy_and_normalises():
    for q in rand_quats(200):
        want = Rotation.from_quat(q).as_matrix()          # scipy order x,y,z,w = pybullet order
        np.testing.assert_allclose(Q.quat_to_matrix(q), want, atol=1e-14)
        # btMatrix3x3::setRotation uses s = 2/|q|^2: a scaled quaternion gives the same matrix
        np.testing.assert_allclose(Q.quat_to_matrix(q * 1.37), want, atol=1e-14)


def test_euler_from_quat_matches_scipy_xyz():
    """pybullet rpy = extrinsic x-y-z (R = Rz(yaw) Ry(pitch) Rx(roll)) = scipy 'xyz'."""
    for q in rand_quats(200):
        rpy = Q.euler_from_quat(q)
        if abs(rpy[1]) > 1.5:
            continue   # near gimbal lock both libraries pick different but equivalent triples
        np.testing.assert_allclose(rpy, Rotation.from_quat(q).as_euler("xyz"), atol=1e-12)


def test_euler_gimbal_branch():
    q = Rotation.from_euler("xyz", [0.0, np.pi / 2, 0.3]).as_quat()
    rpy = Q.euler_from_quat(q)
    assert rpy[0] == 0.0 and rpy[1] == pytest.approx(np.pi / 2)
    np.testing.assert_allclose(Rotation.from_euler("xyz", rpy).as_matrix(), Rotation.from_quat(q).as_matrix(),
                               atol=1e-5)


def test_integrate_q_is_body_frame_exponential_map():
    """BaseAviary._integrateQ (BA:879-892) = q ⊗ exp(ω·dt) with ω in the body frame."""
    for q in rand_quats(50):
        w = RNG.normal(size=3) * 5
        dt = 1 / 240
        got = Q.integrate_q(q, w, dt)
        want = (Rotation.from_quat(q) * Rotation.from_rotvec(w * dt)).as_matrix()
        np.testing.assert_allclose(Rotation.from_quat(got).as_matrix(), want, atol=1e-13)
        assert np.linalg.norm(got) == pytest.approx(1.0, abs=1e-14)   # norm-preserving, no renormalisation
    q0 = np.array([0.1, 0.2, 0.3, 0.9])
    np.testing.assert_array_equal(Q.integrate_q(q0, [1e-9, 0, 0], 1 / 240), q0)   # np.isclose(|ω|, 0) branch


# ---------------------------------------------------------------- DSL PID
P_FOR, I_FOR, D_FOR = np.array([.4, .4, 1.25]), np.array([.05, .05, .05]), np.array([.2, .2, .5])
P_TOR, I_TOR, D_TOR = np.array([70000., 70000., 60000.]), np.array([.0, .0, 500.]), np.array([20000., 20000., 12000.])
MIXER = np.array([[-.5, -.5, -1], [-.5, .5, 1], [.5, .5, -1], [.5, -.5, 1]])
KF, GRAV = 3.16e-10, 9.8 * 0.027


def pybullet_matrix(q):
    return Q.quat_to_matrix(q)


def pybullet_euler(q):
    return Q.euler_from_quat(q)


def reference_pid(state, dt, cur_pos, cur_quat, cur_vel, target_pos, target_rpy, target_vel):
    """DSLPIDControl.computeControl restated in numpy with the reference's scipy calls."""
    int_pos, int_rpy, last_rpy = state[0:3].copy(), state[3:6].copy(), state[6:9].copy()
    # _dslPIDPositionControl (PID:187-208)
    cur_rotation = pybullet_matrix(cur_quat)
    pos_e = target_pos - cur_pos
    vel_e = target_vel - cur_vel
    int_pos = int_pos + pos_e * dt
    int_pos = np.clip(int_pos, -2., 2.)
    int_pos[2] = np.clip(int_pos[2], -0.15, .15)
    target_thrust = P_FOR * pos_e + I_FOR * int_pos + D_FOR * vel_e + np.array([0, 0, GRAV])
    scalar_thrust = max(0., np.dot(target_thrust, cur_rotation[:, 2]))
    thrust = (math.sqrt(scalar_thrust / (4 * KF)) - 4070.3) / 0.2685
    target_z_ax = target_thrust / np.linalg.norm(target_thrust)
    target_x_c = np.array([math.cos(target_rpy[2]), math.sin(target_rpy[2]), 0])
    target_y_ax = np.cross(target_z_ax, target_x_c) / np.linalg.norm(np.cross(target_z_ax, target_x_c))
    target_x_ax = np.cross(target_y_ax, target_z_ax)
    target_rotation = (np.vstack([target_x_ax, target_y_ax, target_z_ax])).transpose()
    target_euler = (Rotation.from_matrix(target_rotation)).as_euler('XYZ', degrees=False)
    # _dslPIDAttitudeControl (PID:240-259)
    cur_rpy = np.array(pybullet_euler(cur_quat))
    target_quat = (Rotation.from_euler('XYZ', target_euler, degrees=False)).as_quat()
    w, x, y, z = target_quat
    target_rotation = (Rotation.from_quat([w, x, y, z])).as_matrix()
    rot_matrix_e = np.dot((target_rotation.transpose()), cur_rotation) - np.dot(cur_rotation.transpose(), target_rotation)
    rot_e = np.array([rot_matrix_e[2, 1], rot_matrix_e[0, 2], rot_matrix_e[1, 0]])
    rpy_rates_e = np.zeros(3) - (cur_rpy - last_rpy) / dt
    last_rpy = cur_rpy
    int_rpy = int_rpy - rot_e * dt
    int_rpy = np.clip(int_rpy, -1500., 1500.)
    int_rpy[0:2] = np.clip(int_rpy[0:2], -1., 1.)
    target_torques = - P_TOR * rot_e + D_TOR * rpy_rates_e + I_TOR * int_rpy
    target_torques = np.clip(target_torques, -3200, 3200)
    pwm = thrust + np.dot(MIXER, target_torques)
    pwm = np.clip(pwm, 20000, 65535)
    return 0.2685 * pwm + 4070.3, np.concatenate([int_pos, int_rpy, last_rpy])


def test_dsl_pid_matches_scipy_restatement():
    worst = 0.0
    for k in range(300):
        q = rand_quats(1)[0]
        if k % 3 == 0:   # near-level attitudes as in flight
            q = Rotation.from_euler("xyz", RNG.normal(size=3) * [0.2, 0.2, 1.0]).as_quat()
        state = RNG.normal(size=9) * [0.3, 0.3, 0.05, 0.5, 0.5, 50, 0.2, 0.2, 1.0]
        pos, vel = RNG.normal(size=3), RNG.normal(size=3) * 0.5
        tpos = pos + RNG.normal(size=3) * 0.2
        trpy = np.array([0, 0, RNG.uniform(-3, 3)])
        tvel = RNG.normal(size=3) * 0.25
        want_rpm, want_state = reference_pid(state, 1 / 30, pos, q, vel, tpos, trpy, tvel)
        got_rpm, got_state = Q.dsl_pid(state, pos, q, vel, tpos, trpy, tvel, ctrl_dt=1 / 30)
        np.testing.assert_allclose(got_state, want_state, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(got_rpm, want_rpm, rtol=1e-9, atol=1e-6)
        worst = max(worst, float(np.abs(got_rpm - want_rpm).max()))
    assert worst < 1e-6
