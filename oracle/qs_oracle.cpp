// qs_oracle.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the
// reference's per-control-step drone update, used as the parity checker and
// as the bench's cpu_baseline ("port").  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it.  The product path never does.
//
// PARITY STATUS: "parity unpinned" against the reference itself.  The
// reference (pure Python on pybullet 3.2.7 + scipy) cannot be imported or run
// in this pipeline (execution denied; pybullet absent) and its
// tests hold no golden vectors.  This restatement is pinned by
// (1) the known-answer tests K1–K9 derived from the reference text
// (tests/test_oracle_kat.py), (2) scipy's Rotation for the conversions the
// reference delegates to scipy/pybullet (tests/test_oracle_conversions.py),
// and (3) committed golden vectors generated from it (tests/golden/).
//
// Every function names the reference function it restates (file:line, paths
// relative to gym_pybullet_drones/).  Arithmetic follows the reference's
// operation order so the fp64 build reproduces numpy's rounding closely.
// Third-party arithmetic restated from its published algorithm (external,
// unverified in this container):
//   - pybullet getMatrixFromQuaternion = btMatrix3x3::setRotation (s = 2/|q|^2)
//   - pybullet getEulerFromQuaternion (pybullet.c; asin branch at ±0.99999)
//   - scipy Rotation XYZ round trip in DSLPIDControl = identity on SO(3)
//     (checked numerically against scipy in tests)

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <string>
#include <algorithm>
#include <memory>
#include <omp.h>

#include "quadswarm.h"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11 "Random123") — the counter-based RNG the
// build uses for resets and the synthetic random policy (SURVEY §7 hard-3).
// ---------------------------------------------------------------------------
struct U4 { uint32_t v[4]; };
inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += W0; k1 += W1; }
    uint64_t p0 = (uint64_t)M0 * c.v[0];
    uint64_t p1 = (uint64_t)M1 * c.v[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    U4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0;
    n.v[1] = lo1;
    n.v[2] = hi0 ^ c.v[3] ^ k1;
    n.v[3] = lo0;
    c = n;
  }
  return c;
}
// 24-bit uniform in [0,1): exactly representable in float and double.
inline double u01(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }

enum { STREAM_ACT = 1, STREAM_RESET = 2 };

// ---------------------------------------------------------------------------
// Constants: cf2x.urdf:5, 11-12, 34 parsed as BaseAviary._parseURDFParameters
// (BaseAviary.py:985-1017); derived constants BaseAviary.py:117-128.
// ---------------------------------------------------------------------------
struct Consts {
  double G = 9.8, M = 0.027, L = 0.0397, T2W = 2.25;
  double IXX = 1.4e-5, IYY = 1.4e-5, IZZ = 2.17e-5;
  double KF = 3.16e-10, KM = 7.94e-12;
  double COLL_H = 0.025, COLL_Z_OFF = 0.0, MAX_SPEED_KMH = 30.0;
  double GND_EFF_COEFF = 11.36859, PROP_RADIUS = 2.31348e-2;
  double DRAG_XY = 9.1785e-7, DRAG_Z = 10.311e-7;
  double DW1 = 2267.18, DW2 = 0.16, DW3 = -0.11;
  double GRAVITY, HOVER_RPM, MAX_RPM, MAX_THRUST, GND_EFF_H_CLIP;
  // prop link COM offsets (cf2x.urdf:42-79) — where LINK_FRAME forces act
  double PROP_XY[4][2] = {{0.028, -0.028}, {-0.028, -0.028}, {-0.028, 0.028}, {0.028, 0.028}};
  // DroneModel.CF2P (QS_FLAG_CF2P): cf2p.urdf differs from cf2x.urdf only in the
  // inertia (cf2p.urdf:12) and the prop links, on the body axes at L (cf2p.urdf:42-79)
  double IXX_P = 2.3951e-5, IYY_P = 2.3951e-5, IZZ_P = 3.2347e-5;
  double PROP_XY_P[4][2] = {{0.0397, 0}, {0, 0.0397}, {-0.0397, 0}, {0, -0.0397}};
  Consts() {
    GRAVITY = G * M;                                           // BA:117
    HOVER_RPM = std::sqrt(GRAVITY / (4 * KF));                 // BA:118
    MAX_RPM = std::sqrt((T2W * GRAVITY) / (4 * KF));           // BA:119
    MAX_THRUST = (4 * KF * MAX_RPM * MAX_RPM);                 // BA:120
    GND_EFF_H_CLIP = 0.25 * PROP_RADIUS *
        std::sqrt((15 * MAX_RPM * MAX_RPM * KF * GND_EFF_COEFF) / MAX_THRUST);  // BA:128
  }
};
const Consts C;

// DSLPIDControl gains (DSLPIDControl.py:37-53); CF2X mixer.
const double P_FOR[3] = {.4, .4, 1.25}, I_FOR[3] = {.05, .05, .05}, D_FOR[3] = {.2, .2, .5};
const double P_TOR[3] = {70000., 70000., 60000.}, I_TOR[3] = {.0, .0, 500.}, D_TOR[3] = {20000., 20000., 12000.};
const double PWM2RPM_SCALE = 0.2685, PWM2RPM_CONST = 4070.3, MIN_PWM = 20000, MAX_PWM = 65535;
const double MIXER[4][3] = {{-.5, -.5, -1}, {-.5, .5, 1}, {.5, .5, -1}, {.5, -.5, 1}};
const double MIXER_P[4][3] = {{0, -1, -1}, {+1, 0, 1}, {0, 1, -1}, {-1, 0, 1}};   // CF2P (DSLPIDControl.py:54-60)

template <class R> inline R clip(R x, R lo, R hi) { return x < lo ? lo : (x > hi ? hi : x); }

// pybullet getMatrixFromQuaternion == btMatrix3x3::setRotation (external):
// normalises implicitly through s = 2/|q|^2.  Row-major out[3][3].
template <class R> void quat_to_matrix(const R q[4], R m[3][3]) {
  R x = q[0], y = q[1], z = q[2], w = q[3];
  R d = x * x + y * y + z * z + w * w;
  R s = R(2) / d;
  R xs = x * s, ys = y * s, zs = z * s;
  R wx = w * xs, wy = w * ys, wz = w * zs;
  R xx = x * xs, xy = x * ys, xz = x * zs;
  R yy = y * ys, yz = y * zs, zz = z * zs;
  m[0][0] = R(1) - (yy + zz); m[0][1] = xy - wz; m[0][2] = xz + wy;
  m[1][0] = xy + wz; m[1][1] = R(1) - (xx + zz); m[1][2] = yz - wx;
  m[2][0] = xz - wy; m[2][1] = yz + wx; m[2][2] = R(1) - (xx + yy);
}

// pybullet getEulerFromQuaternion (pybullet.c, external): roll, pitch, yaw.
template <class R> void euler_from_quat(const R q[4], R rpy[3]) {
  R sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
  R sarg = R(-2) * (q[0] * q[2] - q[3] * q[1]);
  if (sarg <= R(-0.99999)) {
    rpy[0] = 0; rpy[1] = R(-0.5 * M_PI); rpy[2] = R(2) * std::atan2(q[0], -q[1]);
  } else if (sarg >= R(0.99999)) {
    rpy[0] = 0; rpy[1] = R(0.5 * M_PI); rpy[2] = R(2) * std::atan2(-q[0], q[1]);
  } else {
    rpy[0] = std::atan2(R(2) * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
    rpy[1] = std::asin(sarg);
    rpy[2] = std::atan2(R(2) * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
  }
}

template <class R> inline void cross3(const R a[3], const R b[3], R o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
template <class R> inline R norm3(const R a[3]) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

// ---------------------------------------------------------------------------
// Per-drone state (what BaseAviary keeps in pybullet + numpy arrays).
// ---------------------------------------------------------------------------
template <class R> struct Drone {
  R pos[3], quat[4], vel[3], rpy_rates[3], last_rpm[4];
  R int_pos[3], int_rpy[3], last_rpy[3];   // DSLPIDControl.reset (PID:65-78)
  R target[3];                             // MultiHover TARGET_POS
  R rpy[3], ang_v[3];                      // readback (BA:509-519), derived
};

template <class R> struct Params {
  int task, D, E, A, H, S, act_type, O, physics;
  uint32_t aux, flags;
  R dt, ctrl_dt, ep_len_sec;
  int pyb_freq;
  R KF, KM, M, GRAVITY_DYN, Jd[3], Jinv[3], L_SQRT2, HOVER_RPM, SPEED_LIMIT;
  R G_PID;  // BaseControl.GRAVITY = g*m (BaseControl.py:35)
  R DRAG[3], GND_COEFF, PROP_R, GND_CLIP, DW1, DW2, DW3, PROP_XY[4][2];
  bool cf2p;       // DroneModel.CF2P: its torques (BA:852-853), inertia, props and mixer
  R L;             // arm length (the CF2P torques)
  R MIX[4][3];     // DSLPIDControl.MIXER_MATRIX (PID:48-60)
  R sp_R, sp_OMEGA, sp_VZ, sp_center[3];
  std::vector<R> orig_xyz;  // [D][3] ORIGINAL_INIT_XYZS (MH:78-79) / INIT_XYZS
};

// DSLPIDControl.computeControl (PID:82-145) = _dslPIDPositionControl
// (PID:149-208) + _dslPIDAttitudeControl (PID:212-259).  rpm out[4].
template <class R>
void dsl_pid_compute_control(const Params<R>& P, Drone<R>& d, const R cur_pos[3], const R cur_quat[4],
                             const R cur_vel[3], const R target_pos[3], const R target_rpy[3],
                             const R target_vel[3], R rpm[4]) {
  const R dt = P.ctrl_dt;
  // ---- position control (PID:187-208)
  R cur_rot[3][3];
  quat_to_matrix(cur_quat, cur_rot);
  R pos_e[3], vel_e[3];
  for (int i = 0; i < 3; ++i) { pos_e[i] = target_pos[i] - cur_pos[i]; vel_e[i] = target_vel[i] - cur_vel[i]; }
  for (int i = 0; i < 3; ++i) d.int_pos[i] = clip<R>(d.int_pos[i] + pos_e[i] * dt, R(-2.), R(2.));
  d.int_pos[2] = clip<R>(d.int_pos[2], R(-0.15), R(.15));
  R tt[3];
  for (int i = 0; i < 3; ++i)
    tt[i] = R(P_FOR[i]) * pos_e[i] + R(I_FOR[i]) * d.int_pos[i] + R(D_FOR[i]) * vel_e[i] + (i == 2 ? P.G_PID : R(0));
  R st = tt[0] * cur_rot[0][2] + tt[1] * cur_rot[1][2] + tt[2] * cur_rot[2][2];
  R scalar_thrust = st > R(0) ? st : R(0);
  R thrust = (std::sqrt(scalar_thrust / (R(4) * P.KF)) - R(PWM2RPM_CONST)) / R(PWM2RPM_SCALE);
  R ttn = norm3(tt);
  R z_ax[3] = {tt[0] / ttn, tt[1] / ttn, tt[2] / ttn};
  R x_c[3] = {std::cos(target_rpy[2]), std::sin(target_rpy[2]), R(0)};
  R yc[3];
  cross3(z_ax, x_c, yc);
  R ycn = norm3(yc);
  R y_ax[3] = {yc[0] / ycn, yc[1] / ycn, yc[2] / ycn};
  R x_ax[3];
  cross3(y_ax, z_ax, x_ax);
  // target_rotation = vstack([x,y,z]).T; the scipy from_matrix→as_euler('XYZ')
  // →from_euler→as_quat→from_quat→as_matrix round trip (PID:205, 242-244) is
  // the identity on SO(3) (the w,x,y,z relabelling at PID:243 cancels).
  R Rt[3][3];
  for (int i = 0; i < 3; ++i) { Rt[i][0] = x_ax[i]; Rt[i][1] = y_ax[i]; Rt[i][2] = z_ax[i]; }
  // ---- attitude control (PID:240-259)
  R cur_rpy[3];
  euler_from_quat(cur_quat, cur_rpy);
  // rot_matrix_e = Rt^T R - R^T Rt
  R e[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      R a = Rt[0][i] * cur_rot[0][j] + Rt[1][i] * cur_rot[1][j] + Rt[2][i] * cur_rot[2][j];
      R b = cur_rot[0][i] * Rt[0][j] + cur_rot[1][i] * Rt[1][j] + cur_rot[2][i] * Rt[2][j];
      e[i][j] = a - b;
    }
  R rot_e[3] = {e[2][1], e[0][2], e[1][0]};
  R rates_e[3];
  for (int i = 0; i < 3; ++i) rates_e[i] = R(0) - (cur_rpy[i] - d.last_rpy[i]) / dt;   // target_rpy_rates = 0
  for (int i = 0; i < 3; ++i) d.last_rpy[i] = cur_rpy[i];
  for (int i = 0; i < 3; ++i) d.int_rpy[i] = clip<R>(d.int_rpy[i] - rot_e[i] * dt, R(-1500.), R(1500.));
  for (int i = 0; i < 2; ++i) d.int_rpy[i] = clip<R>(d.int_rpy[i], R(-1.), R(1.));
  R tq[3];
  for (int i = 0; i < 3; ++i)
    tq[i] = clip<R>(-R(P_TOR[i]) * rot_e[i] + R(D_TOR[i]) * rates_e[i] + R(I_TOR[i]) * d.int_rpy[i], R(-3200), R(3200));
  for (int m = 0; m < 4; ++m) {
    R pwm = thrust + (P.MIX[m][0] * tq[0] + P.MIX[m][1] * tq[1] + P.MIX[m][2] * tq[2]);
    pwm = clip<R>(pwm, R(MIN_PWM), R(MAX_PWM));
    rpm[m] = R(PWM2RPM_SCALE) * pwm + R(PWM2RPM_CONST);
  }
}

// BaseRLAviary._preprocessAction for one drone (BRL:187-239).
template <class R>
void preprocess_action(const Params<R>& P, Drone<R>& d, const float* a, R rpm[4]) {
  const R zero3[3] = {0, 0, 0};
  switch (P.act_type) {
    case QS_ACT_RPM:  // BRL:191-192
      for (int m = 0; m < 4; ++m) rpm[m] = P.HOVER_RPM * (R(1) + R(0.05) * R(a[m]));
      break;
    case QS_ACT_ONE_D_RPM: {  // BRL:224-225
      R r = P.HOVER_RPM * (R(1) + R(0.05) * R(a[0]));
      for (int m = 0; m < 4; ++m) rpm[m] = r;
    } break;
    case QS_ACT_ONE_D_PID: {  // BRL:226-235
      R tp[3] = {d.pos[0], d.pos[1], d.pos[2] + R(0.1) * R(a[0])};
      dsl_pid_compute_control(P, d, d.pos, d.quat, d.vel, tp, zero3, zero3, rpm);
    } break;
    case QS_ACT_VEL: {  // BRL:208-223
      R v[3] = {R(a[0]), R(a[1]), R(a[2])};
      R n = norm3(v);
      R unit[3] = {0, 0, 0};
      if (n != R(0)) for (int i = 0; i < 3; ++i) unit[i] = v[i] / n;
      R s = P.SPEED_LIMIT * std::fabs(R(a[3]));
      R tv[3] = {s * unit[0], s * unit[1], s * unit[2]};
      R trpy[3] = {0, 0, d.rpy[2]};
      dsl_pid_compute_control(P, d, d.pos, d.quat, d.vel, d.pos, trpy, tv, rpm);
    } break;
    case QS_ACT_PID: {  // BRL:193-207 + BaseAviary._calculateNextStep (BA:1108-1150)
      R dir[3] = {R(a[0]) - d.pos[0], R(a[1]) - d.pos[1], R(a[2]) - d.pos[2]};
      R dist = norm3(dir);
      R np_[3];
      if (dist <= R(1)) { for (int i = 0; i < 3; ++i) np_[i] = R(a[i]); }
      else { for (int i = 0; i < 3; ++i) np_[i] = d.pos[i] + (dir[i] / dist) * R(1); }
      dsl_pid_compute_control(P, d, d.pos, d.quat, d.vel, np_, zero3, zero3, rpm);
    } break;
  }
}

// BaseAviary._integrateQ (BA:879-892).
template <class R> void integrate_q(R q[4], const R w[3], R dt) {
  R p = w[0], qq = w[1], r = w[2];
  R wn = std::sqrt(p * p + qq * qq + r * r);
  if (std::fabs(wn) <= R(1e-8)) return;  // np.isclose(omega_norm, 0)
  R lam[4][4] = {{0, r, -qq, p}, {-r, 0, p, qq}, {qq, -p, 0, r}, {-p, -qq, -r, 0}};
  R th = wn * dt / R(2);
  R c = std::cos(th), s = std::sin(th);
  R k = R(2) / wn;
  R out[4];
  for (int i = 0; i < 4; ++i) {
    R acc = 0;
    for (int j = 0; j < 4; ++j) {
      R mij = (i == j ? c : R(0)) + k * (lam[i][j] * R(0.5)) * s;
      acc += mij * q[j];
    }
    out[i] = acc;
  }
  for (int i = 0; i < 4; ++i) q[i] = out[i];
}

// Snapshot of the drones at substep start (BA:346-347 readback).
template <class R> struct Snap { R pos[3], quat[4], vel[3], rpy[3]; };

// BaseAviary._dynamics (BA:815-877) plus, for aux != 0, the build-defined
// addition of _groundEffect / _drag / _downwash forces (BA:715-811) to the
// DYN force and torque sums (SURVEY §8 physics-mode note).
template <class R>
void dynamics(const Params<R>& P, Drone<R>& d, const R rpm[4], const Snap<R>* snaps, int self) {
  R rot[3][3];
  quat_to_matrix(d.quat, rot);
  R f[4], zt[4];
  for (int m = 0; m < 4; ++m) { f[m] = rpm[m] * rpm[m] * P.KF; zt[m] = rpm[m] * rpm[m] * P.KM; }
  R thrust_z = ((f[0] + f[1]) + f[2]) + f[3];
  R body_z_extra = 0, tx_extra = 0, ty_extra = 0, fw_extra[3] = {0, 0, 0};
  if (P.aux & QS_AUX_GND) {  // _groundEffect (BA:731-750)
    const Snap<R>& sn = snaps[self];
    if (std::fabs(sn.rpy[0]) < R(M_PI / 2) && std::fabs(sn.rpy[1]) < R(M_PI / 2)) {
      R srot[3][3];
      quat_to_matrix(sn.quat, srot);
      for (int m = 0; m < 4; ++m) {
        R h = sn.pos[2] + (srot[2][0] * P.PROP_XY[m][0] + srot[2][1] * P.PROP_XY[m][1]);
        h = h < P.GND_CLIP ? P.GND_CLIP : h;
        R ratio = P.PROP_R / (R(4) * h);
        R g = rpm[m] * rpm[m] * P.KF * P.GND_COEFF * (ratio * ratio);
        body_z_extra += g;
        tx_extra += P.PROP_XY[m][1] * g;   // r x [0,0,g] = (ry g, -rx g, 0)
        ty_extra += -P.PROP_XY[m][0] * g;
      }
    }
  }
  if (P.aux & QS_AUX_DRAG) {  // _drag (BA:770-781): world force -DRAG∘v·Σ(2π rpm_last/60)
    const Snap<R>& sn = snaps[self];
    R srpm = 0;
    for (int m = 0; m < 4; ++m) srpm += R(2 * M_PI) * d.last_rpm[m] / R(60);
    for (int i = 0; i < 3; ++i) fw_extra[i] += (R(-1) * P.DRAG[i] * srpm) * sn.vel[i];
  }
  if (P.aux & QS_AUX_DW) {  // _downwash (BA:798-811), LINK_FRAME z force at the COM
    const Snap<R>& me = snaps[self];
    for (int j = 0; j < P.D; ++j) {
      R dz = snaps[j].pos[2] - me.pos[2];
      R dx = snaps[j].pos[0] - me.pos[0], dy = snaps[j].pos[1] - me.pos[1];
      R dxy = std::sqrt(dx * dx + dy * dy);
      if (dz > R(0) && dxy < R(10)) {
        R ratio = P.PROP_R / (R(4) * dz);
        R alpha = P.DW1 * (ratio * ratio);
        R beta = P.DW2 * dz + P.DW3;
        R q = dxy / beta;
        body_z_extra += -alpha * std::exp(R(-.5) * (q * q));
      }
    }
  }
  R tzb = thrust_z + body_z_extra;
  R fw[3] = {rot[0][2] * tzb, rot[1][2] * tzb, rot[2][2] * tzb - P.GRAVITY_DYN};
  for (int i = 0; i < 3; ++i) fw[i] += fw_extra[i];
  R z_torque = ((-zt[0] + zt[1]) - zt[2]) + zt[3];
  // CF2X (BA:849-851)
  R x_torque, y_torque;
  if (P.cf2p) {   // BaseAviary.py:852-853
    x_torque = (f[1] - f[3]) * P.L + tx_extra;
    y_torque = (-f[0] + f[2]) * P.L + ty_extra;
  } else {        // BaseAviary.py:849-850
    x_torque = -(((f[0] + f[1]) - f[2]) - f[3]) * P.L_SQRT2 + tx_extra;
    y_torque = (((-f[0] + f[1]) + f[2]) - f[3]) * P.L_SQRT2 + ty_extra;
  }
  R w[3] = {d.rpy_rates[0], d.rpy_rates[1], d.rpy_rates[2]};
  R Jw[3] = {P.Jd[0] * w[0], P.Jd[1] * w[1], P.Jd[2] * w[2]};
  R wxJw[3];
  cross3(w, Jw, wxJw);
  R tq[3] = {x_torque - wxJw[0], y_torque - wxJw[1], z_torque - wxJw[2]};
  R wdot[3] = {P.Jinv[0] * tq[0], P.Jinv[1] * tq[1], P.Jinv[2] * tq[2]};
  for (int i = 0; i < 3; ++i) d.vel[i] = d.vel[i] + P.dt * (fw[i] / P.M);
  for (int i = 0; i < 3; ++i) w[i] = w[i] + P.dt * wdot[i];
  for (int i = 0; i < 3; ++i) d.pos[i] = d.pos[i] + P.dt * d.vel[i];
  integrate_q(d.quat, w, P.dt);
  // resetBaseVelocity(vel, R_old·ω) (BA:871-875); rpy_rates stored (BA:877)
  for (int i = 0; i < 3; ++i) {
    d.ang_v[i] = rot[i][0] * w[0] + rot[i][1] * w[1] + rot[i][2] * w[2];
    d.rpy_rates[i] = w[i];
  }
}

// ---------------------------------------------------------------------------
// Physics.PYB: the drone as Bullet integrates it (p.stepSimulation, BA:369-370)
// after BaseAviary._physics (BA:679-711) applied its forces.  Restated from the
// published btMultiBody algorithm (pybullet 3.2.7, external — unverified here,
// parity unpinned):
//  * cf2x.urdf loads as one rigid body (the prop and COM links are fixed and
//    massless): mass M, inertia diag(IXX, IYY, IZZ) about the base COM.
//  * each prop force [0,0,f_i] acts in LINK_FRAME at its link's COM
//    (assets/cf2x.urdf:42-79) → body torque r_i × f_i; the yaw torque acts on
//    link 4 (the COM) in LINK_FRAME; gravity [0,0,-G·M] (BA:479).
//  * btMultiBody's default damping (linear = angular = 0.04, not removed by
//    BA:492-494) as its bias force m·v·(k + k|v|), I·ω·(k + k|ω|), and the
//    gyroscopic term ω × Iω, evaluated at the step's starting velocities.
//  * semi-implicit Euler: velocities first, then the position with the new
//    velocity, then the orientation by the exponential map of the world
//    angular velocity (btMultiBody::stepPositionsMultiDof: |ω|dt clamped to
//    π/4, sinc Taylor branch below |ω| = 0.001), renormalised.
//  * ground plane z = 0 (plane.urdf) against the drone's collision cylinder
//    (r 0.06, length 0.025, cf2x.urdf:32-35): a penetrating lowest point is
//    pushed back to z = 0 and the downward normal velocity removed
//    (inelastic, frictionless — Bullet's contact solver is not restated).
// With aux forces (PYB_GND / PYB_DRAG / PYB_DW) the same external forces as
// DYN's aux path are applied (BA:715-811).
// ---------------------------------------------------------------------------
constexpr double kPybDamping = 0.04;
constexpr double kCylR = 0.06, kCylHalfLen = 0.0125;

template <class R>
void pyb_dynamics(const Params<R>& P, Drone<R>& d, const R rpm[4], const Snap<R>* snaps, int self) {
  R rot[3][3];
  quat_to_matrix(d.quat, rot);
  R f[4], zt[4];
  for (int m = 0; m < 4; ++m) { f[m] = rpm[m] * rpm[m] * P.KF; zt[m] = rpm[m] * rpm[m] * P.KM; }
  // body-frame force (z) and torque of the prop forces at the prop-link COMs
  R fzb = ((f[0] + f[1]) + f[2]) + f[3];
  R tb[3] = {0, 0, ((-zt[0] + zt[1]) - zt[2]) + zt[3]};
  for (int m = 0; m < 4; ++m) { tb[0] += P.PROP_XY[m][1] * f[m]; tb[1] += -P.PROP_XY[m][0] * f[m]; }
  R fw_extra[3] = {0, 0, 0};
  if (P.aux & QS_AUX_GND) {  // _groundEffect (BA:731-750): LINK_FRAME forces at the props
    const Snap<R>& sn = snaps[self];
    if (std::fabs(sn.rpy[0]) < R(M_PI / 2) && std::fabs(sn.rpy[1]) < R(M_PI / 2)) {
      R srot[3][3];
      quat_to_matrix(sn.quat, srot);
      for (int m = 0; m < 4; ++m) {
        R h = sn.pos[2] + (srot[2][0] * P.PROP_XY[m][0] + srot[2][1] * P.PROP_XY[m][1]);
        h = h < P.GND_CLIP ? P.GND_CLIP : h;
        R ratio = P.PROP_R / (R(4) * h);
        R g = rpm[m] * rpm[m] * P.KF * P.GND_COEFF * (ratio * ratio);
        fzb += g;
        tb[0] += P.PROP_XY[m][1] * g;
        tb[1] += -P.PROP_XY[m][0] * g;
      }
    }
  }
  if (P.aux & QS_AUX_DRAG) {  // _drag (BA:770-781): world force from the previous rpm
    const Snap<R>& sn = snaps[self];
    R srpm = 0;
    for (int m = 0; m < 4; ++m) srpm += R(2 * M_PI) * d.last_rpm[m] / R(60);
    for (int i = 0; i < 3; ++i) fw_extra[i] += (R(-1) * P.DRAG[i] * srpm) * sn.vel[i];
  }
  if (P.aux & QS_AUX_DW) {  // _downwash (BA:798-811): LINK_FRAME z force on link 4 (the COM)
    const Snap<R>& me = snaps[self];
    for (int j = 0; j < P.D; ++j) {
      R dz = snaps[j].pos[2] - me.pos[2];
      R dx = snaps[j].pos[0] - me.pos[0], dy = snaps[j].pos[1] - me.pos[1];
      R dxy = std::sqrt(dx * dx + dy * dy);
      if (dz > R(0) && dxy < R(10)) {
        R ratio = P.PROP_R / (R(4) * dz);
        R alpha = P.DW1 * (ratio * ratio);
        R beta = P.DW2 * dz + P.DW3;
        R q = dxy / beta;
        fzb += -alpha * std::exp(R(-.5) * (q * q));
      }
    }
  }
  const R k = R(kPybDamping);
  // linear: world force, damping, semi-implicit velocity update
  R Fw[3] = {rot[0][2] * fzb + fw_extra[0], rot[1][2] * fzb + fw_extra[1],
             (rot[2][2] * fzb - P.GRAVITY_DYN) + fw_extra[2]};
  R vn = norm3(d.vel);
  R vd = k + k * vn;
  R acc[3];
  for (int i = 0; i < 3; ++i) acc[i] = Fw[i] / P.M - vd * d.vel[i];
  // angular (body frame): torque − gyroscopic − damping
  R w[3] = {d.rpy_rates[0], d.rpy_rates[1], d.rpy_rates[2]};
  R Jw[3] = {P.Jd[0] * w[0], P.Jd[1] * w[1], P.Jd[2] * w[2]};
  R wxJw[3];
  cross3(w, Jw, wxJw);
  R wd = k + k * norm3(w);
  R wdot[3];
  for (int i = 0; i < 3; ++i) wdot[i] = P.Jinv[i] * ((tb[i] - wxJw[i]) - wd * Jw[i]);
  for (int i = 0; i < 3; ++i) d.vel[i] = d.vel[i] + P.dt * acc[i];
  for (int i = 0; i < 3; ++i) w[i] = w[i] + P.dt * wdot[i];
  for (int i = 0; i < 3; ++i) d.pos[i] = d.pos[i] + P.dt * d.vel[i];
  // orientation: exp map of the world angular velocity, then renormalise
  R ww[3];
  for (int i = 0; i < 3; ++i) ww[i] = rot[i][0] * w[0] + rot[i][1] * w[1] + rot[i][2] * w[2];
  R ang = norm3(ww);
  const R kMaxAng = R(0.25 * M_PI);
  if (ang * P.dt > kMaxAng) ang = kMaxAng / P.dt;
  R ax[3];
  if (ang < R(0.001)) {
    R c = R(0.5) * P.dt - (P.dt * P.dt * P.dt) * R(0.020833333333) * ang * ang;
    for (int i = 0; i < 3; ++i) ax[i] = ww[i] * c;
  } else {
    R c = std::sin(R(0.5) * ang * P.dt) / ang;
    for (int i = 0; i < 3; ++i) ax[i] = ww[i] * c;
  }
  R dw_ = std::cos(ang * P.dt * R(0.5));
  const R* q = d.quat;
  // Hamilton product dq ⊗ q, quaternions stored (x, y, z, w)
  R nq[4] = {dw_ * q[0] + ax[0] * q[3] + ax[1] * q[2] - ax[2] * q[1],
             dw_ * q[1] - ax[0] * q[2] + ax[1] * q[3] + ax[2] * q[0],
             dw_ * q[2] + ax[0] * q[1] - ax[1] * q[0] + ax[2] * q[3],
             dw_ * q[3] - ax[0] * q[0] - ax[1] * q[1] - ax[2] * q[2]};
  R qn = std::sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
  for (int i = 0; i < 4; ++i) d.quat[i] = nq[i] / qn;
  // ground plane: keep the collision cylinder's lowest point at z >= 0
  R nrot[3][3];
  quat_to_matrix(d.quat, nrot);
  R cz = std::fabs(nrot[2][2]);
  R sz = std::sqrt(std::max(R(0), R(1) - nrot[2][2] * nrot[2][2]));
  R zmin = d.pos[2] - (R(kCylHalfLen) * cz + R(kCylR) * sz);
  if (zmin < R(0)) {
    d.pos[2] -= zmin;
    if (d.vel[2] < R(0)) d.vel[2] = R(0);
  }
  // readback: getBaseVelocity's world angular velocity (BA:514-515) at the new pose
  for (int i = 0; i < 3; ++i) {
    d.ang_v[i] = nrot[i][0] * w[0] + nrot[i][1] * w[1] + nrot[i][2] * w[2];
    d.rpy_rates[i] = w[i];
  }
}

// Drone–drone contact of the PYB mode (Bullet keeps every drone's collision
// cylinder live: assets/cf2x.urdf:31-36, BaseAviary.py:484-491, the collision
// filter at BA:500-503 is commented out).  Restated like the ground plane:
// inelastic and frictionless, equal masses.  Pair (i, j), i < j in drone order,
// once per substep after every drone's step and ground check:
//   overlap if the centres are closer than 2r horizontally and closer than the
//   two tilted half-heights e = h|R22| + r·sqrt(1 − R22²) vertically;
//   separated along the axis of the smaller penetration (vertical, or the
//   horizontal centre line), each drone moved by half of it; if the pair is
//   approaching along that axis both take the mean of their velocity
//   components on it (the inelastic response), tangential velocity unchanged.
template <class R> void drone_contacts(Drone<R>* dr, int D) {
  const R r2 = R(2 * kCylR), h = R(kCylHalfLen), rr = R(kCylR);
  std::vector<R> ez(D);
  for (int i = 0; i < D; ++i) {
    R rot[3][3];
    quat_to_matrix(dr[i].quat, rot);
    const R c = rot[2][2];
    ez[i] = h * std::fabs(c) + rr * std::sqrt(std::max(R(0), R(1) - c * c));
  }
  for (int i = 0; i < D; ++i)
    for (int j = i + 1; j < D; ++j) {
      Drone<R>& a = dr[i];
      Drone<R>& b = dr[j];
      const R dx = b.pos[0] - a.pos[0], dy = b.pos[1] - a.pos[1], dz = b.pos[2] - a.pos[2];
      const R d2 = dx * dx + dy * dy;
      if (!(d2 < r2 * r2)) continue;
      const R pz = (ez[i] + ez[j]) - std::fabs(dz);
      if (!(pz > R(0))) continue;
      const R dxy = std::sqrt(d2);
      const R pxy = r2 - dxy;
      if (pz < pxy) {   // vertical separation; j is above i when dz >= 0
        const R sg = dz >= R(0) ? R(1) : R(-1);
        const R half = R(0.5) * pz;
        a.pos[2] = a.pos[2] - sg * half;
        b.pos[2] = b.pos[2] + sg * half;
        const R rel = (b.vel[2] - a.vel[2]) * sg;
        if (rel < R(0)) {
          const R m = R(0.5) * (a.vel[2] + b.vel[2]);
          a.vel[2] = m;
          b.vel[2] = m;
        }
      } else {          // horizontal separation along the centre line
        R nx = R(1), ny = R(0);
        if (dxy > R(0)) { nx = dx / dxy; ny = dy / dxy; }
        const R half = R(0.5) * pxy;
        a.pos[0] = a.pos[0] - nx * half; a.pos[1] = a.pos[1] - ny * half;
        b.pos[0] = b.pos[0] + nx * half; b.pos[1] = b.pos[1] + ny * half;
        const R rel = (b.vel[0] - a.vel[0]) * nx + (b.vel[1] - a.vel[1]) * ny;
        if (rel < R(0)) {
          const R hr = R(0.5) * rel;
          a.vel[0] = a.vel[0] + hr * nx; a.vel[1] = a.vel[1] + hr * ny;
          b.vel[0] = b.vel[0] - hr * nx; b.vel[1] = b.vel[1] - hr * ny;
        }
      }
    }
}

// ---------------------------------------------------------------------------
// The vectorised env (oracle of qs_handle).
// ---------------------------------------------------------------------------
template <class R> struct Sim {
  Params<R> P;
  int64_t env_offset;
  uint32_t k0 = 0, k1 = 0;
  std::vector<Drone<R>> drones;          // [E*D]
  std::vector<float> hist;               // [H][N][A]
  std::vector<int32_t> step_counter, episode, total_steps, ep_len;
  std::vector<double> ep_return;
  std::vector<qs_episode_rec> log;
  int reset_error = 0;

  int N() const { return P.E * P.D; }

  // MultiHoverAviary.reset (MH:75-110): rejection sampling of
  // ORIGINAL_INIT_XYZS + U(-.25,.25), z clipped to [0.1,1]; reject if any pair
  // < 0.5 m or any z < 0.1.  np.random is replaced by Philox:
  // try t uses counter (t, env, episode, (2<<24)|drone) for drone's 3 draws.
  // The first accepted t (sequential order) wins.  SpiralAviary keeps its
  // deterministic INIT_XYZS (SP:47-53).
  void draw_init(int e, R out[][3]) {
    const int D = P.D;
    const uint32_t genv = (uint32_t)(env_offset + e);
    if (P.task != QS_TASK_MULTIHOVER) {   // BaseAviary.reset: INIT_XYZS as given (BA:245-255)
      for (int d = 0; d < D; ++d) for (int i = 0; i < 3; ++i) out[d][i] = P.orig_xyz[d * 3 + i];
      return;
    }
    const uint32_t max_tries = 1u << 24;
    for (uint32_t t = 0; t < max_tries; ++t) {
      for (int d = 0; d < D; ++d) {
        U4 c = {{t, genv, (uint32_t)episode[e], (uint32_t)((STREAM_RESET << 24) | d)}};
        U4 r = philox4x32_10(c, k0, k1);
        for (int i = 0; i < 3; ++i) {
          R noise = R(0.5 * u01(r.v[i]) - 0.25);
          out[d][i] = P.orig_xyz[d * 3 + i] + noise;
        }
        out[d][2] = clip<R>(out[d][2], R(0.1), R(1.0));
      }
      bool bad = false;
      for (int a = 0; a < D && !bad; ++a)
        for (int b = a + 1; b < D && !bad; ++b) {
          R dx = out[a][0] - out[b][0], dy = out[a][1] - out[b][1], dz = out[a][2] - out[b][2];
          // volatile-free exact ordering: ((dx*dx + dy*dy) + dz*dz)
          R s = (dx * dx + dy * dy) + dz * dz;
          if (std::sqrt(s) < R(0.5)) bad = true;
        }
      for (int d = 0; d < D && !bad; ++d) if (out[d][2] < R(0.1)) bad = true;
      if (!bad) return;
    }
    reset_error = 1;
  }

  // BaseAviary.reset → _housekeeping (BA:245-255, 458-477) for one env.
  void reset_env(int e) {
    const int D = P.D;
    std::vector<R> tmp(D * 3);
    R(*init)[3] = reinterpret_cast<R(*)[3]>(tmp.data());
    draw_init(e, init);
    for (int d = 0; d < D; ++d) {
      Drone<R>& dr = drones[e * D + d];
      for (int i = 0; i < 3; ++i) {
        dr.pos[i] = init[d][i];
        dr.vel[i] = 0; dr.rpy_rates[i] = 0; dr.rpy[i] = 0; dr.ang_v[i] = 0;
      }
      dr.quat[0] = dr.quat[1] = dr.quat[2] = 0; dr.quat[3] = 1;   // getQuaternionFromEuler(0,0,0)
      for (int m = 0; m < 4; ++m) dr.last_rpm[m] = 0;             // BA:468
      // TARGET_POS = INIT_XYZS + [0,0,1/(i+1)] (MH:106)
      dr.target[0] = init[d][0]; dr.target[1] = init[d][1];
      dr.target[2] = init[d][2] + R(1.0 / (d + 1));
    }
    step_counter[e] = 0;
  }

  void hist_slot_obs(int e, int d, float* o) const {
    // obs action history, oldest first (BRL:317-318); ring newest = total-1
    const int N_ = N(), A = P.A, H = P.H, a = e * P.D + d;
    for (int i = 0; i < H; ++i) {
      int slot = (int)((total_steps[e] + i) % H);
      for (int k = 0; k < A; ++k) o[12 + i * A + k] = hist[((size_t)slot * N_ + a) * A + k];
    }
  }

  // SpiralFormationAviary._spiral_reference (SP:82-99).
  void spiral_ref(int e, int d, R pos_ref[3], R vel_ref[3], R& phase) const {
    R t = R((double)step_counter[e] / (double)P.pyb_freq);
    phase = P.sp_OMEGA * t + R(2 * M_PI) * R(d) / R(P.D);
    pos_ref[0] = P.sp_center[0] + P.sp_R * std::cos(phase);
    pos_ref[1] = P.sp_center[1] + P.sp_R * std::sin(phase);
    pos_ref[2] = R(0.3) + P.sp_VZ * t;
    vel_ref[0] = -P.sp_R * P.sp_OMEGA * std::sin(phase);
    vel_ref[1] = P.sp_R * P.sp_OMEGA * std::cos(phase);
    vel_ref[2] = P.sp_VZ;
  }

  // BaseRLAviary._computeObs (BRL:307-319) + SpiralAviary._computeObs
  // (SP:120-146).  float32 output row per drone.
  void compute_obs(int e, float* obs_env) const {
    const int D = P.D, O = P.O;
    for (int d = 0; d < D; ++d) {
      const Drone<R>& dr = drones[e * D + d];
      float* o = obs_env + (size_t)d * O;
      for (int i = 0; i < 3; ++i) {
        o[i] = (float)dr.pos[i]; o[3 + i] = (float)dr.rpy[i];
        o[6 + i] = (float)dr.vel[i]; o[9 + i] = (float)dr.ang_v[i];
      }
      hist_slot_obs(e, d, o);
      if (P.task == QS_TASK_SPIRAL) {
        R pr[3], vr[3], ph;
        spiral_ref(e, d, pr, vr, ph);
        float* x = o + 12 + P.H * P.A;
        for (int i = 0; i < 3; ++i) {
          x[i] = (float)(pr[i] - dr.pos[i]);
          x[3 + i] = (float)(vr[i] - dr.quat[i]);   // "vel" = state[3:6] = quat xyz (SP:130)
          x[8 + i] = (float)vr[i];
        }
        x[6] = (float)std::sin(ph); x[7] = (float)std::cos(ph);
      }
    }
  }

  // FlockAviary._computeReward (FlockAviary.py:74-149): velocity alignment +
  // flock speed - spacing penalty - spacing variance, per env.
  R flock_reward(int e) const {
    const int D = P.D;
    const Drone<R>* dr = &drones[e * D];
    const R EPS = R(1e-3);
    R ali = 0;
    std::vector<R> vn(D);
    for (int i = 0; i < D; ++i) vn[i] = norm3(dr[i].vel);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j)
        if (j != i) {
          R dd = (dr[i].vel[0] * dr[j].vel[0] + dr[i].vel[1] * dr[j].vel[1]) + dr[i].vel[2] * dr[j].vel[2];
          ali += (dd / (vn[i] + EPS)) / (vn[j] + EPS);
        }
    ali = D > 1 ? ali / R(D * (D - 1)) : R(0);
    R cv[3] = {0, 0, 0};
    for (int i = 0; i < D; ++i) for (int k = 0; k < 3; ++k) cv[k] += dr[i].vel[k];
    for (int k = 0; k < 3; ++k) cv[k] /= R(D);
    R speed = norm3(cv);
    R spac_rew = 0, var = 0;
    if (D > 1) {
      std::vector<R> sp(D);
      for (int i = 0; i < D; ++i) {
        R m = R(INFINITY);
        for (int j = 0; j < D; ++j)
          if (j != i) {
            R dp[3] = {dr[j].pos[0] - dr[i].pos[0], dr[j].pos[1] - dr[i].pos[1], dr[j].pos[2] - dr[i].pos[2]};
            R dist = norm3(dp);
            m = dist < m ? dist : m;
          }
        sp[i] = m;
      }
      R mean = 0;
      for (int i = 0; i < D; ++i) mean += sp[i];
      mean /= R(D);
      for (int i = 0; i < D; ++i) var += (sp[i] - mean) * (sp[i] - mean);
      var /= R(D);
      if (!(R(1.0) < mean && mean < R(3.0)))
        spac_rew = std::min(std::fabs(mean - R(1.0)), std::fabs(mean - R(3.0)));
    }
    return ((ali + speed) - spac_rew) - var;
  }

  // MeetupAviary._computeReward (MeetupAviary.py:71-93): -2·|p_i - p_{D-1-i}|² per pair.
  R meetup_reward(int e) const {
    const int D = P.D;
    const Drone<R>* dr = &drones[e * D];
    R total = 0;
    for (int i = 0; i < D / 2; ++i) {
      R dp[3] = {dr[i].pos[0] - dr[D - 1 - i].pos[0], dr[i].pos[1] - dr[D - 1 - i].pos[1],
                 dr[i].pos[2] - dr[D - 1 - i].pos[2]};
      R n = norm3(dp);
      total += (R(-1) * (n * n)) * R(2);
    }
    return total;
  }

  // LeaderFollowerAviary._computeReward (LeaderFollowerAviary.py:71-98): the leader
  // hovers at (0,0,0.5); follower i matches the leader's height at its own x, y.
  R leader_reward(int e) const {
    const int D = P.D;
    const Drone<R>* dr = &drones[e * D];
    R dp[3] = {R(0) - dr[0].pos[0], R(0) - dr[0].pos[1], R(0.5) - dr[0].pos[2]};
    R n0 = norm3(dp);
    R total = R(-1) * (n0 * n0);
    for (int i = 1; i < D; ++i) {
      R dz = dr[0].pos[2] - dr[i].pos[2];
      R n = std::sqrt(dz * dz);   // |(x_i, y_i, z_0) - p_i|: only z differs
      total += (-(R(1) / R(D))) * (n * n);
    }
    return total;
  }

  // MultiHoverAviary._computeReward (MH:128-186) / SpiralAviary (SP:150-181).
  R compute_reward(int e) const {
    const int D = P.D;
    if (P.task == QS_TASK_FLOCK) return flock_reward(e);
    if (P.task == QS_TASK_MEETUP) return meetup_reward(e);
    if (P.task == QS_TASK_LEADERFOLLOWER) return leader_reward(e);
    R reward = 0;
    for (int d = 0; d < D; ++d) {
      const Drone<R>& dr = drones[e * D + d];
      if (P.task == QS_TASK_MULTIHOVER) {
        R ex = dr.pos[0] - dr.target[0], ey = dr.pos[1] - dr.target[1];
        R err_xy = std::sqrt(ex * ex + ey * ey);
        R err_z = dr.pos[2] - dr.target[2];
        R vel_z = dr.vel[2];
        R r_xy = R(1.0) / (R(1) + err_xy);
        R r_z = std::exp(R(-7.5) * std::fabs(err_z));
        R r_vel = std::fabs(err_z) < R(0.2) ? R(-1.5) * (vel_z * vel_z) : R(0.0);
        R hover = (err_xy < R(0.03) && std::fabs(err_z) < R(0.03) && std::fabs(vel_z) < R(0.03)) ? R(0.5) : R(0.0);
        reward += ((r_xy + r_z) + r_vel) + hover;
      } else {
        R pr[3], vr[3], ph;
        spiral_ref(e, d, pr, vr, ph);
        R dp[3] = {dr.pos[0] - pr[0], dr.pos[1] - pr[1], dr.pos[2] - pr[2]};
        R dv[3] = {dr.quat[0] - vr[0], dr.quat[1] - vr[1], dr.quat[2] - vr[2]};
        R np_ = norm3(dp), nv = norm3(dv);
        R r_pos = std::exp(R(-4.0) * (np_ * np_));
        R r_vel = std::exp(R(-2.0) * (nv * nv));
        R rx = dr.pos[0] - P.sp_center[0], ry = dr.pos[1] - P.sp_center[1];
        R rn = std::sqrt(rx * rx + ry * ry);
        R r_tan = 0;
        if (rn > R(1e-3)) {
          R radx = rx / rn, rady = ry / rn;
          R tanx = -rady, tany = radx;
          R vx = dr.quat[0], vy = dr.quat[1];
          R vn = std::sqrt(vx * vx + vy * vy);
          if (vn > R(1e-3)) {
            R dot = (vx / vn) * tanx + (vy / vn) * tany;
            r_tan = dot > R(0) ? dot : R(0);
          }
        }
        reward += (R(1.0) * r_pos + R(2.0) * r_vel) + R(1.0) * r_tan;
      }
    }
    return reward / R(D);
  }

  // Flock / LeaderFollower never terminate (FlockAviary.py:153-165,
  // LeaderFollowerAviary.py:102-114); Meetup does when every pair is within
  // 0.1 m (MeetupAviary.py:97-117; vacuously true for one drone).
  // _computeTruncated of the three (FlockAviary.py:169-186, MeetupAviary.py:
  // 121-151, LeaderFollowerAviary.py:118-144): any drone out of the box or
  // tilted (|roll| or |pitch| > 0.4), or the time limit.
  bool marl_terminated(int e) const {
    if (P.task != QS_TASK_MEETUP) return false;
    const int D = P.D;
    const Drone<R>* dr = &drones[e * D];
    for (int i = 0; i < D / 2; ++i) {
      R dp[3] = {dr[i].pos[0] - dr[D - 1 - i].pos[0], dr[i].pos[1] - dr[D - 1 - i].pos[1],
                 dr[i].pos[2] - dr[D - 1 - i].pos[2]};
      if (norm3(dp) > R(0.1)) return false;
    }
    return true;
  }
  bool marl_out_of_bounds(int e) const {
    for (int d = 0; d < P.D; ++d) {
      const Drone<R>& x = drones[e * P.D + d];
      bool tilt = std::fabs(x.rpy[0]) > R(.4) || std::fabs(x.rpy[1]) > R(.4);
      bool out;
      if (P.task == QS_TASK_FLOCK)
        out = std::fabs(x.pos[0]) > R(10.0) || std::fabs(x.pos[1]) > R(10.0) || x.pos[2] > R(10.0);
      else if (P.task == QS_TASK_MEETUP)
        out = std::fabs(x.pos[0]) > R(5.0) || std::fabs(x.pos[1]) > R(5.0) || x.pos[2] > R(3.0) || x.pos[2] < R(0.1);
      else
        out = std::fabs(x.pos[0]) > R(2.0) || std::fabs(x.pos[1]) > R(2.0) || x.pos[2] > R(2.0);
      if (out || tilt) return true;
    }
    return false;
  }

  // _computeTerminated (MH:216-241 / SP:185-191); reasons bits per drone.
  bool compute_terminated(int e, uint8_t* reasons) const {
    if (P.task >= QS_TASK_FLOCK) {
      if (reasons) std::memset(reasons, 0, P.D);
      return marl_terminated(e);
    }
    bool term = false;
    for (int d = 0; d < P.D; ++d) {
      const Drone<R>& dr = drones[e * P.D + d];
      uint8_t b = 0;
      if (P.task == QS_TASK_MULTIHOVER) {
        if (dr.pos[2] < R(0.03)) b |= QS_REASON_CRASH;
        if (std::fabs(dr.rpy[0]) > R(1.2) || std::fabs(dr.rpy[1]) > R(1.2)) b |= QS_REASON_FLIP;
        if (std::fabs(dr.pos[0]) > R(3.0) || std::fabs(dr.pos[1]) > R(3.0)) b |= QS_REASON_OOB;
      } else {
        if (dr.pos[2] < R(0.05) || dr.pos[2] > R(3.0)) b |= QS_REASON_ZRANGE;
      }
      if (b) term = true;
      if (reasons) reasons[d] = b;
    }
    return term;
  }

  // BaseAviary.step (BA:259-383) for env e + worker auto-reset
  // (subproc_vec_env.py:188-206) + VecRecordEpisodeStatistics (rec:144-172).
  void step_env(int e, const float* act_env, float* obs_env, R* rew, uint8_t* term, uint8_t* trunc,
                float* tobs_env, uint8_t* reasons_env, float* act_out_env) {
    const int D = P.D, A = P.A, H = P.H, N_ = N();
    float act_local[64 * 4];
    const float* act = act_env;
    if (!act) {  // synthetic random policy: U(-1,1) from Philox
      const uint32_t genv = (uint32_t)(env_offset + e);
      for (int d = 0; d < D; ++d) {
        U4 c = {{(uint32_t)total_steps[e], genv, 0u, (uint32_t)((STREAM_ACT << 24) | d)}};
        U4 r = philox4x32_10(c, k0, k1);
        for (int k = 0; k < A; ++k) act_local[d * A + k] = (float)(2.0 * u01(r.v[k]) - 1.0);
      }
      act = act_local;
    }
    if (act_out_env) std::memcpy(act_out_env, act, sizeof(float) * D * A);
    // action_buffer.append(action) (BRL:187)
    const int slot = total_steps[e] % H;
    for (int d = 0; d < D; ++d)
      for (int k = 0; k < A; ++k) hist[((size_t)slot * N_ + e * D + d) * A + k] = act[d * A + k];
    // _preprocessAction (BRL:188-239): uses the state at step start
    std::vector<R> rpm(D * 4);
    for (int d = 0; d < D; ++d) preprocess_action(P, drones[e * D + d], act + d * A, &rpm[d * 4]);
    // substeps (BA:343-372)
    std::vector<Snap<R>> snaps(D);
    for (int s = 0; s < P.S; ++s) {
      for (int d = 0; d < D; ++d) {  // _updateAndStoreKinematicInformation (BA:346-347)
        Drone<R>& dr = drones[e * D + d];
        for (int i = 0; i < 3; ++i) { snaps[d].pos[i] = dr.pos[i]; snaps[d].vel[i] = dr.vel[i]; }
        for (int i = 0; i < 4; ++i) snaps[d].quat[i] = dr.quat[i];
        euler_from_quat(dr.quat, dr.rpy);
        for (int i = 0; i < 3; ++i) snaps[d].rpy[i] = dr.rpy[i];
      }
      for (int d = 0; d < D; ++d) {
        if (P.physics == QS_PHYS_PYB) pyb_dynamics(P, drones[e * D + d], &rpm[d * 4], snaps.data(), d);
        else dynamics(P, drones[e * D + d], &rpm[d * 4], snaps.data(), d);
      }
      if (P.physics == QS_PHYS_PYB && D > 1) drone_contacts(&drones[e * D], D);   // Bullet's drone–drone contacts
      for (int d = 0; d < D; ++d)  // last_clipped_action = clipped_action (BA:372)
        for (int m = 0; m < 4; ++m) drones[e * D + d].last_rpm[m] = rpm[d * 4 + m];
    }
    for (int d = 0; d < D; ++d) euler_from_quat(drones[e * D + d].quat, drones[e * D + d].rpy);  // BA:374
    // The obs history's newest entry is this step's action.
    total_steps[e] += 1;
    compute_obs(e, obs_env);
    R r = compute_reward(e);
    uint8_t rs[64];
    bool te = compute_terminated(e, rs);
    bool tr = ((double)step_counter[e] / (double)P.pyb_freq) > (double)P.ep_len_sec;  // MH:267-268
    if (P.task >= QS_TASK_FLOCK) tr = marl_out_of_bounds(e) || tr;
    step_counter[e] += P.S;                                                          // BA:382
    if (rew) rew[e] = r;
    if (term) term[e] = te;
    if (trunc) trunc[e] = tr;
    if (reasons_env) std::memcpy(reasons_env, rs, D);
    ep_return[e] += (double)r;
    ep_len[e] += 1;
    if (te || tr) {
      if (tobs_env) std::memcpy(tobs_env, obs_env, sizeof(float) * D * P.O);
      qs_episode_rec rec;
      rec.ret = ep_return[e]; rec.len = ep_len[e]; rec.env = (int32_t)(env_offset + e);
      rec.seq = total_steps[e];
#pragma omp critical
      log.push_back(rec);
      ep_return[e] = 0; ep_len[e] = 0;
      if (!(P.flags & QS_FLAG_NO_AUTORESET)) {   // worker.step_env (subproc_vec_env.py:195-206)
        episode[e] += 1;
        reset_env(e);
        compute_obs(e, obs_env);
      }
    }
  }
};

template <class R> struct Handle {
  Sim<R> sim;
};

struct OracleHandle {
  int precision;
  void* sim;   // Sim<float>* or Sim<double>*
};

template <class R> int make_params(const qs_spec* s, Params<R>& P) {
  if (s->task < QS_TASK_MULTIHOVER || s->task > QS_TASK_LEADERFOLLOWER) return fail(QS_E_INVALID, "bad task");
  if (s->num_drones < 1 || s->num_drones > 64) return fail(QS_E_INVALID, "num_drones must be 1..64");
  if (s->num_envs < 1) return fail(QS_E_INVALID, "num_envs must be >= 1");
  if (s->physics != QS_PHYS_DYN && s->physics != QS_PHYS_PYB) return fail(QS_E_INVALID, "bad physics");
  if (s->pyb_freq <= 0 || s->ctrl_freq <= 0 || s->pyb_freq % s->ctrl_freq)
    return fail(QS_E_INVALID, "pyb_freq is not divisible by env_freq");   // BA:79-80
  P.task = s->task; P.D = s->num_drones; P.E = s->num_envs; P.act_type = s->act_type; P.aux = s->aux_forces;
  P.physics = s->physics;
  P.flags = s->flags;
  switch (s->act_type) {
    case QS_ACT_RPM: case QS_ACT_VEL: P.A = 4; break;
    case QS_ACT_PID: P.A = 3; break;
    case QS_ACT_ONE_D_RPM: case QS_ACT_ONE_D_PID: P.A = 1; break;
    default: return fail(QS_E_INVALID, "bad act_type");
  }
  P.H = s->ctrl_freq / 2;                        // BRL:66 ACTION_BUFFER_SIZE = ctrl_freq//2
  P.S = s->pyb_freq / s->ctrl_freq;              // BA:81
  P.O = 12 + P.H * P.A + (P.task == QS_TASK_SPIRAL ? 11 : 0);
  P.pyb_freq = s->pyb_freq;
  P.dt = R(1.0 / s->pyb_freq); P.ctrl_dt = R(1.0 / s->ctrl_freq);
  P.ep_len_sec = R(s->episode_len_sec);
  P.KF = R(C.KF); P.KM = R(C.KM); P.M = R(C.M); P.GRAVITY_DYN = R(C.GRAVITY);
  P.cf2p = (s->flags & QS_FLAG_CF2P) != 0;
  const double IX = P.cf2p ? C.IXX_P : C.IXX, IY = P.cf2p ? C.IYY_P : C.IYY, IZ = P.cf2p ? C.IZZ_P : C.IZZ;
  P.Jd[0] = R(IX); P.Jd[1] = R(IY); P.Jd[2] = R(IZ);
  P.Jinv[0] = R(1.0 / IX); P.Jinv[1] = R(1.0 / IY); P.Jinv[2] = R(1.0 / IZ);
  P.L = R(C.L);
  for (int m = 0; m < 4; ++m)
    for (int k = 0; k < 3; ++k) P.MIX[m][k] = R(P.cf2p ? MIXER_P[m][k] : MIXER[m][k]);
  P.L_SQRT2 = R(C.L / std::sqrt(2.0));
  P.HOVER_RPM = R(C.HOVER_RPM);
  P.SPEED_LIMIT = R(0.03 * C.MAX_SPEED_KMH * (1000.0 / 3600.0));    // BRL:94-95
  P.G_PID = R(9.8 * C.M);
  P.DRAG[0] = R(C.DRAG_XY); P.DRAG[1] = R(C.DRAG_XY); P.DRAG[2] = R(C.DRAG_Z);
  P.GND_COEFF = R(C.GND_EFF_COEFF); P.PROP_R = R(C.PROP_RADIUS); P.GND_CLIP = R(C.GND_EFF_H_CLIP);
  P.DW1 = R(C.DW1); P.DW2 = R(C.DW2); P.DW3 = R(C.DW3);
  for (int m = 0; m < 4; ++m)
    for (int k = 0; k < 2; ++k) P.PROP_XY[m][k] = R(P.cf2p ? C.PROP_XY_P[m][k] : C.PROP_XY[m][k]);
  P.sp_R = R(s->spiral_radius); P.sp_OMEGA = R(2 * M_PI / s->spiral_period); P.sp_VZ = R(s->height_rate);
  for (int i = 0; i < 3; ++i) P.sp_center[i] = R(s->target_center[i]);
  P.orig_xyz.resize(P.D * 3);
  for (int d = 0; d < P.D; ++d) {
    double xyz[3];
    if (s->initial_xyzs) { for (int i = 0; i < 3; ++i) xyz[i] = s->initial_xyzs[d * 3 + i]; }
    else if (P.task == QS_TASK_SPIRAL) {   // SP:47-53
      xyz[0] = s->spiral_radius * std::cos(2 * M_PI * d / P.D);
      xyz[1] = s->spiral_radius * std::sin(2 * M_PI * d / P.D);
      xyz[2] = 0.3;
    } else {                                // BA:194-197
      xyz[0] = d * 4 * C.L; xyz[1] = d * 4 * C.L;
      xyz[2] = C.COLL_H / 2 - C.COLL_Z_OFF + .1;
    }
    for (int i = 0; i < 3; ++i) P.orig_xyz[d * 3 + i] = R(xyz[i]);
  }
  if (P.task == QS_TASK_MULTIHOVER && !s->initial_xyzs && P.D >= 6)
    return fail(QS_E_INVALID, "MultiHover reset with the default diagonal layout cannot complete for D >= 6 "
                              "(SURVEY §7 hard-2); pass initial_xyzs");
  return QS_OK;
}

template <class R> Sim<R>* make_sim(const qs_spec* s, int* rc) {
  auto* sim = new Sim<R>();
  *rc = make_params<R>(s, sim->P);
  if (*rc) { delete sim; return nullptr; }
  sim->env_offset = s->env_offset;
  const int N = s->num_envs * s->num_drones;
  sim->drones.assign(N, Drone<R>{});
  std::memset(sim->drones.data(), 0, sizeof(Drone<R>) * N);
  sim->hist.assign((size_t)sim->P.H * N * sim->P.A, 0.f);
  sim->step_counter.assign(s->num_envs, 0);
  sim->episode.assign(s->num_envs, 0);
  sim->total_steps.assign(s->num_envs, 0);
  sim->ep_len.assign(s->num_envs, 0);
  sim->ep_return.assign(s->num_envs, 0.0);
  return sim;
}

template <class R> void sim_reset(Sim<R>* sim, uint64_t seed, float* obs) {
  sim->k0 = (uint32_t)seed; sim->k1 = (uint32_t)(seed >> 32);
  const int E = sim->P.E, N = sim->N();
  std::memset(sim->drones.data(), 0, sizeof(Drone<R>) * N);
  std::fill(sim->hist.begin(), sim->hist.end(), 0.f);
  for (int e = 0; e < E; ++e) {
    sim->episode[e] = 0; sim->total_steps[e] = 0; sim->ep_len[e] = 0; sim->ep_return[e] = 0;
  }
  sim->log.clear();
  sim->reset_error = 0;
  for (int e = 0; e < E; ++e) {
    sim->reset_env(e);
    if (obs) sim->compute_obs(e, obs + (size_t)e * sim->P.D * sim->P.O);
  }
}

template <class R> void sim_step(Sim<R>* sim, const float* act, const qs_step_out* out, int nthreads) {
  const int E = sim->P.E, D = sim->P.D, O = sim->P.O, A = sim->P.A;
  std::vector<float> scratch;
  float* obs = out ? out->obs : nullptr;
  if (!obs) { scratch.resize((size_t)E * D * O); obs = scratch.data(); }
  R* rew = out ? (R*)out->reward : nullptr;
#pragma omp parallel for num_threads(nthreads) schedule(static) if (nthreads > 1)
  for (int e = 0; e < E; ++e) {
    sim->step_env(e, act ? act + (size_t)e * D * A : nullptr, obs + (size_t)e * D * O, rew,
                  out ? out->terminated : nullptr, out ? out->truncated : nullptr,
                  (out && out->terminal_obs) ? out->terminal_obs + (size_t)e * D * O : nullptr,
                  (out && out->reasons) ? out->reasons + (size_t)e * D : nullptr,
                  (out && out->actions_out) ? out->actions_out + (size_t)e * D * A : nullptr);
  }
  // deterministic log order: (seq, env) as the reference's env loop would append
  std::stable_sort(sim->log.begin(), sim->log.end(), [](const qs_episode_rec& a, const qs_episode_rec& b) {
    return a.seq != b.seq ? a.seq < b.seq : a.env < b.env;
  });
}

template <class R> int sim_state_io(Sim<R>* sim, int block, void* buf, int dir) {
  const int N = sim->N(), E = sim->P.E;
  if (block == QS_STATE_AGENT) {
    R* b = (R*)buf;
    for (int a = 0; a < N; ++a) {
      Drone<R>& d = sim->drones[a];
      R* fields[QS_AGENT_FIELDS] = {&d.pos[0], &d.pos[1], &d.pos[2], &d.quat[0], &d.quat[1], &d.quat[2], &d.quat[3],
                                    &d.vel[0], &d.vel[1], &d.vel[2], &d.rpy_rates[0], &d.rpy_rates[1], &d.rpy_rates[2],
                                    &d.last_rpm[0], &d.last_rpm[1], &d.last_rpm[2], &d.last_rpm[3],
                                    &d.int_pos[0], &d.int_pos[1], &d.int_pos[2], &d.int_rpy[0], &d.int_rpy[1], &d.int_rpy[2],
                                    &d.last_rpy[0], &d.last_rpy[1], &d.last_rpy[2], &d.target[0], &d.target[1], &d.target[2]};
      for (int f = 0; f < QS_AGENT_FIELDS; ++f) {
        if (dir) *fields[f] = b[(size_t)f * N + a]; else b[(size_t)f * N + a] = *fields[f];
      }
      if (dir) euler_from_quat(d.quat, d.rpy);
    }
  } else if (block == QS_STATE_ENV) {
    int32_t* b = (int32_t*)buf;
    std::vector<int32_t>* f[QS_ENV_FIELDS] = {&sim->step_counter, &sim->episode, &sim->total_steps, &sim->ep_len};
    for (int k = 0; k < QS_ENV_FIELDS; ++k)
      for (int e = 0; e < E; ++e) { if (dir) (*f[k])[e] = b[(size_t)k * E + e]; else b[(size_t)k * E + e] = (*f[k])[e]; }
  } else if (block == QS_STATE_HISTORY) {
    float* b = (float*)buf;
    if (dir) std::memcpy(sim->hist.data(), b, sizeof(float) * sim->hist.size());
    else std::memcpy(b, sim->hist.data(), sizeof(float) * sim->hist.size());
  } else if (block == QS_STATE_EP_RETURN) {
    double* b = (double*)buf;
    for (int e = 0; e < E; ++e) { if (dir) sim->ep_return[e] = b[e]; else b[e] = sim->ep_return[e]; }
  } else {
    return fail(QS_E_INVALID, "bad state block");
  }
  return QS_OK;
}

}  // namespace

// ===========================================================================
// extern "C" surface (mirrors include/quadswarm.h with host pointers).
// ===========================================================================
extern "C" {

const char* qso_last_error(void) { return g_err.c_str(); }

int qso_create(const qs_spec* spec, OracleHandle** out) {
  if (!spec || !out) return fail(QS_E_INVALID, "null argument");
  int rc = 0;
  auto* h = new OracleHandle();
  h->precision = spec->precision;
  if (spec->precision == 8) h->sim = make_sim<double>(spec, &rc);
  else if (spec->precision == 4) h->sim = make_sim<float>(spec, &rc);
  else { delete h; return fail(QS_E_INVALID, "precision must be 4 or 8"); }
  if (rc) { delete h; return rc; }
  *out = h;
  return QS_OK;
}

int qso_destroy(OracleHandle* h) {
  if (!h) return QS_OK;
  if (h->precision == 8) delete (Sim<double>*)h->sim; else delete (Sim<float>*)h->sim;
  delete h;
  return QS_OK;
}

int qso_get_dims(const OracleHandle* h, qs_dims* d) {
  auto fill = [&](auto* s) {
    d->num_envs = s->P.E; d->num_drones = s->P.D; d->num_agents = s->N(); d->act_dim = s->P.A;
    d->obs_dim = s->P.O; d->hist_len = s->P.H; d->substeps = s->P.S; d->precision = h->precision;
    d->agent_fields = QS_AGENT_FIELDS; d->env_fields = QS_ENV_FIELDS;
  };
  if (h->precision == 8) fill((Sim<double>*)h->sim); else fill((Sim<float>*)h->sim);
  return QS_OK;
}

int qso_reset(OracleHandle* h, uint64_t seed, float* obs) {
  if (h->precision == 8) sim_reset((Sim<double>*)h->sim, seed, obs); else sim_reset((Sim<float>*)h->sim, seed, obs);
  return QS_OK;
}

int qso_step(OracleHandle* h, const float* actions, const qs_step_out* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (h->precision == 8) sim_step((Sim<double>*)h->sim, actions, out, nthreads);
  else sim_step((Sim<float>*)h->sim, actions, out, nthreads);
  return QS_OK;
}

// CPU-baseline driver: `steps` random-policy control steps, obs into a
// scratch buffer, OpenMP over envs (the reference's worker pool stepping its
// envs serially per worker, subproc_vec_env.py:186-215).
int qso_run_random(OracleHandle* h, int steps, int nthreads) {
  qs_dims d;
  qso_get_dims(h, &d);
  std::vector<float> obs((size_t)d.num_agents * d.obs_dim);
  std::vector<double> rew(d.num_envs);
  std::vector<uint8_t> te(d.num_envs), tr(d.num_envs);
  qs_step_out out{};
  out.obs = obs.data(); out.reward = rew.data(); out.terminated = te.data(); out.truncated = tr.data();
  std::vector<float> rewf(d.num_envs);
  if (h->precision == 4) out.reward = rewf.data();
  for (int s = 0; s < steps; ++s) qso_step(h, nullptr, &out, nthreads);
  return QS_OK;
}

// env.reset() on masked envs (MultiHoverAviary.reset, MH:75-110): PID state
// and action history persist.
int qso_reset_envs(OracleHandle* h, const uint8_t* mask, float* obs) {
  auto go = [&](auto* s) {
    for (int e = 0; e < s->P.E; ++e) {
      if (mask && !mask[e]) continue;
      s->episode[e] += 1;
      s->reset_env(e);
      if (obs) s->compute_obs(e, obs + (size_t)e * s->P.D * s->P.O);
    }
  };
  if (h->precision == 8) go((Sim<double>*)h->sim); else go((Sim<float>*)h->sim);
  return QS_OK;
}

int qso_state_io(OracleHandle* h, int block, void* buf, int dir) {
  if (h->precision == 8) return sim_state_io((Sim<double>*)h->sim, block, buf, dir);
  return sim_state_io((Sim<float>*)h->sim, block, buf, dir);
}

int64_t qso_episode_log(OracleHandle* h, qs_episode_rec* dst, int64_t cap) {
  auto take = [&](auto* s) -> int64_t {
    int64_t n = (int64_t)s->log.size(), k = std::min(n, cap);
    for (int64_t i = 0; i < k; ++i) dst[i] = s->log[n - k + i];
    return n;
  };
  if (h->precision == 8) return take((Sim<double>*)h->sim);
  return take((Sim<float>*)h->sim);
}

int qso_reset_error(OracleHandle* h) {
  return h->precision == 8 ? ((Sim<double>*)h->sim)->reset_error : ((Sim<float>*)h->sim)->reset_error;
}

// ---- unit-level entry points for the KATs (fp64 only) ---------------------
void qso_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  U4 c = {{ctr[0], ctr[1], ctr[2], ctr[3]}};
  U4 r = philox4x32_10(c, key[0], key[1]);
  for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}
void qso_quat_to_matrix(const double q[4], double m[9]) { quat_to_matrix<double>(q, (double(*)[3])m); }
void qso_euler_from_quat(const double q[4], double rpy[3]) { euler_from_quat<double>(q, rpy); }
void qso_integrate_q(double q[4], const double w[3], double dt) { integrate_q<double>(q, w, dt); }
void qso_constants(double out[8]) {
  out[0] = C.GRAVITY; out[1] = C.HOVER_RPM; out[2] = C.MAX_RPM; out[3] = C.MAX_THRUST;
  out[4] = C.GND_EFF_H_CLIP; out[5] = 0.03 * C.MAX_SPEED_KMH * (1000.0 / 3600.0);
  out[6] = C.L / std::sqrt(2.0); out[7] = C.COLL_H / 2 - C.COLL_Z_OFF + .1;
}
// One DSLPIDControl.computeControl call on a fresh or given controller state
// (pid_state: int_pos[3], int_rpy[3], last_rpy[3], updated in place).
void qso_dsl_pid(double pid_state[9], const double cur_pos[3], const double cur_quat[4], const double cur_vel[3],
                 const double target_pos[3], const double target_rpy[3], const double target_vel[3],
                 double ctrl_dt, double rpm[4]) {
  Params<double> P;
  qs_spec s{};
  s.task = QS_TASK_MULTIHOVER; s.num_envs = 1; s.num_drones = 1; s.act_type = QS_ACT_ONE_D_PID;
  s.physics = QS_PHYS_DYN; s.pyb_freq = 240; s.ctrl_freq = 30; s.precision = 8; s.episode_len_sec = 8;
  make_params<double>(&s, P);
  P.ctrl_dt = ctrl_dt;
  Drone<double> d{};
  for (int i = 0; i < 3; ++i) { d.int_pos[i] = pid_state[i]; d.int_rpy[i] = pid_state[3 + i]; d.last_rpy[i] = pid_state[6 + i]; }
  dsl_pid_compute_control(P, d, cur_pos, cur_quat, cur_vel, target_pos, target_rpy, target_vel, rpm);
  for (int i = 0; i < 3; ++i) { pid_state[i] = d.int_pos[i]; pid_state[3 + i] = d.int_rpy[i]; pid_state[6 + i] = d.last_rpy[i]; }
}

// compute_returns_and_advantages → _compute_single_agent_returns
// (mappo/buffer.py:428-614) for data laid out [T][N] (N = E*D agents),
// terminal_vals [T][N], last_val [N].  The reference's arrays are float32 and
// its pinned numpy 2.2.6 (environment.yml:63) applies NEP 50: a float32 scalar
// combined with a Python float (γ, λ) stays float32, the Python float rounded
// to float32 first.  So each line is a float32 operation in source order:
//   rew_adjusted = rews[i] + γ·tv[i]                    (buffer.py:593)
//   ret = rew_adjusted + (γ·masks[i])·ret                 (:602, ret starts as last_val)
//   td = (rew_adjusted + (γ·masks[i])·v_ext[i+1]) − v[i]  (:608)
//   adv = ((adv·λ)·γ)·masks[i] + td                       (:609; adv = ret − v[i] without GAE)
// stored into float64 result arrays (exact).  -ffp-contract=off: no FMA.
void qso_gae(int T, int64_t N, const float* rews, const float* vals, const float* masks, const float* terminal_vals,
             const float* last_val, double gamma, int use_gae, double lam, double* rets, double* advs) {
  const float g = (float)gamma, lm = (float)lam;
  for (int64_t n = 0; n < N; ++n) {
    float ret = last_val[n], adv = 0.0f;
    for (int i = T - 1; i >= 0; --i) {
      const size_t k = (size_t)i * N + n;
      const float rew_adj = rews[k] + g * terminal_vals[k];
      ret = rew_adj + (g * masks[k]) * ret;
      if (!use_gae) adv = ret - vals[k];
      else {
        const float vnext = (i + 1 < T) ? vals[k + N] : last_val[n];
        const float td = (rew_adj + (g * masks[k]) * vnext) - vals[k];
        adv = ((adv * lm) * g) * masks[k] + td;
      }
      rets[k] = (double)ret; advs[k] = (double)adv;
    }
  }
}

}  // extern "C"
