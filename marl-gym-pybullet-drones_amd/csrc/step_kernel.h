// step_kernel.h — MI355X (gfx950) batched quadrotor-swarm control step (device code).
//
// One launch advances every (env, drone) of a shard by one control step:
// action → RPM (incl. the DSL PID), PYB_STEPS_PER_CTRL rigid-body substeps,
// readback, MultiHover/Spiral obs + reward + termination, and the vec-env
// auto-reset.  It replaces BaseAviary.step (BaseAviary.py:259-383) driven by
// SubprocVecEnv workers (subproc_vec_env.py:188-206); see include/quadswarm.h
// for the per-entry-point reference mapping.
//
// Layout (DESIGN.md §HBM layout): per-agent state is structure-of-arrays
// [field][N] (N = E*D, agent a = env*D + drone) so lane i of a wavefront
// touches element i of every field — every state load/store is a fully
// coalesced 256 B (fp32) wave access.  A workgroup owns whole envs
// (EPB = floor(64/D) envs × D drones, one wavefront), so the per-env reductions (reward
// mean, any-terminated), the O(D²) downwash neighbour scan and the reset
// rejection search all run through LDS with no inter-workgroup traffic.
// The path is elementwise ODE + a small PID: no contraction, so no MFMA; the
// bound is HBM bandwidth.

#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <string>
#include <vector>
#include <new>

#include "quadswarm.h"

#ifdef QS_DEV_BUILD
#include "step_kernel_dev.h"   // timing probes (dev builds only)
#else
namespace qs_dev {
constexpr bool kNoCompute = false, kNoResetDraw = false;
}
#define QS_STAMP(k) do { } while (0)
#define QS_STAMP_SINK(x) do { } while (0)
#define QS_RS_BEGIN() do { } while (0)
#define QS_RS_JOIN(futile) do { } while (0)
#define QS_RS_CHUNK(found) do { } while (0)
#define QS_RS_PICK() do { } while (0)
#define QS_RS_END(n) do { } while (0)
#endif

namespace qs {

// One wavefront per workgroup: a wave owns floor(64/D) whole envs, so every
// per-env reduction, neighbour scan and reset search stays inside one wave and
// the workgroup barriers below cost nothing (no inter-wave coupling).
constexpr int kBlock = 64;
// Per-env record, kEnvRec int32 words: the QS_ENV_FIELDS counters (words 0-3,
// QS_E_* order), the episode return as f64 (words 4-5), the number of episodes
// this env has logged (word 6, kEnvLogWord), word 7 spare (zero; the
// precomputed resets live in their own array, Params::reset_pre, which the
// step kernel only reads, so no search need race the record's store).  32 B per env
// make a wave's envs (D = 8) one 256-B span, loaded and stored whole: written
// field by field, [field][E] arrays took partial-line writes.
constexpr int kEnvRec = 8;
constexpr int kEnvRetWord = 4;
constexpr int kEnvLogWord = 6;
constexpr int kEnvPreWord = 7;
constexpr uint32_t kMaxResetTries = 1u << 24;
constexpr int kResetNoneDev = 0x7f7f7f7f;   // deferred reset search: "no accepted try yet"
// reset_pre[e]: the precomputed search for episode ep of env e (written only by
// reset_precompute in reset_search_kernel).  Bits 24-30 hold ep & 0x7f (the tag: a word whose tag
// is not the episode being entered is void, so nothing need clear it when the
// env resets); bit 31 set: bits 0-23 are ep's first accepted try; clear: bits
// 0-23 count the 256-try chunks (tries 0 .. 256·c − 1) already rejected.
constexpr uint32_t kPreFound = 0x80000000u;
__device__ __forceinline__ bool pre_tag_is(int32_t w, uint32_t ep) { return (((uint32_t)w >> 24) & 0x7fu) == (ep & 0x7fu); }
// deferred reset search queue (reset_search_kernel): 128-B lines of int32
// words in `reset_queue` — line 0 {count, envs written}, line 1 + slot {claim
// word (u64: chunks claimed | best try << 32), env id, gang}
constexpr int kRqLine = 32, kRqWin = 1, kRqEnv = 2, kRqGang = 3;
constexpr int kRqDone = 1 << 24;   // gang value of a slot whose env has been written
enum { STREAM_ACT = 1, STREAM_RESET = 2 };
enum { MODE_STEP = 0, MODE_RESET_ALL = 1, MODE_RESET_MASK = 2 };

// ------------------------------------------------------- CF2X constants
// cf2x.urdf:5, 11-12, 34 and BaseAviary.py:117-128, as compile-time literals so
// they fold into the instruction stream (no kernel-argument SGPRs, no spills).
// The three square-root-derived values are the correctly rounded doubles of
// their defining expressions; qs_create re-derives them with std::sqrt and
// refuses to run if any differs (check_consts below).
namespace cf2x {
constexpr double G = 9.8, M = 0.027, L = 0.0397, KF = 3.16e-10, KM = 7.94e-12;
constexpr double IXX = 1.4e-5, IYY = 1.4e-5, IZZ = 2.17e-5;
constexpr double GRAVITY = G * M;                       // BaseAviary.py:117
constexpr double L_SQRT2 = 0.028072139213105935;        // L / sqrt(2)      (BA:849-850)
constexpr double HOVER_RPM = 14468.429183500699;        // sqrt(G M / 4 KF) (BA:118)
constexpr double GND_CLIP = 0.037763713492095015;       // BaseAviary.py:125-126
constexpr double SPEED_LIMIT = 0.03 * 30.0 * (1000.0 / 3600.0);   // BaseRLAviary.py:88
constexpr double G_PID = 9.8 * M;                       // DSLPIDControl.py:43 (GRAVITY)
constexpr double DRAG_XY = 9.1785e-7, DRAG_Z = 10.311e-7;
constexpr double GND_COEFF = 11.36859, PROP_R = 2.31348e-2;
constexpr double DW1 = 2267.18, DW2 = 0.16, DW3 = -0.11;
}  // namespace cf2x
// Prop-link COM offsets (assets/cf2x.urdf:42-79), Bullet's default multibody
// damping (linear = angular = 0.04) and the collision cylinder (cf2x.urdf:32-35).
constexpr double kPropX[4] = {0.028, -0.028, -0.028, 0.028}, kPropY[4] = {-0.028, -0.028, 0.028, 0.028};
constexpr double kPybDamping = 0.04, kCylR = 0.06, kCylHalfLen = 0.0125;
// The drone model (QS_FLAG_CF2P selects DroneModel.CF2P, the + configuration):
// cf2p.urdf differs from cf2x.urdf only in the inertia (cf2p.urdf:12) and the
// prop links, on the body axes at L (cf2p.urdf:42-79); the torques
// (BaseAviary.py:849-853) and the DSL PID mixer (DSLPIDControl.py:48-60) follow.
template <bool CF2P> struct Model {
  static constexpr double IXX = cf2x::IXX, IYY = cf2x::IYY, IZZ = cf2x::IZZ;
  static constexpr double PX[4] = {kPropX[0], kPropX[1], kPropX[2], kPropX[3]};
  static constexpr double PY[4] = {kPropY[0], kPropY[1], kPropY[2], kPropY[3]};
  static constexpr double MIX[4][3] = {{-.5, -.5, -1}, {-.5, .5, 1}, {.5, .5, -1}, {.5, -.5, 1}};
};
template <> struct Model<true> {
  static constexpr double IXX = 2.3951e-5, IYY = 2.3951e-5, IZZ = 3.2347e-5;
  static constexpr double PX[4] = {cf2x::L, 0, -cf2x::L, 0}, PY[4] = {0, cf2x::L, 0, -cf2x::L};
  static constexpr double MIX[4][3] = {{0, -1, -1}, {+1, 0, 1}, {0, 1, -1}, {-1, 0, 1}};
};

// Compile-time shape of an action type (BaseRLAviary.py:262-277).
template <int ACT> struct Act {
  static constexpr int A = (ACT == QS_ACT_RPM || ACT == QS_ACT_VEL) ? 4 : (ACT == QS_ACT_PID ? 3 : 1);
  static constexpr bool pid = ACT == QS_ACT_PID || ACT == QS_ACT_VEL || ACT == QS_ACT_ONE_D_PID;
};

// ---------------------------------------------------------------- math utils
template <class T> struct M;
template <> struct M<float> {
  __device__ static float sqrt_(float x) { return sqrtf(x); }
  // hardware v_sin/v_cos (argument in revolutions): ~1e-6 absolute over the
  // angles used here (yaw in [-π, π], Spiral phases < 20 rad), no library range
  // reduction in the instruction stream
  __device__ static float sin_(float x) { return __sinf(x); }
  __device__ static float cos_(float x) { return __cosf(x); }
  // atan2 on the fp32 hot path: reduction to [0,1] with one hardware reciprocal
  // and a degree-7 polynomial in a² (fitted here; |error| ≤ 2e-7 rad, ~3 ulp),
  // about a third of the instructions of the library atan2f.
  __device__ static float atan2_(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
    const float z = a * a;
    float p = __builtin_fmaf(z, -0.004785229451954365f, 0.02457403391599655f);
    p = __builtin_fmaf(z, p, -0.059928297996520996f);
    p = __builtin_fmaf(z, p, 0.0994439497590065f);
    p = __builtin_fmaf(z, p, -0.14030005037784576f);
    p = __builtin_fmaf(z, p, 0.1997147500514984f);
    p = __builtin_fmaf(z, p, -0.3333210051059723f);
    p = __builtin_fmaf(z, p, 0.9999999403953552f);
    float r = a * p;
    if (ay > ax) r = 1.57079637f - r;
    if (x < 0.f) r = 3.14159274f - r;
    return copysignf(r, y);
  }
  __device__ static float asin_(float x) { return asinf(x); }
  __device__ static float exp_(float x) { return expf(x); }
  __device__ static float abs_(float x) { return fabsf(x); }
  __device__ static float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
  __device__ static float mul_rn(float a, float b) { return __fmul_rn(a, b); }
  __device__ static float add_rn(float a, float b) { return __fadd_rn(a, b); }
  __device__ static float sub_rn(float a, float b) { return __fsub_rn(a, b); }
  // fp32 hot path: hardware reciprocal / reciprocal square root (≤1 ulp) in place
  // of the scaled division sequences; constant divisors become multiplies.
  __device__ static float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
  __device__ static float rsqrt(float x) { return __builtin_amdgcn_rsqf(x); }
  __device__ static float divc(float x, double c) { return x * float(1.0 / c); }
};
template <> struct M<double> {
  __device__ static double sqrt_(double x) { return sqrt(x); }
  __device__ static double sin_(double x) { return sin(x); }
  __device__ static double cos_(double x) { return cos(x); }
  __device__ static double atan2_(double y, double x) { return atan2(y, x); }
  __device__ static double asin_(double x) { return asin(x); }
  __device__ static double exp_(double x) { return exp(x); }
  __device__ static double abs_(double x) { return fabs(x); }
  __device__ static double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
  __device__ static double mul_rn(double a, double b) { return __dmul_rn(a, b); }
  __device__ static double add_rn(double a, double b) { return __dadd_rn(a, b); }
  __device__ static double sub_rn(double a, double b) { return __dsub_rn(a, b); }
  // fp64 keeps the reference's exact divisions (the tight fp64 parity gate).
  __device__ static double rcp(double x) { return 1.0 / x; }
  __device__ static double rsqrt(double x) { return 1.0 / sqrt(x); }
  __device__ static double divc(double x, double c) { return x / c; }
};

template <class T> __device__ __forceinline__ T clampv(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
// fp32: one v_med3_f32 (same result as the compare/select form for every non-NaN x, lo <= hi)
template <> __device__ __forceinline__ float clampv<float>(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }

// cos θ and sin θ / |ω| for the exp-map update (BaseAviary.py:889-891), with
// θ = |ω|·dt/2, from u = θ² = |ω|²·(dt/2)² — no square root and no division
// in flight (θ < 0.25, i.e. |ω| < 120 rad/s at 240 Hz).  Taylor series in u,
// truncated where the next term is < 1e-10 of an fp32 ulp (fp32) or < 1e-4 of
// an fp64 ulp (fp64).  Larger θ falls back to the library sin/cos.
template <class T> __device__ __forceinline__ void expmap_coeffs(T wn2, T hdt, T hdt2, T& c, T& k) {
  using F = M<T>;
  const T u = wn2 * hdt2;
  if (u < T(0.0625)) {
    T s, cc;
    if constexpr (sizeof(T) == 4) {
      s = F::fma_(u, F::fma_(u, F::fma_(u, T(-1.0 / 5040), T(1.0 / 120)), T(-1.0 / 6)), T(1));
      cc = F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, T(1.0 / 40320), T(-1.0 / 720)), T(1.0 / 24)), T(-0.5)), T(1));
    } else {
      s = F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, T(1.0 / 6227020800.0), T(-1.0 / 39916800.0)),
                                                           T(1.0 / 362880)), T(-1.0 / 5040)), T(1.0 / 120)), T(-1.0 / 6)), T(1));
      cc = F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, F::fma_(u, T(1.0 / 479001600.0), T(-1.0 / 3628800.0)),
                                                            T(1.0 / 40320)), T(-1.0 / 720)), T(1.0 / 24)), T(-0.5)), T(1));
    }
    c = cc;
    k = hdt * s;             // sin θ / |ω| = (dt/2) · sinc θ
  } else {
    const T wn = F::sqrt_(wn2);
    const T th = wn * hdt;
    c = F::cos_(th);
    k = F::sin_(th) / wn;
  }
}

// Philox4x32-10 (Random123).  Same stream definition as the oracle.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* g_ptr_t;

struct U4 { uint32_t x, y, z, w; };
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    // one 32x32->64 product per multiplier (a single v_mad_u64_u32, where separate
    // lo/hi halves are two quarter-rate v_mul_lo/v_mul_hi)
#ifndef QS_PHILOX_MAD64
    uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
#else
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32), lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
#endif
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}
// 24-bit uniform in [0,1), exact in float and double.
template <class T> __device__ __forceinline__ T u01(uint32_t x) { return T(x >> 8) * T(1.0 / 16777216.0); }

// -------------------------------------------------------------- parameters
template <class T> struct Params {
  // sizes
  int E, D, N, O, H, S, EPB;
  int mode;
  int task;               // qs_task (the MARL family kernel switches on it at run time)
  uint32_t aux, flags;
  int pyb_freq;
  double ep_len_sec;
  uint32_t k0, k1;
  long long env_offset;
  T dt, hdt, hdt2, ctrl_dt, ctrl_hz;   // PYB_TIMESTEP, dt/2, (dt/2)², CTRL_TIMESTEP, CTRL_FREQ
  T sp_R, sp_OMEGA, sp_VZ, sp_cx, sp_cy, sp_cz;
  // device buffers
  T* st;                  // [QS_AGENT_FIELDS][N]
  int32_t* env;           // [E][kEnvRec] per-env records (see kEnvRec)
  float* hist;            // [H][N][A]
  const T* orig_xyz;      // [D][3]
  qs_episode_rec* log;    // [E][log_per_env] per-env rings of completed episodes
  int log_per_env;
  int* err;               // [1] reset search overflow flag
  int* reset_queue;       // deferred MultiHover reset searches (reset_search_kernel's records); or NULL
  int reject_free;        // MultiHover layout whose reset draws can never be rejected: try 0 is the reset
  int32_t* reset_pre;     // [E] each env's precomputed next-episode reset search (kPre* encoding); or NULL
  int stage_rows;         // obs rows staged in LDS per pass
  unsigned long long* stamps;   // dev builds only (QS_STAMPS_BUILD)
  // per-step I/O
  const uint8_t* reset_mask;   // MODE_RESET_MASK: [E] or NULL (= all)
  const float* act_in;
  float* obs;
  T* rew;
  uint8_t* term;
  uint8_t* trunc;
  float* tobs;
  uint8_t* reasons;
  float* act_out;
};

// ---------------------------------------------------- conversions (external)
// pybullet getMatrixFromQuaternion = btMatrix3x3::setRotation (s = 2/|q|²).
template <class T> __device__ __forceinline__ void quat_to_rot(const T q[4], T R[9]) {
  T x = q[0], y = q[1], z = q[2], w = q[3];
  T d = x * x + y * y + z * z + w * w;
  T s = T(2) * M<T>::rcp(d);
  T xs = x * s, ys = y * s, zs = z * s;
  T wx = w * xs, wy = w * ys, wz = w * zs;
  T xx = x * xs, xy = x * ys, xz = x * zs;
  T yy = y * ys, yz = y * zs, zz = z * zs;
  R[0] = T(1) - (yy + zz); R[1] = xy - wz; R[2] = xz + wy;
  R[3] = xy + wz; R[4] = T(1) - (xx + zz); R[5] = yz - wx;
  R[6] = xz - wy; R[7] = yz + wx; R[8] = T(1) - (xx + yy);
}
// Third column of the same matrix (the body z axis): all the force model of a
// DYN substep needs; s = 2/|q|² supplied by the caller.
template <class T> __device__ __forceinline__ void quat_to_zaxis_s(const T q[4], T s, T& r2, T& r5, T& r8) {
  T x = q[0], y = q[1], z = q[2], w = q[3];
  T xs = x * s, ys = y * s, zs = z * s;
  r2 = x * zs + w * ys;
  r5 = y * zs - w * xs;
  r8 = T(1) - (x * xs + y * ys);
}
// pybullet getEulerFromQuaternion.
template <class T> __device__ __forceinline__ void quat_to_rpy(const T q[4], T rpy[3]) {
  using F = M<T>;
  T sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
  T sarg = T(-2) * (q[0] * q[2] - q[3] * q[1]);
  if (sarg <= T(-0.99999)) {
    rpy[0] = 0; rpy[1] = T(-0.5 * M_PI); rpy[2] = T(2) * F::atan2_(q[0], -q[1]);
  } else if (sarg >= T(0.99999)) {
    rpy[0] = 0; rpy[1] = T(0.5 * M_PI); rpy[2] = T(2) * F::atan2_(-q[0], q[1]);
  } else {
    rpy[0] = F::atan2_(T(2) * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
    rpy[1] = F::asin_(sarg);
    rpy[2] = F::atan2_(T(2) * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
  }
}

// ------------------------------------------------------------ DSL PID
// DSLPIDControl.computeControl (DSLPIDControl.py:82-259), one drone.
// pid: int_pos[3], int_rpy[3], last_rpy[3] (updated in place); rpy = the
// current attitude (computed once by the caller, DSLPIDControl.py:240).
template <class T, bool CF2P = false>
__device__ __forceinline__ void dsl_pid(T ctrl_dt, T ctrl_hz, T pid[9], const T pos[3], const T q[4], const T vel[3],
                                        const T rpy[3], const T tpos[3], T tyaw, const T tvel[3], T rpm[4]) {
  if constexpr (qs_dev::kNoCompute) {
    rpm[0] = rpm[1] = rpm[2] = rpm[3] = T(cf2x::HOVER_RPM) + T(1e-3) * pos[2];
    return;
  }
  using F = M<T>;
  const T dt = ctrl_dt;
  T R[9];
  quat_to_rot(q, R);
  T pe[3], ve[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) { pe[i] = tpos[i] - pos[i]; ve[i] = tvel[i] - vel[i]; }
#pragma unroll
  for (int i = 0; i < 3; ++i) pid[i] = clampv(pid[i] + pe[i] * dt, T(-2), T(2));
  pid[2] = clampv(pid[2], T(-0.15), T(0.15));
  const T PF[3] = {T(.4), T(.4), T(1.25)}, IF[3] = {T(.05), T(.05), T(.05)}, DF[3] = {T(.2), T(.2), T(.5)};
  T tt[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) tt[i] = PF[i] * pe[i] + IF[i] * pid[i] + DF[i] * ve[i];
  tt[2] += T(cf2x::G_PID);
  T st = tt[0] * R[2] + tt[1] * R[5] + tt[2] * R[8];
  st = st > T(0) ? st : T(0);
  T thrust = F::divc(F::sqrt_(F::divc(st, 4 * cf2x::KF)) - T(4070.3), 0.2685);
  T inv = F::rsqrt(tt[0] * tt[0] + tt[1] * tt[1] + tt[2] * tt[2]);
  T z[3] = {tt[0] * inv, tt[1] * inv, tt[2] * inv};
  T xc0 = F::cos_(tyaw), xc1 = F::sin_(tyaw);
  // y = (z × x_c)/|z × x_c| with x_c = (xc0, xc1, 0)
  T y[3] = {-z[2] * xc1, z[2] * xc0, z[0] * xc1 - z[1] * xc0};
  T yi = F::rsqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
  y[0] *= yi; y[1] *= yi; y[2] *= yi;
  T x[3] = {y[1] * z[2] - y[2] * z[1], y[2] * z[0] - y[0] * z[2], y[0] * z[1] - y[1] * z[0]};
  // target_rotation columns x,y,z (scipy XYZ round trip = identity on SO(3)).
  // rot_e = vee(Rt^T R - R^T Rt)
  const T* Rt0 = x; const T* Rt1 = y; const T* Rt2 = z;   // columns
  auto Rt = [&](int i, int j) -> T { return j == 0 ? Rt0[i] : (j == 1 ? Rt1[i] : Rt2[i]); };
  auto E = [&](int i, int j) -> T {
    T a = Rt(0, i) * R[0 * 3 + j] + Rt(1, i) * R[1 * 3 + j] + Rt(2, i) * R[2 * 3 + j];
    T b = R[0 * 3 + i] * Rt(0, j) + R[1 * 3 + i] * Rt(1, j) + R[2 * 3 + i] * Rt(2, j);
    return a - b;
  };
  T rot_e[3] = {E(2, 1), E(0, 2), E(1, 0)};
  T rate_e[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T drpy = rpy[i] - pid[6 + i];
    if constexpr (sizeof(T) == 4) rate_e[i] = -(drpy * ctrl_hz);
    else rate_e[i] = T(0) - drpy / dt;
    pid[6 + i] = rpy[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) pid[3 + i] = clampv(pid[3 + i] - rot_e[i] * dt, T(-1500), T(1500));
  pid[3] = clampv(pid[3], T(-1), T(1));
  pid[4] = clampv(pid[4], T(-1), T(1));
  const T PT[3] = {T(70000.), T(70000.), T(60000.)}, IT[3] = {T(0), T(0), T(500.)}, DT[3] = {T(20000.), T(20000.), T(12000.)};
  T tq[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) tq[i] = clampv(-PT[i] * rot_e[i] + DT[i] * rate_e[i] + IT[i] * pid[3 + i], T(-3200), T(3200));
  // the mixer (DSLPIDControl.py:48-60)
  using MD = Model<CF2P>;
  const T MX[4][3] = {{T(MD::MIX[0][0]), T(MD::MIX[0][1]), T(MD::MIX[0][2])},
                      {T(MD::MIX[1][0]), T(MD::MIX[1][1]), T(MD::MIX[1][2])},
                      {T(MD::MIX[2][0]), T(MD::MIX[2][1]), T(MD::MIX[2][2])},
                      {T(MD::MIX[3][0]), T(MD::MIX[3][1]), T(MD::MIX[3][2])}};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    T pwm = thrust + (MX[m][0] * tq[0] + MX[m][1] * tq[1] + MX[m][2] * tq[2]);
    pwm = clampv(pwm, T(20000), T(65535));
    rpm[m] = T(0.2685) * pwm + T(4070.3);
  }
}

// Drone–drone contact of the PYB mode, the oracle's drone_contacts
// (oracle/qs_oracle.cpp): pairs i < j of one env in drone
// order, inelastic and frictionless push-out between the collision cylinders.
// p / v / ez: the env's positions, velocities and tilted half-heights in LDS.
template <class T>
__device__ void contact_pairs(T (*p)[3], T (*v)[3], const T* ez, int D) {
  using F = M<T>;
  const T r2 = T(2 * kCylR);
  for (int i = 0; i < D; ++i)
    for (int j = i + 1; j < D; ++j) {
      const T dx = p[j][0] - p[i][0], dy = p[j][1] - p[i][1], dz = p[j][2] - p[i][2];
      const T d2 = dx * dx + dy * dy;
      if (!(d2 < r2 * r2)) continue;
      const T pz = (ez[i] + ez[j]) - F::abs_(dz);
      if (!(pz > T(0))) continue;
      const T dxy = F::sqrt_(d2);
      const T pxy = r2 - dxy;
      if (pz < pxy) {   // vertical: j above i when dz >= 0
        const T sg = dz >= T(0) ? T(1) : T(-1);
        const T half = T(0.5) * pz;
        p[i][2] = p[i][2] - sg * half;
        p[j][2] = p[j][2] + sg * half;
        const T rel = (v[j][2] - v[i][2]) * sg;
        if (rel < T(0)) {
          const T m = T(0.5) * (v[i][2] + v[j][2]);
          v[i][2] = m;
          v[j][2] = m;
        }
      } else {          // horizontal, along the centre line
        T nx = T(1), ny = T(0);
        if (dxy > T(0)) { nx = dx / dxy; ny = dy / dxy; }
        const T half = T(0.5) * pxy;
        p[i][0] = p[i][0] - nx * half; p[i][1] = p[i][1] - ny * half;
        p[j][0] = p[j][0] + nx * half; p[j][1] = p[j][1] + ny * half;
        const T rel = (v[j][0] - v[i][0]) * nx + (v[j][1] - v[i][1]) * ny;
        if (rel < T(0)) {
          const T hr = T(0.5) * rel;
          v[i][0] = v[i][0] + hr * nx; v[i][1] = v[i][1] + hr * ny;
          v[j][0] = v[j][0] - hr * nx; v[j][1] = v[j][1] - hr * ny;
        }
      }
    }
}

__device__ __forceinline__ float wave_min(float x) {
  for (int o = 32; o > 0; o >>= 1) x = fminf(x, __shfl_xor(x, o, 64));
  return x;
}

// --------------------------------------------------- LDS workspace layout
template <class T> struct Shared {
  union {
    alignas(16) T cand[kBlock][3];  // reset candidates / MARL-task positions
    alignas(16) float4 dw4[kBlock]; // fp32 downwash snapshot during the substeps (one float4 per drone)
  };
  T velw[kBlock][3];        // MARL-task velocities (Flock alignment and speed)
  T rew[kBlock];            // per-drone reward terms
  uint8_t bits[kBlock];     // per-drone termination reason bits
  int reject[kBlock];       // per-group rejection flag (reset search)
  int done[kBlock];         // per-env done flag (EPB <= kBlock)
  int need[kBlock];         // per-env: still searching
  uint32_t win_try[kBlock]; // per-env winning try index
  int win_group;
  int any;
  uint32_t ep_bcast;
  int qcount, qbase;        // deferred reset search: this workgroup's queue slots
  int32_t rec[kBlock * kEnvRec];   // per-env records on their way out
};

// Drone d's position for reset try `try_idx` (MultiHoverAviary.reset, MH:83-95):
// the original layout plus U(-0.25, 0.25)³ noise, z clipped to [0.1, 1].
template <class T>
__device__ __forceinline__ void reset_candidate(const Params<T>& P, const T orig[3], int d, uint32_t try_idx,
                                                uint32_t genv, uint32_t episode, T& px, T& py, T& pz) {
  using F = M<T>;
  U4 r = philox(U4{try_idx, genv, episode, (uint32_t)((STREAM_RESET << 24) | d)}, P.k0, P.k1);
  T n0 = T(0.5) * u01<T>(r.x) - T(0.25), n1 = T(0.5) * u01<T>(r.y) - T(0.25), n2 = T(0.5) * u01<T>(r.z) - T(0.25);
  px = F::add_rn(orig[0], n0);
  py = F::add_rn(orig[1], n1);
  pz = clampv(F::add_rn(orig[2], n2), T(0.1), T(1.0));
}
// MH:96-101 pair test: closer than 0.5 m (the same _rn operation order as the oracle).
template <class T> __device__ __forceinline__ bool too_close(T ax, T ay, T az, T bx, T by, T bz) {
  using F = M<T>;
  T dx = F::sub_rn(ax, bx), dy = F::sub_rn(ay, by), dz = F::sub_rn(az, bz);
  T ss = F::add_rn(F::add_rn(F::mul_rn(dx, dx), F::mul_rn(dy, dy)), F::mul_rn(dz, dz));
  return F::sqrt_(ss) < T(0.5);
}

// Reset search (MultiHoverAviary.reset rejection loop, MH:83-102), group g
// (= threads g*D .. g*D+D-1) evaluates `try_idx` for its env.
// Writes cand positions for its group and flags rejection in s.reject[g].
// The candidate is also returned in c[3] (phase 1 keeps try 0's draw: the
// usual winner, whose position is then not drawn a second time).
template <class T>
__device__ void eval_candidate(const Params<T>& P, Shared<T>& s, const T orig[3], int g, int d, uint32_t try_idx,
                               uint32_t genv, uint32_t episode, bool active, T* c = nullptr) {
  const int tid = threadIdx.x;
  if (active) {
    T px, py, pz;
    reset_candidate(P, orig, d, try_idx, genv, episode, px, py, pz);
    s.cand[tid][0] = px; s.cand[tid][1] = py; s.cand[tid][2] = pz;
    if (c) { c[0] = px; c[1] = py; c[2] = pz; }
  }
  __syncthreads();
  if (active) {
    const int base = g * P.D;
    T px = s.cand[tid][0], py = s.cand[tid][1], pz = s.cand[tid][2];
    bool bad = pz < T(0.1);
    for (int j = d + 1; j < P.D; ++j)
      if (too_close(px, py, pz, s.cand[base + j][0], s.cand[base + j][1], s.cand[base + j][2])) bad = true;
    if (bad) s.reject[g] = 1;
  }
  __syncthreads();
}

// Cache policy.  Every byte the step touches is streamed: read once, written
// once per launch.  Default-policy stores leave ~30 MB dirty in the eight L2s
// and the end-of-launch write-back then runs as a serial tail; non-temporal
// (nt) stores stream to HBM while the launch computes (C3: 17.5 → 13.2 µs,
// profiles/).  aux = 2 is the nt bit of buffer/global_load_lds instructions.
#ifndef QS_SUB_CONTRACT
#define QS_SUB_CONTRACT 1
#endif
#ifndef QS_STATE_STORE_AUX
#define QS_STATE_STORE_AUX 2
#endif
#ifndef QS_STATE_LOAD_AUX
#define QS_STATE_LOAD_AUX 0
#endif
#ifndef QS_HIST_DMA_AUX
#define QS_HIST_DMA_AUX 0
#endif
#ifndef QS_NT_OBS
#define QS_NT_OBS 1
#endif
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void obs_store4(float4* p, float4 v) {
  if constexpr (QS_NT_OBS) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
  else *p = v;
}
template <class V> __device__ __forceinline__ void nt_store(V* p, V v) {
  if constexpr (QS_NT_OBS) __builtin_nontemporal_store(v, p);
  else *p = v;
}
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f3v __attribute__((ext_vector_type(3)));
// A consecutive floats (A-aligned row of [N][A]) as one non-temporal vector store.
template <int A> __device__ __forceinline__ void store_act(float* p, const float* v) {
  if constexpr (A == 4) nt_store(reinterpret_cast<f4v*>(p), f4v{v[0], v[1], v[2], v[3]});
  else if constexpr (A == 2) nt_store(reinterpret_cast<f2v*>(p), f2v{v[0], v[1]});
  else if constexpr (A == 3) { nt_store(reinterpret_cast<f2v*>(p), f2v{v[0], v[1]}); nt_store(p + 2, v[2]); }
  else {
#pragma unroll
    for (int k = 0; k < A; ++k) nt_store(p + k, v[k]);
  }
}

// Raw-buffer access to the SoA state: descriptor over the whole [F][N] array
// (wave-uniform, from kernel arguments), field base in soffset (SGPR), lane's
// 32-bit byte offset in voffset — one buffer instruction per field, no 64-bit
// per-lane address arithmetic (cdna_hip_programming.md T8).
template <class T> struct SoA {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned fstride;   // bytes per field = N * sizeof(T)
  unsigned voff;      // lane's byte offset = a * sizeof(T)
  __device__ __forceinline__ T ld(int f) const {
    if constexpr (sizeof(T) == 4) {
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)voff, (int)(f * fstride), QS_STATE_LOAD_AUX));
    } else {
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)voff, (int)(f * fstride), QS_STATE_LOAD_AUX));
    }
  }
  __device__ __forceinline__ void st(int f, T v) const {
    if constexpr (sizeof(T) == 4) {
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc, (int)voff, (int)(f * fstride), QS_STATE_STORE_AUX);
    } else {
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), rsrc, (int)voff, (int)(f * fstride), QS_STATE_STORE_AUX);
    }
  }
};

// s_waitcnt vmcnt(0) as a real instruction (not inline asm), so the compiler's
// wait-count tracking knows every earlier load has landed and does not insert
// conservative vmcnt(0) waits later — those would also wait for the early
// state stores to drain (vmcnt retires loads and stores in issue order).
// gfx9 encoding: vmcnt[3:0]=0, expcnt[6:4]=7, lgkmcnt[11:8]=15, vmcnt_hi[15:14]=0.
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// Keeps the loads on either side in source order (the scheduler would
// interleave them), so operands needed first are issued first.
__device__ __forceinline__ void issue_fence() { __asm__ volatile("" ::: "memory"); }

// ------------------------------------------------------- MARL task rewards
// Per-env rewards of FlockAviary.py:74-149, MeetupAviary.py:71-93 and
// LeaderFollowerAviary.py:71-98 from the env's drones' positions p[D][3] and
// velocities v[D][3] (LDS), in the reference's summation order.
constexpr int kTaskMarl = QS_TASK_FLOCK;   // kernel family of the three run-time MARL tasks
// Nearest-neighbour distance of drone i (FlockAviary.py:120-128).
template <class T> __device__ __forceinline__ T flock_spacing(const T (*p)[3], int D, int i) {
  T m = T(INFINITY);
  for (int j = 0; j < D; ++j)
    if (j != i) {
      const T dx = p[j][0] - p[i][0], dy = p[j][1] - p[i][1], dz = p[j][2] - p[i][2];
      const T dist = M<T>::sqrt_(dx * dx + dy * dy + dz * dz);
      m = dist < m ? dist : m;
    }
  return m;
}
// MeetupAviary._computeTerminated (MeetupAviary.py:97-117): every pair within 0.1 m.
template <class T> __device__ bool meetup_met(const T (*p)[3], int D) {
  for (int i = 0; i < D / 2; ++i) {
    const T dx = p[i][0] - p[D - 1 - i][0], dy = p[i][1] - p[D - 1 - i][1], dz = p[i][2] - p[D - 1 - i][2];
    if (M<T>::sqrt_(dx * dx + dy * dy + dz * dz) > T(0.1)) return false;
  }
  return true;
}

template <class T> __device__ T marl_reward(int task, const T (*p)[3], const T (*v)[3], int D) {
  using F = M<T>;
  auto n3 = [](T a, T b, T c) { return M<T>::sqrt_(a * a + b * b + c * c); };
  if (task == QS_TASK_FLOCK) {
    const T EPS = T(1e-3);
    T ali = 0;
    for (int i = 0; i < D; ++i) {
      const T ni = n3(v[i][0], v[i][1], v[i][2]);
      for (int j = 0; j < D; ++j)
        if (j != i) {
          const T nj = n3(v[j][0], v[j][1], v[j][2]);
          const T dd = (v[i][0] * v[j][0] + v[i][1] * v[j][1]) + v[i][2] * v[j][2];
          ali += (dd / (ni + EPS)) / (nj + EPS);
        }
    }
    ali = D > 1 ? ali / T(D * (D - 1)) : T(0);
    T c0 = 0, c1 = 0, c2 = 0;
    for (int i = 0; i < D; ++i) { c0 += v[i][0]; c1 += v[i][1]; c2 += v[i][2]; }
    const T speed = n3(c0 / T(D), c1 / T(D), c2 / T(D));
    T pen = 0, var = 0;
    if (D > 1) {
      T mean = 0;
      for (int i = 0; i < D; ++i) mean += flock_spacing(p, D, i);
      mean /= T(D);
      for (int i = 0; i < D; ++i) { const T dv = flock_spacing(p, D, i) - mean; var += dv * dv; }
      var /= T(D);
      if (!(T(1.0) < mean && mean < T(3.0))) {
        const T a = F::abs_(mean - T(1.0)), b = F::abs_(mean - T(3.0));
        pen = a < b ? a : b;
      }
    }
    return ((ali + speed) - pen) - var;
  }
  if (task == QS_TASK_MEETUP) {
    T total = 0;
    for (int i = 0; i < D / 2; ++i) {
      const T n = n3(p[i][0] - p[D - 1 - i][0], p[i][1] - p[D - 1 - i][1], p[i][2] - p[D - 1 - i][2]);
      total += (T(-1) * (n * n)) * T(2);
    }
    return total;
  }
  // LeaderFollower
  const T n0 = n3(T(0) - p[0][0], T(0) - p[0][1], T(0.5) - p[0][2]);
  T total = T(-1) * (n0 * n0);
  for (int i = 1; i < D; ++i) {
    const T dz = p[0][2] - p[i][2];
    const T n = F::sqrt_(dz * dz);
    total += (-(T(1) / T(D))) * (n * n);
  }
  return total;
}
// ------------------------------------------------------ fp32 downwash terms
// _downwash (BaseAviary.py:798-811) on a drone dz below a neighbour at
// horizontal distance² d2: α·exp(−½(dxy/β)²), α = DW1·(PROP_R/(4dz))²,
// β = DW2·dz + DW3.  fp32: reciprocals instead of divisions, exp as exp2.
__device__ __forceinline__ float dw_term(float dz, float d2) {
  const float r = __builtin_amdgcn_rcpf(dz);
  const float alpha = float(cf2x::DW1 * (cf2x::PROP_R / 4) * (cf2x::PROP_R / 4)) * (r * r);
  const float rb = __builtin_amdgcn_rcpf(float(cf2x::DW2) * dz + float(cf2x::DW3));
  return alpha * __builtin_amdgcn_exp2f((d2 * (rb * rb)) * float(-0.5 / M_LN2));
}
// DPP row_ror:K — a lane reads lane (i − K) mod 16 of its 16-lane row.
template <int K> __device__ __forceinline__ float row_ror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + K, 0xF, 0xF, false));
}
// D = 16: an env is one DPP row.  The pair term depends on |Δz| and Δxy² only,
// so each unordered pair is formed once: for K = 1..7 a lane forms the pair with
// its row neighbour K away, keeps the term when that drone is above it and hands
// it back (row_ror 16−K) when it is below; the K = 8 pairs are seen from both
// ends and each end keeps what is its own.  8 pair terms per drone instead of
// 16, no LDS, no barrier; the sum order differs from the reference's j loop
// (fp32 rounding only).
template <int K> __device__ __forceinline__ void dw16_pair(float px, float py, float pz, float& f) {
  const float qx = row_ror<K>(px), qy = row_ror<K>(py), qz = row_ror<K>(pz);
  const float dz = qz - pz, dx = qx - px, dy = qy - py;
  const float d2 = dx * dx + dy * dy;
  const bool near = d2 < 100.f;
  const float t = dw_term(fabsf(dz), d2);
  f = (near && dz > 0.f) ? f - t : f;
  if constexpr (K < 8) {
    const float back = row_ror<16 - K>((near && dz < 0.f) ? t : 0.f);
    f = f - back;
  }
}
// Four independent partial sums (pairs K ≡ 1, 2, 3, 0 mod 4), added at the end:
// the eight pair terms no longer wait on one 15-deep subtraction chain (two
// waves per SIMD could not hide it, C5's SQ counters)
__device__ __forceinline__ float downwash16(float px, float py, float pz) {
  float f1 = 0.f, f2 = 0.f, f3 = 0.f, f4 = 0.f;
  dw16_pair<1>(px, py, pz, f1); dw16_pair<2>(px, py, pz, f2); dw16_pair<3>(px, py, pz, f3);
  dw16_pair<4>(px, py, pz, f4);
#ifndef QS_DW_HALF   // (dev probe: half the pair terms, the cost of a two-lanes-per-drone split's half)
  dw16_pair<5>(px, py, pz, f1); dw16_pair<6>(px, py, pz, f2);
  dw16_pair<7>(px, py, pz, f3); dw16_pair<8>(px, py, pz, f4);
#endif
  return (f1 + f2) + (f3 + f4);
}


// ---------------------------------------------------------------- the step
// TASK (qs_task) and ACT (qs_action_type) are compile-time: each launch runs
// a kernel with only its own task's obs/reward code and its own action
// preprocessing, with the action width A folded into every index.  CF is the
// control frequency when it is the task's default at pyb_freq 240 (MultiHover
// 30 Hz, Spiral 48 Hz): the substep count, history length and obs width are
// then constants (fully unrolled substeps, constant obs offsets); CF = 0 reads
// them from P.
// AUXM selects the extra-force code: 0 compiles out the ground-effect / drag /
// downwash forces (the common P.aux == 0 case: a run-time force branch inside
// the unrolled substeps cost 0.65 µs of the 10.5 µs C3 launch); 1 = downwash
// only (C5's PYB_DW), kept on the fp32 fast substep; 2 = any combination
// through the general substep (the P.aux bits decide at run time); 3 = the
// same for DroneModel.CF2P (QS_FLAG_CF2P).
template <class T, int TASK, int ACT, int CF, int PHYS, int AUXM>
__global__ void __launch_bounds__(kBlock) step_kernel(Params<T> P) {
  using F = M<T>;
  constexpr bool kP = AUXM == 3;   // DroneModel.CF2P
  using MD = Model<kP>;
  constexpr int A = Act<ACT>::A;
  constexpr bool kPid = Act<ACT>::pid;
  constexpr bool kHover = TASK == QS_TASK_MULTIHOVER;
  constexpr bool kSpiral = TASK == QS_TASK_SPIRAL;
  constexpr bool kMarl = TASK == kTaskMarl;   // Flock / Meetup / LeaderFollower (P.task)
  __shared__ Shared<T> s;
  const int tid = threadIdx.x;
  const int D = P.D, N = P.N;
  const int H = CF ? CF / 2 : P.H;
  const int S = qs_dev::kNoCompute ? 0 : (CF ? 240 / CF : P.S);
  const int O = CF ? 12 + (CF / 2) * A + (kSpiral ? 11 : 0) : P.O;
  const int lenv = tid / D, d = tid - lenv * D;
  const int e = blockIdx.x * P.EPB + lenv;
  const bool valid = (lenv < P.EPB) && (e < P.E);
  const int a = e * D + d;
  const uint32_t genv = (uint32_t)(P.env_offset + e);
  SoA<T> SA;
  SA.rsrc = __builtin_amdgcn_make_buffer_rsrc(P.st, 0, (int)((unsigned)QS_AGENT_FIELDS * (unsigned)N * sizeof(T)), 0x00020000);
  SA.fstride = (unsigned)N * (unsigned)sizeof(T);
  SA.voff = (unsigned)a * (unsigned)sizeof(T);
  QS_STAMP(0);

  // ---------------- loads
  // Every global read of the launch is issued here, unconditionally and
  // branch-free: buffer loads return 0 out of range, so idle lanes (offset
  // kOOB) and absent optional inputs (zero-size descriptor) need no branch.
  // With straight-line issue the compiler's wait counts stay exact, so each
  // phase waits only for its own operands (vmcnt retires in issue order).
  // Nothing is read after the first store (see wait_vm0).
  constexpr unsigned kOOB = 0x80000000u;
  auto rsrc = [](const void* ptr, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), 0, (int)bytes, 0x00020000);
  };
  SA.voff = valid ? SA.voff : kOOB;
  const unsigned E = (unsigned)P.E;
  // env counters first: the synthetic action draw needs only `total`
  typedef unsigned v2u_t __attribute__((ext_vector_type(2)));
  static_assert(QS_E_STEP_COUNTER == 0 && QS_E_EPISODE == 1 && QS_E_TOTAL_STEPS == 2 && QS_E_EP_LEN == 3, "record");
  const __amdgpu_buffer_rsrc_t env_r = rsrc(P.env, (unsigned)kEnvRec * E * 4u);
  const unsigned ev = valid ? (unsigned)e * kEnvRec * 4u : kOOB;
  const v2u_t c01 = __builtin_amdgcn_raw_buffer_load_b64(env_r, (int)ev, 0, 0);
  const v2u_t c23 = __builtin_amdgcn_raw_buffer_load_b64(env_r, (int)ev, 8, 0);
  int32_t step_counter = (int32_t)c01.x, episode = (int32_t)c01.y;
  int32_t total = (int32_t)c23.x, ep_len = (int32_t)c23.y;
  const double ep_ret0 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(env_r, (int)ev, kEnvRetWord * 4, 0));
  const v2u_t c67 = __builtin_amdgcn_raw_buffer_load_b64(env_r, (int)ev, kEnvLogWord * 4, 0);
  const int32_t log_n0 = (int32_t)c67.x;
  // the precomputed search (kPreFound encoding): the next episode's try, or the
  // chunks it has rejected so far, so a queued env's search starts past them; a
  // null buffer reads 0 (num_records 0)
  const int32_t pre0 = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(
      rsrc(P.reset_pre, P.reset_pre ? E * 4u : 0u), valid ? (int)(e * 4u) : (int)kOOB, 0, 0);
  issue_fence();
  T pos[3], q[4], vel[3], w[3], lrpm[4], pid[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, tgt[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    pos[i] = SA.ld(QS_F_POS + i);
    vel[i] = SA.ld(QS_F_VEL + i);
    w[i] = SA.ld(QS_F_RPY_RATES + i);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = SA.ld(QS_F_QUAT + i);
  {   // last rpm: read only by the drag model (zero offset range otherwise: no traffic)
    SoA<T> LR = SA;
    LR.voff = (AUXM != 0 && (P.aux & QS_AUX_DRAG)) ? SA.voff : kOOB;
#pragma unroll
    for (int i = 0; i < 4; ++i) lrpm[i] = LR.ld(QS_F_LAST_RPM + i);
  }
  if constexpr (kPid) {
#pragma unroll
    for (int i = 0; i < 9; ++i) pid[i] = SA.ld(QS_F_PID_INT_POS + i);
  }
  if constexpr (kHover) {
#pragma unroll
    for (int i = 0; i < 3; ++i) tgt[i] = SA.ld(QS_F_TARGET + i);
  }
  // trainer actions (absent: zero-size descriptor), episode return, reset mask
  float act_in[A];
  {
    const __amdgpu_buffer_rsrc_t r = rsrc(P.act_in, P.act_in ? (unsigned)N * A * 4u : 0u);
    const unsigned v = valid ? (unsigned)a * A * 4u : kOOB;
#pragma unroll
    for (int k = 0; k < A; ++k) act_in[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(v + 4u * k), 0, 0));
  }
  const uint8_t mask_v = __builtin_amdgcn_raw_buffer_load_b8(
      rsrc(P.reset_mask, P.reset_mask ? E : 0u), valid ? e : (int)kOOB, 0, 0);
  const bool masked = P.reset_mask == nullptr || mask_v != 0;
  T orig[3];   // every search group needs it, also those past the last env (reset phase 2)
#pragma unroll
  for (int i = 0; i < 3; ++i) orig[i] = P.orig_xyz[d * 3 + i];
  issue_fence();
  // ---------------- the whole action-history ring (BaseRLAviary.py:66, 187,
  // 317-318): all H slots, so the addresses do not depend on the loaded ring
  // head and the reads issue with the state loads.  With the default control
  // frequency (CF != 0, H constant) the ring goes into registers with plain
  // buffer loads, issued last: the compiler's exact wait counts then let the
  // PID start as soon as the state has landed while the ring still streams.
  // Otherwise it goes into LDS by LDS-DMA, lane-linear [slot][lane][A] (A = 3
  // as [slot][k][lane]: a dwordx3 DMA does not land lane-linear at 12 B).
  extern __shared__ float4 dyn_lds4[];   // float4: 16-B aligned staging for the obs stores
  float* const dyn_lds = reinterpret_cast<float*>(dyn_lds4);
  float* const hist_pref = dyn_lds;
  float* const stage = dyn_lds + (CF ? 0 : (size_t)H * kBlock * A);
  constexpr int HR = CF ? CF / 2 : 1;
  float hreg[HR][A];
  if constexpr (CF != 0) {
    const __amdgpu_buffer_rsrc_t hr = rsrc(P.hist, (unsigned)HR * (unsigned)N * A * 4u);
    const unsigned hv = valid ? (unsigned)a * A * 4u : kOOB;
#pragma unroll
    for (int sl = 0; sl < HR; ++sl) {
      const int so = (int)((unsigned)sl * (unsigned)N * A * 4u);
      // (dword loads with the component in the immediate offset: the backend
      // merges a slot's A dwords into one dwordx2/x4 load; ROCm 7.2's clang
      // lowers __builtin_amdgcn_raw_buffer_load_b128 to a single dword load)
#pragma unroll
      for (int k = 0; k < A; ++k)
        hreg[sl][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(hr, (int)(hv + 4u * k), so, 0));
    }
  } else {
    const int a_src = valid ? a : blockIdx.x * P.EPB * D;   // idle lanes read a valid row
    for (int sl = 0; sl < H; ++sl) {
      const float* src = P.hist + ((size_t)sl * N + a_src) * A;
      if constexpr (A == 1) {
        __builtin_amdgcn_global_load_lds((g_ptr_t)src, (lds_ptr_t)(hist_pref + sl * kBlock), 4, 0, QS_HIST_DMA_AUX);
      } else if constexpr (A == 3) {
        for (int k = 0; k < 3; ++k)
          __builtin_amdgcn_global_load_lds((g_ptr_t)(src + k), (lds_ptr_t)(hist_pref + (sl * 3 + k) * kBlock), 4, 0, QS_HIST_DMA_AUX);
      } else {
        __builtin_amdgcn_global_load_lds((g_ptr_t)src, (lds_ptr_t)(hist_pref + sl * kBlock * 4), 16, 0, QS_HIST_DMA_AUX);
      }
    }
  }
  auto hist_at = [&](int sl, int k) -> float {   // LDS image (CF == 0): ring slot sl, component k, this lane
    return A == 3 ? hist_pref[(sl * 3 + k) * kBlock + tid] : hist_pref[(sl * kBlock + tid) * A + k];
  };
  // history ring head: this step's action goes to slot total % H
  const int wslot = total % H;
  // kinematic state + last_clipped_action (BaseAviary.py:509-519, 560)
  auto store_kin = [&]() {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      SA.st(QS_F_POS + i, pos[i]);
      SA.st(QS_F_VEL + i, vel[i]);
      SA.st(QS_F_RPY_RATES + i, w[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) SA.st(QS_F_QUAT + i, q[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) SA.st(QS_F_LAST_RPM + i, lrpm[i]);
  };
  T angv[3] = {0, 0, 0}, rpy[3] = {0, 0, 0};
  double ep_ret_out = ep_ret0;   // VecRecordEpisodeStatistics accumulators after this call
  int32_t ep_len_out = ep_len;
  int32_t log_n = log_n0;        // episodes logged by this env
  bool done_env = false;
  int obs_sc = step_counter;   // step_counter seen by _computeObs (before BaseAviary.py:382)

  float cur_act[A];            // this step's action (newest history entry)
#pragma unroll
  for (int k = 0; k < A; ++k) cur_act[k] = 0.f;
  QS_STAMP_SINK(pos[0] + q[3] + pid[0] + tgt[0] + (T)total);
  // ---------------- action (trainer-provided or synthetic random policy)
  if (P.mode == MODE_STEP) {
    if (P.act_in) {
#pragma unroll
      for (int k = 0; k < A; ++k) cur_act[k] = act_in[k];
    } else {
      U4 r = philox(U4{(uint32_t)total, genv, 0u, (uint32_t)((STREAM_ACT << 24) | d)}, P.k0, P.k1);
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int k = 0; k < A; ++k) cur_act[k] = 2.0f * u01<float>(rr[k]) - 1.0f;
    }
  }
  QS_STAMP(1);
  if (P.mode == MODE_STEP) {
    const float* act = cur_act;
    // ---------------- _preprocessAction (BaseRLAviary.py:188-239)
    T rpm[4] = {0, 0, 0, 0};
    if (valid) {
      const T z3[3] = {0, 0, 0};
      if constexpr (ACT == QS_ACT_RPM) {
#pragma unroll
        for (int m = 0; m < 4; ++m) rpm[m] = T(cf2x::HOVER_RPM) * (T(1) + T(0.05) * T(act[m]));
      } else if constexpr (ACT == QS_ACT_ONE_D_RPM) {
        T r = T(cf2x::HOVER_RPM) * (T(1) + T(0.05) * T(act[0]));
        rpm[0] = rpm[1] = rpm[2] = rpm[3] = r;
      } else {
        if (!qs_dev::kNoCompute) quat_to_rpy(q, rpy);   // DSLPIDControl.py:240 (and the VEL target yaw, BRL:221)
        if constexpr (ACT == QS_ACT_ONE_D_PID) {
          T tp[3] = {pos[0], pos[1], pos[2] + T(0.1) * T(act[0])};
          dsl_pid<T, kP>(P.ctrl_dt, P.ctrl_hz, pid, pos, q, vel, rpy, tp, T(0), z3, rpm);
        } else if constexpr (ACT == QS_ACT_VEL) {
          T v0 = T(act[0]), v1 = T(act[1]), v2 = T(act[2]);
          T n = F::sqrt_(v0 * v0 + v1 * v1 + v2 * v2);
          T u0 = 0, u1 = 0, u2 = 0;
          if (n != T(0)) { u0 = v0 / n; u1 = v1 / n; u2 = v2 / n; }
          T sp = T(cf2x::SPEED_LIMIT) * F::abs_(T(act[3]));
          T tv[3] = {sp * u0, sp * u1, sp * u2};
          dsl_pid<T, kP>(P.ctrl_dt, P.ctrl_hz, pid, pos, q, vel, rpy, pos, rpy[2], tv, rpm);
        } else {   // QS_ACT_PID: _calculateNextStep (BaseAviary.py:1108-1150)
          T dir[3] = {T(act[0]) - pos[0], T(act[1]) - pos[1], T(act[2]) - pos[2]};
          T dist = F::sqrt_(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
          T np_[3];
          if (dist <= T(1)) { np_[0] = T(act[0]); np_[1] = T(act[1]); np_[2] = T(act[2]); }
          else { for (int i = 0; i < 3; ++i) np_[i] = pos[i] + (dir[i] / dist) * T(1); }
          dsl_pid<T, kP>(P.ctrl_dt, P.ctrl_hz, pid, pos, q, vel, rpy, np_, T(0), z3, rpm);
        }
      }
    }
    // Every load of the launch has landed before the first store, so no later
    // wait is held up by the stores (see wait_vm0).  The compiler's own waits
    // let the action draw and the PID start as soon as the state loads land,
    // with the history LDS-DMA (issued last) still streaming.
    wait_vm0();
    if (valid) {
      // one vector store per lane for the A components (a wave writes whole
      // lines; per-component dword stores left 16-B-strided partial lines)
      if (P.act_out) store_act<A>(P.act_out + (size_t)a * A, act);
      // action_buffer.append(action) (BaseRLAviary.py:187): ring slot total % H
      store_act<A>(P.hist + ((size_t)wslot * N + a) * A, act);
      if constexpr (kPid) {   // PID integrators are final: store now, drains under the substeps
#pragma unroll
        for (int i = 0; i < 9; ++i) SA.st(QS_F_PID_INT_POS + i, pid[i]);
      }
    }
    QS_STAMP(2);
    // ---------------- PYB_STEPS_PER_CTRL substeps (BaseAviary.py:343-372)
    T f[4], zt[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) { f[m] = rpm[m] * rpm[m] * T(cf2x::KF); zt[m] = rpm[m] * rpm[m] * T(cf2x::KM); }
    const T thrust_z = ((f[0] + f[1]) + f[2]) + f[3];
    const T tz = ((-zt[0] + zt[1]) - zt[2]) + zt[3];
    // BaseAviary.py:849-850 (CF2X), 852-853 (CF2P)
    const T tx = kP ? (f[1] - f[3]) * T(cf2x::L) : -(((f[0] + f[1]) - f[2]) - f[3]) * T(cf2x::L_SQRT2);
    const T ty = kP ? (-f[0] + f[2]) * T(cf2x::L) : (((-f[0] + f[1]) + f[2]) - f[3]) * T(cf2x::L_SQRT2);
    // PYB: the four prop forces act at their links' COMs (assets/cf2x.urdf:42-79, cf2p.urdf:42-79)
    const T pbx = (((T(MD::PY[0]) * f[0]) + T(MD::PY[1]) * f[1]) + T(MD::PY[2]) * f[2]) + T(MD::PY[3]) * f[3];
    const T pby = (((-T(MD::PX[0]) * f[0]) + -T(MD::PX[1]) * f[1]) + -T(MD::PX[2]) * f[2]) + -T(MD::PX[3]) * f[3];
    const T dt = P.dt;
    // The exp-map update preserves |q| (cos²θ + sin²θ = 1), so in fp32 Bullet's
    // s = 2/|q|² (getMatrixFromQuaternion) is formed once per control step; it
    // moves by rounding only between substeps.
    const T s2 = T(2) * F::rcp(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    T R[9];   // PYB: rotation of the current pose, carried across substeps
    if constexpr (PHYS == QS_PHYS_PYB) quat_to_rot(q, R);
    // Drone–drone contact (PYB; Bullet keeps every drone's collision cylinder,
    // cf2x.urdf:31-36, BaseAviary.py:484-503).  Broad phase: Mw = the wave's
    // smallest horizontal centre distance at the step start.  A drone that has
    // moved at most B = (Mw − 2r)/2 − margin horizontally cannot close a gap to
    // 2r with another drone that has also moved at most B, so the exact pair
    // pass (contact_pairs, one lane per env over LDS) runs only from the first
    // substep at which some drone of the wave has moved farther, and then for
    // the rest of the step.  |Δxy| per substep <= dt (|vx| + |vy|).
    float c_budget = 0.f, c_moved = 0.f;
    bool c_slow = false;
    if constexpr (PHYS == QS_PHYS_PYB) {
      if (D > 1) {
        __syncthreads();
        s.cand[tid][0] = pos[0]; s.cand[tid][1] = pos[1];
        __syncthreads();
        float m2 = 1e30f;
        if (valid) {
          const int base = lenv * D;
          for (int j = 0; j < D; ++j) {
            const float dx = float(s.cand[base + j][0] - pos[0]), dy = float(s.cand[base + j][1] - pos[1]);
            const float q2 = dx * dx + dy * dy;
            m2 = (j != d && q2 < m2) ? q2 : m2;
          }
        }
        c_budget = 0.5f * (sqrtf(wave_min(m2)) - float(2 * kCylR)) - 1e-4f;
        c_slow = c_budget <= 0.f;
      }
    }
    // after the substep's integration and ground check (pos, vel final); r8 = R22
    auto contacts = [&](T r8) {
      if (D < 2) return;
      c_moved += float(dt) * (fabsf(float(vel[0])) + fabsf(float(vel[1])));
      if (!c_slow) c_slow = __ballot(valid && c_moved > c_budget) != 0;   // wave-uniform
      if (!c_slow) return;
      __syncthreads();
      s.cand[tid][0] = pos[0]; s.cand[tid][1] = pos[1]; s.cand[tid][2] = pos[2];
      s.velw[tid][0] = vel[0]; s.velw[tid][1] = vel[1]; s.velw[tid][2] = vel[2];
      s.rew[tid] = T(kCylHalfLen) * F::abs_(r8) + T(kCylR) * F::sqrt_(T(1) - r8 * r8 > T(0) ? T(1) - r8 * r8 : T(0));
      __syncthreads();
      if (valid && d == 0) contact_pairs<T>(&s.cand[tid], &s.velw[tid], &s.rew[tid], D);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 3; ++i) { pos[i] = s.cand[tid][i]; vel[i] = s.velw[tid][i]; }
    };
    // fp32 without extra forces at pyb_freq 240 (the hot configurations): the
    // substep is restated algebraically with every per-control-step constant
    // hoisted — the thrust, gravity and torque terms premultiplied by dt/M and
    // dt/J, the body z axis from q directly (s = 2/|q|² once per step), the
    // gyroscopic term reduced with IXX == IYY, and the PYB world-frame exp map
    // applied as the equivalent right product q ⊗ exp(ω_body dt/2) (R(q)ω = q ω q*).
    // Same mathematics as the general path below; fp32 rounding only.
    constexpr bool kFastSub = sizeof(T) == 4 && AUXM < 2 && CF != 0;
    // _downwash (BaseAviary.py:798-811) for the fast substep: the body-z force of the
    // drones above, from the neighbours' substep-start positions.  D = 16 through
    // DPP (downwash16); otherwise one float4 per drone in LDS, four neighbours in
    // flight, the pair test as a select (no branch in the unrolled loop).
    auto downwash_f32 = [&]() -> float {
      const float px = float(pos[0]), py = float(pos[1]), pz = float(pos[2]);
      if (D == 16) return downwash16(px, py, pz);   // wave-uniform
      float4* const nb = s.dw4;
      __syncthreads();
      nb[tid] = make_float4(px, py, pz, 0.f);
      __syncthreads();
      float f = 0.f;
      if (valid) {
        const float4* const en = nb + lenv * D;
#pragma unroll 4
        for (int j = 0; j < D; ++j) {
          const float4 q4 = en[j];
          const float dz = q4.z - pz, dx = q4.x - px, dy = q4.y - py;
          const float d2 = dx * dx + dy * dy;
          const float t = dw_term(dz, d2);
          f = (dz > 0.f && d2 < 100.f) ? f - t : f;
        }
      }
      return f;
    };
    if constexpr (kFastSub) {
#pragma clang fp contract(fast)
      constexpr double kDt = 1.0 / 240.0;   // CF != 0 ⇒ pyb_freq == 240 (step_launch_impl.h)
      constexpr double IXX = cf2x::IXX, IYY = cf2x::IYY, IZZ = cf2x::IZZ;
      static_assert(cf2x::IXX == cf2x::IYY, "gyroscopic reduction assumes IXX == IYY (cf2x.urdf:11-12)");
      constexpr float kx = float(kDt * (IZZ - IYY) / IXX), ky = float(kDt * (IXX - IZZ) / IYY);
      constexpr float kHdt = float(kDt / 2), kHdt2 = float(kDt / 2 * (kDt / 2));
      const float dtm = float(kDt / cf2x::M);
      // exp-map coefficients: c = cos θ, k = sin θ / |ω|, θ = |ω| dt / 2
      auto expmap = [&](float wn2, float& c, float& k) {
        const float u = wn2 * kHdt2;
        if (u < 0.0625f) {
          k = __builtin_fmaf(u, __builtin_fmaf(u, __builtin_fmaf(u, float(kDt / 2 * (-1.0 / 5040)), float(kDt / 2 / 120)),
                                               float(kDt / 2 * (-1.0 / 6))), kHdt);
          c = __builtin_fmaf(u, __builtin_fmaf(u, __builtin_fmaf(u, __builtin_fmaf(u, float(1.0 / 40320), float(-1.0 / 720)),
                                                                 float(1.0 / 24)), -0.5f), 1.0f);
        } else {
          // rare (|ω| > 120 rad/s): hardware sin/cos, no library range reduction
          // unrolled into every substep
          const float wn = sqrtf(wn2), th = wn * kHdt;
          c = __cosf(th);
          k = __sinf(th) * __builtin_amdgcn_rcpf(wn);
        }
      };
      if constexpr (PHYS == QS_PHYS_PYB) {
        const float kd = float(kDt * kPybDamping);
        float g1 = thrust_z * dtm, g2 = 2.0f * g1, c8 = g1 - float(cf2x::GRAVITY * kDt / cf2x::M);
        const float bx = float(kDt / IXX) * pbx, by = float(kDt / IYY) * pby, bz = float(kDt / IZZ) * tz;
        constexpr float amax2 = float((0.25 * M_PI / kDt) * (0.25 * M_PI / kDt));
#pragma unroll
        for (int sub = 0; sub < S; ++sub) {
          if constexpr (AUXM == 1) {
            g1 = (thrust_z + downwash_f32()) * dtm;
            g2 = 2.0f * g1;
            c8 = g1 - float(cf2x::GRAVITY * kDt / cf2x::M);
          }
          const float x = q[0], y = q[1], z = q[2], qw = q[3];
          const float m = __builtin_fmaf(-kd, sqrtf(vel[0] * vel[0] + vel[1] * vel[1] + vel[2] * vel[2]), 1.0f - kd);
          const float mw = __builtin_fmaf(-kd, sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]), 1.0f - kd);
          vel[0] = vel[0] * m + g2 * (x * z + qw * y);
          vel[1] = vel[1] * m + g2 * (y * z - qw * x);
          vel[2] = vel[2] * m + (c8 - g2 * (x * x + y * y));
          const float w0 = w[0], w1 = w[1], w2 = w[2];
          w[0] = w0 * mw + (bx - kx * (w1 * w2));
          w[1] = w1 * mw + (by - ky * (w2 * w0));
          w[2] = w2 * mw + bz;
#pragma unroll
          for (int i = 0; i < 3; ++i) pos[i] = pos[i] + float(kDt) * vel[i];
          float ang2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
          ang2 = ang2 > amax2 ? amax2 : ang2;
          float c, kk;
          expmap(ang2, c, kk);
          const float e0 = w[0] * kk, e1 = w[1] * kk, e2 = w[2] * kk;
          const float n0 = c * x + qw * e0 + (y * e2 - z * e1);
          const float n1 = c * y + qw * e1 + (z * e0 - x * e2);
          const float n2 = c * z + qw * e2 + (x * e1 - y * e0);
          const float n3 = c * qw - (x * e0 + y * e1 + z * e2);
          const float rn = __builtin_amdgcn_rsqf(n0 * n0 + n1 * n1 + n2 * n2 + n3 * n3);
          q[0] = n0 * rn; q[1] = n1 * rn; q[2] = n2 * rn; q[3] = n3 * rn;
          if (pos[2] < float(kCylHalfLen + kCylR)) {   // ground plane vs the collision cylinder
            const float r8 = 1.0f - 2.0f * (q[0] * q[0] + q[1] * q[1]);
            const float sz2 = 1.0f - r8 * r8;
            const float zmin = pos[2] - (float(kCylHalfLen) * fabsf(r8) + float(kCylR) * sqrtf(sz2 > 0.f ? sz2 : 0.f));
            if (zmin < 0.f) {
              pos[2] = pos[2] - zmin;
              if (vel[2] < 0.f) vel[2] = 0.f;
            }
          }
          contacts(1.0f - 2.0f * (q[0] * q[0] + q[1] * q[1]));   // drone–drone (rare: broad phase above)
        }
        T Rn[9];   // getBaseVelocity: world angular velocity at the new pose
        quat_to_rot(q, Rn);
        angv[0] = Rn[0] * w[0] + Rn[1] * w[1] + Rn[2] * w[2];
        angv[1] = Rn[3] * w[0] + Rn[4] * w[1] + Rn[5] * w[2];
        angv[2] = Rn[6] * w[0] + Rn[7] * w[1] + Rn[8] * w[2];
      } else {
        float gk = thrust_z * s2 * dtm, c8 = (thrust_z - float(cf2x::GRAVITY)) * dtm;
        const float ax = float(kDt / IXX) * tx, ay = float(kDt / IYY) * ty, az = float(kDt / IZZ) * tz;
#pragma unroll
        for (int sub = 0; sub < S; ++sub) {
          if constexpr (AUXM == 1) {
            const float zb = thrust_z + downwash_f32();
            gk = zb * s2 * dtm;
            c8 = (zb - float(cf2x::GRAVITY)) * dtm;
          }
          const float x = q[0], y = q[1], z = q[2], qw = q[3];
          vel[0] = vel[0] + gk * (x * z + qw * y);
          vel[1] = vel[1] + gk * (y * z - qw * x);
          vel[2] = (vel[2] + c8) - gk * (x * x + y * y);
          const float w0 = w[0], w1 = w[1], w2 = w[2];
          w[0] = (w0 + ax) - kx * (w1 * w2);
          w[1] = (w1 + ay) - ky * (w2 * w0);
          w[2] = w2 + az;
#pragma unroll
          for (int i = 0; i < 3; ++i) pos[i] = pos[i] + float(kDt) * vel[i];
          if (sub == S - 1) {   // world angular velocity R_old·ω (BaseAviary.py:871-875)
            T Ro[9];
            quat_to_rot(q, Ro);
            angv[0] = Ro[0] * w[0] + Ro[1] * w[1] + Ro[2] * w[2];
            angv[1] = Ro[3] * w[0] + Ro[4] * w[1] + Ro[5] * w[2];
            angv[2] = Ro[6] * w[0] + Ro[7] * w[1] + Ro[8] * w[2];
          }
          const float wn2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
          if (wn2 > 1e-16f) {   // _integrateQ (BaseAviary.py:879-892)
            float c, k;
            expmap(wn2, c, k);
            const float kp = k * w[0], kq = k * w[1], kr = k * w[2];
            q[0] = c * x + (kr * y - kq * z + kp * qw);
            q[1] = c * y + (-kr * x + kp * z + kq * qw);
            q[2] = c * z + (kq * x - kp * y + kr * qw);
            q[3] = c * qw + (-kp * x - kq * y - kr * z);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) lrpm[m] = rpm[m];   // last_clipped_action (BaseAviary.py:372)
    } else {
    // One substep (BaseAviary.py:343-372).  kAux: ground effect / drag /
    // downwash enabled; the common force-free path is compiled separately.
#pragma unroll
    for (int sub = 0; sub < S; ++sub) {
#if QS_SUB_CONTRACT
      // a*b+c → fma inside the substep (≈25 % fewer instructions).  The one
      // sum whose exact cancellation matters — the gyroscopic ω × Jω, zero
      // about a symmetric axis — is written with non-contractable _rn ops.
#pragma clang fp contract(fast)
#endif
      T R2, R5, R8;
      // fp64 (the tight-parity path) re-forms s every substep exactly as Bullet does
      const T sq = sizeof(T) == 8 ? T(2) * F::rcp(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]) : s2;
      quat_to_zaxis_s(q, sq, R2, R5, R8);
      T zb = thrust_z, txe = 0, tye = 0, fwx = 0, fwy = 0, fwz = 0;
      if (AUXM != 0 && P.aux) {
        // no contraction here: the four ground-effect torque arms cancel exactly
        // for a level drone only in plain multiply-then-add arithmetic
#pragma clang fp contract(off)
        if (P.aux & QS_AUX_GND) {  // _groundEffect (BaseAviary.py:731-750)
          T srpy[3], R[9];
          quat_to_rpy(q, srpy);
          quat_to_rot(q, R);
          if (F::abs_(srpy[0]) < T(M_PI / 2) && F::abs_(srpy[1]) < T(M_PI / 2)) {
            const T PX[4] = {T(MD::PX[0]), T(MD::PX[1]), T(MD::PX[2]), T(MD::PX[3])};
            const T PY[4] = {T(MD::PY[0]), T(MD::PY[1]), T(MD::PY[2]), T(MD::PY[3])};
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              T h = pos[2] + (R[6] * PX[m] + R[7] * PY[m]);
              h = h < T(cf2x::GND_CLIP) ? T(cf2x::GND_CLIP) : h;
              T ratio = T(cf2x::PROP_R) / (T(4) * h);
              T g = rpm[m] * rpm[m] * T(cf2x::KF) * T(cf2x::GND_COEFF) * (ratio * ratio);
              zb += g; txe += PY[m] * g; tye += -PX[m] * g;
            }
          }
        }
        if (P.aux & QS_AUX_DRAG) {  // _drag (BaseAviary.py:770-781), previous-substep rpm
          T sr = 0;
#pragma unroll
          for (int m = 0; m < 4; ++m) sr += T(2 * M_PI) * lrpm[m] / T(60);
          fwx += (T(-1) * T(cf2x::DRAG_XY) * sr) * vel[0];
          fwy += (T(-1) * T(cf2x::DRAG_XY) * sr) * vel[1];
          fwz += (T(-1) * T(cf2x::DRAG_Z) * sr) * vel[2];
        }
        if (P.aux & QS_AUX_DW) {  // _downwash (BaseAviary.py:798-811): neighbours' substep-start z via LDS
          __syncthreads();
          s.cand[tid][0] = pos[0]; s.cand[tid][1] = pos[1]; s.cand[tid][2] = pos[2];
          __syncthreads();
          if (valid) {
            const int base = lenv * D;
            for (int j = 0; j < D; ++j) {
              T dz = s.cand[base + j][2] - pos[2];
              T dx = s.cand[base + j][0] - pos[0], dy = s.cand[base + j][1] - pos[1];
              T dxy = F::sqrt_(dx * dx + dy * dy);
              if (dz > T(0) && dxy < T(10)) {
                T ratio = T(cf2x::PROP_R) / (T(4) * dz);
                T alpha = T(cf2x::DW1) * (ratio * ratio);
                T beta = T(cf2x::DW2) * dz + T(cf2x::DW3);
                T qq = dxy / beta;
                zb += -alpha * F::exp_(T(-.5) * (qq * qq));
              }
            }
          }
        }
      }
      if constexpr (PHYS == QS_PHYS_PYB) {
        // Bullet's step of the _physics forces (BA:679-711, 369-370), restated
        // as the oracle's pyb_dynamics.  No contraction: the
        // torque sums cancel exactly for equal rotors only without FMA, and the
        // fp64 build tracks the oracle over long free-running rollouts.
        // R is the rotation of the (normalised) q, carried from the previous
        // substep's ground check.
#pragma clang fp contract(off)
        const T k = T(kPybDamping);
        T fw0 = R[2] * zb + fwx, fw1 = R[5] * zb + fwy, fw2 = (R[8] * zb - T(cf2x::GRAVITY)) + fwz;
        const T vd = k + k * F::sqrt_(vel[0] * vel[0] + vel[1] * vel[1] + vel[2] * vel[2]);
        const T a0 = F::divc(fw0, cf2x::M) - vd * vel[0], a1 = F::divc(fw1, cf2x::M) - vd * vel[1];
        const T a2 = F::divc(fw2, cf2x::M) - vd * vel[2];
        T Jw0 = T(MD::IXX) * w[0], Jw1 = T(MD::IYY) * w[1], Jw2 = T(MD::IZZ) * w[2];
        T c0 = w[1] * Jw2 - w[2] * Jw1, c1 = w[2] * Jw0 - w[0] * Jw2, c2 = w[0] * Jw1 - w[1] * Jw0;
        const T wdm = k + k * F::sqrt_(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        T wd0 = T(1.0 / MD::IXX) * (((pbx + txe) - c0) - wdm * Jw0);
        T wd1 = T(1.0 / MD::IYY) * (((pby + tye) - c1) - wdm * Jw1);
        T wd2 = T(1.0 / MD::IZZ) * ((tz - c2) - wdm * Jw2);
        vel[0] = vel[0] + dt * a0;
        vel[1] = vel[1] + dt * a1;
        vel[2] = vel[2] + dt * a2;
        w[0] = w[0] + dt * wd0;
        w[1] = w[1] + dt * wd1;
        w[2] = w[2] + dt * wd2;
#pragma unroll
        for (int i = 0; i < 3; ++i) pos[i] = pos[i] + dt * vel[i];
        // exp map of the world angular velocity (|ω|dt clamped to π/4), renormalised
        const T ww0 = R[0] * w[0] + R[1] * w[1] + R[2] * w[2];
        const T ww1 = R[3] * w[0] + R[4] * w[1] + R[5] * w[2];
        const T ww2 = R[6] * w[0] + R[7] * w[1] + R[8] * w[2];
        T ang2 = ww0 * ww0 + ww1 * ww1 + ww2 * ww2;
        const T amax = T(0.25 * M_PI) / dt;
        if (ang2 > amax * amax) ang2 = amax * amax;
        T c, kk;
        expmap_coeffs(ang2, P.hdt, P.hdt2, c, kk);   // cos(|ω|dt/2), sin(|ω|dt/2)/|ω|
        const T e0 = ww0 * kk, e1 = ww1 * kk, e2 = ww2 * kk;
        const T x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
        T n0 = ((c * x0 + e0 * x3) + e1 * x2) - e2 * x1;
        T n1 = ((c * x1 - e0 * x2) + e1 * x3) + e2 * x0;
        T n2 = ((c * x2 + e0 * x1) - e1 * x0) + e2 * x3;
        T n3 = ((c * x3 - e0 * x0) - e1 * x1) - e2 * x2;
        if constexpr (sizeof(T) == 4) {
          const T rn = F::rsqrt(n0 * n0 + n1 * n1 + n2 * n2 + n3 * n3);
          q[0] = n0 * rn; q[1] = n1 * rn; q[2] = n2 * rn; q[3] = n3 * rn;
        } else {
          const T qn = F::sqrt_(n0 * n0 + n1 * n1 + n2 * n2 + n3 * n3);
          q[0] = n0 / qn; q[1] = n1 / qn; q[2] = n2 / qn; q[3] = n3 / qn;
        }
        quat_to_rot(q, R);   // the new pose: ground check, readback, next substep
        // ground plane vs the collision cylinder (cf2x.urdf:32-35); the cylinder
        // reaches at most kCylHalfLen + kCylR below its centre
        if (pos[2] < T(kCylHalfLen + kCylR)) {
          const T cz = F::abs_(R[8]);
          const T sz = F::sqrt_(T(1) - R[8] * R[8] > T(0) ? T(1) - R[8] * R[8] : T(0));
          const T zmin = pos[2] - (T(kCylHalfLen) * cz + T(kCylR) * sz);
          if (zmin < T(0)) {
            pos[2] = pos[2] - zmin;
            if (vel[2] < T(0)) vel[2] = T(0);
          }
        }
        contacts(R[8]);   // drone–drone (rare: broad phase above)
        if (sub == S - 1) {   // getBaseVelocity: world angular velocity at the new pose
          angv[0] = R[0] * w[0] + R[1] * w[1] + R[2] * w[2];
          angv[1] = R[3] * w[0] + R[4] * w[1] + R[5] * w[2];
          angv[2] = R[6] * w[0] + R[7] * w[1] + R[8] * w[2];
        }
      } else {
        // _dynamics (BaseAviary.py:836-877)
        T fw0 = R2 * zb + fwx, fw1 = R5 * zb + fwy, fw2 = (R8 * zb - T(cf2x::GRAVITY)) + fwz;
        T Jw0 = T(MD::IXX) * w[0], Jw1 = T(MD::IYY) * w[1], Jw2 = T(MD::IZZ) * w[2];
        T c0 = w[1] * Jw2 - w[2] * Jw1, c1 = w[2] * Jw0 - w[0] * Jw2, c2 = w[0] * Jw1 - w[1] * Jw0;
        T wd0 = T(1.0 / MD::IXX) * ((tx + txe) - c0), wd1 = T(1.0 / MD::IYY) * ((ty + tye) - c1);
        T wd2 = T(1.0 / MD::IZZ) * (tz - c2);
        vel[0] = vel[0] + dt * F::divc(fw0, cf2x::M);
        vel[1] = vel[1] + dt * F::divc(fw1, cf2x::M);
        vel[2] = vel[2] + dt * F::divc(fw2, cf2x::M);
        w[0] = w[0] + dt * wd0;
        w[1] = w[1] + dt * wd1;
        w[2] = w[2] + dt * wd2;
  #pragma unroll
        for (int i = 0; i < 3; ++i) pos[i] = pos[i] + dt * vel[i];
        if (sub == S - 1) {
          // world angular velocity R_old·ω written to Bullet (BaseAviary.py:871-875);
          // only the last substep's value reaches the obs.
          T R[9];
          quat_to_rot(q, R);
          angv[0] = R[0] * w[0] + R[1] * w[1] + R[2] * w[2];
          angv[1] = R[3] * w[0] + R[4] * w[1] + R[5] * w[2];
          angv[2] = R[6] * w[0] + R[7] * w[1] + R[8] * w[2];
        }
        // _integrateQ (BaseAviary.py:879-892); np.isclose(|ω|, 0) ⇔ |ω| <= 1e-8
        const T wn2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
        if (wn2 > T(1e-16)) {
          T c, k;
          expmap_coeffs(wn2, P.hdt, P.hdt2, c, k);
          const T p_ = w[0], q_ = w[1], r_ = w[2];
          const T x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
          q[0] = c * x0 + k * (r_ * x1 - q_ * x2 + p_ * x3);
          q[1] = c * x1 + k * (-r_ * x0 + p_ * x2 + q_ * x3);
          q[2] = c * x2 + k * (q_ * x0 - p_ * x1 + r_ * x3);
          q[3] = c * x3 + k * (-p_ * x0 - q_ * x1 - r_ * x2);
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) lrpm[m] = rpm[m];   // last_clipped_action (BaseAviary.py:372)
    }
    }   // general substep path
    quat_to_rpy(q, rpy);   // readback (BaseAviary.py:374, 518)
    total += 1;
    // Kinematic state is final unless this env auto-resets (rewritten below):
    // store now so the writes drain under the reward / obs phases.
    if (valid) store_kin();
    QS_STAMP(3);

    // ---------------- reward / termination per drone
    T rterm = 0;
    uint8_t bits = 0;
    if (valid) {
      if constexpr (kHover) {  // MultiHoverAviary.py:128-186, 216-241
        T ex = pos[0] - tgt[0], ey = pos[1] - tgt[1];
        T err_xy = F::sqrt_(ex * ex + ey * ey);
        T err_z = pos[2] - tgt[2];
        T vz = vel[2];
        T r_xy = F::rcp(T(1) + err_xy);
        T r_z = F::exp_(T(-7.5) * F::abs_(err_z));
        T r_vel = F::abs_(err_z) < T(0.2) ? T(-1.5) * (vz * vz) : T(0);
        T hover = (err_xy < T(0.03) && F::abs_(err_z) < T(0.03) && F::abs_(vz) < T(0.03)) ? T(0.5) : T(0);
        rterm = ((r_xy + r_z) + r_vel) + hover;
        if (pos[2] < T(0.03)) bits |= QS_REASON_CRASH;
        if (F::abs_(rpy[0]) > T(1.2) || F::abs_(rpy[1]) > T(1.2)) bits |= QS_REASON_FLIP;
        if (F::abs_(pos[0]) > T(3.0) || F::abs_(pos[1]) > T(3.0)) bits |= QS_REASON_OOB;
      } else if constexpr (kMarl) {
        // Flock/Meetup/LeaderFollower._computeTruncated: out of the task's box or
        // |roll|, |pitch| > 0.4 (FlockAviary.py:169-186, MeetupAviary.py:121-151,
        // LeaderFollowerAviary.py:118-144); the env reward is formed below
        bool out;
        if (P.task == QS_TASK_FLOCK)
          out = F::abs_(pos[0]) > T(10.0) || F::abs_(pos[1]) > T(10.0) || pos[2] > T(10.0);
        else if (P.task == QS_TASK_MEETUP)
          out = F::abs_(pos[0]) > T(5.0) || F::abs_(pos[1]) > T(5.0) || pos[2] > T(3.0) || pos[2] < T(0.1);
        else
          out = F::abs_(pos[0]) > T(2.0) || F::abs_(pos[1]) > T(2.0) || pos[2] > T(2.0);
        if (out || F::abs_(rpy[0]) > T(.4) || F::abs_(rpy[1]) > T(.4)) bits = 1;
      } else {  // SpiralAviary.py:82-99, 150-191
        T t = T((double)step_counter / (double)P.pyb_freq);
        T ph = P.sp_OMEGA * t + T(2 * M_PI) * T(d) / T(D);
        T prx = P.sp_cx + P.sp_R * F::cos_(ph), pry = P.sp_cy + P.sp_R * F::sin_(ph), prz = T(0.3) + P.sp_VZ * t;
        T vrx = -P.sp_R * P.sp_OMEGA * F::sin_(ph), vry = P.sp_R * P.sp_OMEGA * F::cos_(ph), vrz = P.sp_VZ;
        T dp0 = pos[0] - prx, dp1 = pos[1] - pry, dp2 = pos[2] - prz;
        T dv0 = q[0] - vrx, dv1 = q[1] - vry, dv2 = q[2] - vrz;   // "vel" = quat xyz (SP:156)
        T np_ = F::sqrt_(dp0 * dp0 + dp1 * dp1 + dp2 * dp2), nv = F::sqrt_(dv0 * dv0 + dv1 * dv1 + dv2 * dv2);
        T r_pos = F::exp_(T(-4.0) * (np_ * np_));
        T r_vel = F::exp_(T(-2.0) * (nv * nv));
        T rx = pos[0] - P.sp_cx, ry = pos[1] - P.sp_cy;
        T rn = F::sqrt_(rx * rx + ry * ry);
        T r_tan = 0;
        if (rn > T(1e-3)) {
          T tnx = -(ry / rn), tny = rx / rn;
          T vx = q[0], vy = q[1];
          T vn = F::sqrt_(vx * vx + vy * vy);
          if (vn > T(1e-3)) {
            T dot = (vx / vn) * tnx + (vy / vn) * tny;
            r_tan = dot > T(0) ? dot : T(0);
          }
        }
        rterm = (T(1.0) * r_pos + T(2.0) * r_vel) + T(1.0) * r_tan;
        if (pos[2] < T(0.05) || pos[2] > T(3.0)) bits |= QS_REASON_ZRANGE;
      }
    }
    s.rew[tid] = rterm;
    s.bits[tid] = bits;
    if constexpr (kMarl) {
#pragma unroll
      for (int i = 0; i < 3; ++i) { s.cand[tid][i] = pos[i]; s.velw[tid][i] = vel[i]; }
    }
    __syncthreads();
    // per-env reduction in drone order (reference: reward += ... for i in range(D))
    bool dn = false;
    double ret = 0;
    int len = 0;
    if (valid && d == 0) {
      T rsum = 0;
      uint8_t any = 0;
      for (int j = 0; j < D; ++j) { rsum += s.rew[tid + j]; any |= s.bits[tid + j]; }
      T r = rsum / T(D);
      bool te = any != 0;
      bool tr = ((double)step_counter / (double)P.pyb_freq) > P.ep_len_sec;   // MultiHoverAviary.py:267-268
      if constexpr (kMarl) {
        r = marl_reward<T>(P.task, &s.cand[tid], &s.velw[tid], D);
        te = P.task == QS_TASK_MEETUP && meetup_met<T>(&s.cand[tid], D);
        tr = any != 0 || tr;   // (no termination-reason strings for these tasks)
      }
      if (P.rew) P.rew[e] = r;
      if (P.term) P.term[e] = te;
      if (P.trunc) P.trunc[e] = tr;
      ret = ep_ret0 + (double)r;
      len = ep_len + 1;
      dn = te || tr;
      ep_ret_out = dn ? 0.0 : ret;
      ep_len_out = dn ? 0 : len;
      s.done[lenv] = dn;
    }
    // Episode log (VecRecordEpisodeStatistics, record_episode_statistics.py:155-166):
    // each env appends to its own ring, slot = its logged count mod log_per_env —
    // no atomic (a returned global slot made the finishing waves wait ~µs for it
    // and for all their outstanding stores, and they set the launch's tail).
    if (dn) {
      qs_episode_rec rec;
      rec.ret = ret; rec.len = len; rec.env = (int32_t)genv; rec.seq = total;
      P.log[(size_t)e * P.log_per_env + (unsigned)log_n % (unsigned)P.log_per_env] = rec;
      log_n = log_n + 1;
    }
    if (P.reasons && valid) P.reasons[a] = kMarl ? 0 : bits;
    step_counter += S;   // BaseAviary.py:382
    __syncthreads();
    done_env = valid && s.done[lenv];
  } else if (P.mode == MODE_RESET_ALL) {
    wait_vm0();
    // qs_reset: every env starts episode 0 (history is zero after qs_reset)
    done_env = valid;
  } else {
    wait_vm0();
    // qs_reset_envs: env.reset() on the masked envs; the obs lists the latest
    // action (ring slot wslot-1) last
    if (total > 0) {   // (no global read here: it would blur the step path's wait counts)
      const int sl = wslot == 0 ? H - 1 : wslot - 1;
      if constexpr (CF != 0) {
#pragma unroll
        for (int r = 0; r < HR; ++r)
#pragma unroll
          for (int k = 0; k < A; ++k) cur_act[k] = r == sl ? hreg[r][k] : cur_act[k];
      } else {
#pragma unroll
        for (int k = 0; k < A; ++k) cur_act[k] = hist_at(sl, k);
      }
    }
    done_env = valid && masked;
  }
  // worker.step_env resets on done unless this is a single-env facade
  const bool do_reset = done_env && !(P.mode == MODE_STEP && (P.flags & QS_FLAG_NO_AUTORESET));

  // ---------------- obs writer (BaseRLAviary._computeObs + Spiral extras)
  auto write_obs_row = [&](float* o, int sc) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      o[i] = (float)pos[i]; o[3 + i] = (float)rpy[i]; o[6 + i] = (float)vel[i]; o[9 + i] = (float)angv[i];
    }
    // history, oldest first: ring slots base .. base+H-2 (mod H), then this
    // step's action (BaseRLAviary.py:317-318)
    const int base = P.mode == MODE_STEP ? wslot + 1 : wslot;
    if constexpr (CF != 0) {   // register ring: slot sl goes to column (sl - base) mod H
#pragma unroll
      for (int sl = 0; sl < HR; ++sl) {
        int col = sl - base;
        col += col < 0 ? HR : 0;
        if (col != HR - 1) {
#pragma unroll
          for (int k = 0; k < A; ++k) o[12 + col * A + k] = hreg[sl][k];
        }
      }
    } else {
      int sl = base >= H ? base - H : base;
      for (int i = 0; i < H - 1; ++i) {
#pragma unroll
        for (int k = 0; k < A; ++k) o[12 + i * A + k] = hist_at(sl, k);
        if (++sl == H) sl = 0;
      }
    }
#pragma unroll
    for (int k = 0; k < A; ++k) o[12 + (H - 1) * A + k] = cur_act[k];   // newest = this step's action
    if constexpr (kSpiral) {
      T t = T((double)sc / (double)P.pyb_freq);
      T ph = P.sp_OMEGA * t + T(2 * M_PI) * T(d) / T(D);
      T sn = F::sin_(ph), cs = F::cos_(ph);
      T prx = P.sp_cx + P.sp_R * cs, pry = P.sp_cy + P.sp_R * sn, prz = T(0.3) + P.sp_VZ * t;
      T vrx = -P.sp_R * P.sp_OMEGA * sn, vry = P.sp_R * P.sp_OMEGA * cs, vrz = P.sp_VZ;
      float* x = o + 12 + H * A;
      x[0] = (float)(prx - pos[0]); x[1] = (float)(pry - pos[1]); x[2] = (float)(prz - pos[2]);
      x[3] = (float)(vrx - q[0]); x[4] = (float)(vry - q[1]); x[5] = (float)(vrz - q[2]);
      x[6] = (float)sn; x[7] = (float)cs;
      x[8] = (float)vrx; x[9] = (float)vry; x[10] = (float)vrz;
    }
  };

  QS_STAMP(4);
  if (valid && done_env && P.mode == MODE_STEP && P.tobs) write_obs_row(P.tobs + (size_t)a * O, obs_sc);

  // ---------------- auto-reset (worker.step_env → env.reset)
  s.any = 0;
  __syncthreads();
  if (do_reset && d == 0) s.any = 1;
  __syncthreads();
  if (s.any) {
    if (d == 0 && lenv < P.EPB) s.need[lenv] = do_reset ? 1 : 0;
    if (P.mode != MODE_RESET_ALL && do_reset) episode += 1;
    T init[3] = {orig[0], orig[1], orig[2]};
    if constexpr (kHover) {
      if (P.reject_free) {   // workgroup-uniform: no pair test, no barriers
        if (do_reset && !qs_dev::kNoResetDraw)
          reset_candidate(P, orig, d, 0u, genv, (uint32_t)episode, init[0], init[1], init[2]);
      } else {
        // The next episode's first accepted try, when reset_search_kernel's
        // precompute has found it ahead of time (reset_pre, tagged with this episode)
        const bool pre_ok = P.reset_pre && P.mode != MODE_RESET_ALL && do_reset && pre0 < 0 &&
                            pre_tag_is(pre0, (uint32_t)episode);
        if (pre_ok) reset_candidate(P, orig, d, (uint32_t)pre0 & 0xffffffu, genv, (uint32_t)episode, init[0], init[1], init[2]);
        // Phase 1: every other group tries index 0 for its own env.
        if (tid < P.EPB) { s.reject[tid] = 0; s.win_try[tid] = 0; }
        __syncthreads();
        if (!qs_dev::kNoResetDraw)
          eval_candidate(P, s, orig, lenv, d, 0u, genv, (uint32_t)episode, do_reset && !pre_ok, pre_ok ? nullptr : init);
        if (d == 0 && do_reset && s.reject[lenv] == 0) s.need[lenv] = 0;
        if (tid == 0) s.qcount = 0;
        __syncthreads();
        if (P.reset_queue) {
          // deferred: reset_search_kernel (next launch, same stream) finds the first
          // accepted try and rewrites the env's position, target and obs; try 0
          // stands in until then.  One returning atomic per
          // workgroup reserves its slots (a per-env one serialised the rejected
          // envs of a workgroup behind ~1 µs round trips each).
          int local = -1;
          if (d == 0 && lenv < P.EPB && s.need[lenv]) local = atomicAdd(&s.qcount, 1);
          __syncthreads();
          if (tid == 0 && s.qcount) s.qbase = atomicAdd(&P.reset_queue[0], s.qcount);
          __syncthreads();
          if (local >= 0) {
            const int slot = s.qbase + local;
            // claim word {chunks claimed, best try none}, env id, gang 0.  The
            // precomputed search rejected tries [0, 256·pre_c): the claims start at
            // the chunk (tries 1 + 256k … 256k + 256) that holds try 256·pre_c
            const int pre_c = pre0 >= 0 && pre_tag_is(pre0, (uint32_t)episode) ? (pre0 & 0xffffff) : 0;
            const int k0 = pre_c > 0 ? pre_c - 1 : 0;
            *reinterpret_cast<int4*>(P.reset_queue + kRqLine * (1 + slot)) =
                make_int4(k0, kResetNoneDev, (int)(blockIdx.x * P.EPB + lenv), 0);
            s.need[lenv] = 0;
          }
          __syncthreads();
        }
        // Phase 2 (in-kernel search): for each still-rejected env, all groups
        // search in parallel, tries base+g; the smallest accepted index wins
        // (= sequential order).
        for (int k = 0; k < P.EPB; ++k) {
          if (!s.need[k]) continue;   // block-uniform (LDS)
          const int ek = blockIdx.x * P.EPB + k;
          const uint32_t genv_k = (uint32_t)(P.env_offset + ek);
          // episode number of env k lives in its drone-0 thread; broadcast via LDS
          __syncthreads();
          if (tid == k * D) s.ep_bcast = (uint32_t)episode;
          __syncthreads();
          const uint32_t epk = s.ep_bcast;
          uint32_t base = 1;
          for (;;) {
            if (tid < P.EPB) s.reject[tid] = 0;
            if (tid == 0) s.win_group = 1 << 30;
            __syncthreads();
            const bool act_ = lenv < P.EPB && base + (uint32_t)lenv < kMaxResetTries;   // tries [0, cap)
            eval_candidate(P, s, orig, lenv, d, base + (uint32_t)lenv, genv_k, epk, act_);
            if (act_ && d == 0 && s.reject[lenv] == 0) atomicMin(&s.win_group, lenv);
            __syncthreads();
            if (s.win_group < (1 << 30) || base + P.EPB >= kMaxResetTries) {
              if (tid == 0) {
                if (s.win_group < (1 << 30)) s.win_try[k] = base + (uint32_t)s.win_group;
                else { s.win_try[k] = 0; atomicExch(P.err, 1); }
              }
              __syncthreads();
              break;
            }
            base += (uint32_t)P.EPB;
          }
          if (tid == 0) s.need[k] = 2;   // resolved by phase 2 (win_try holds the index)
          __syncthreads();
        }
        // try 0 accepted (the usual case): its draw is already in init (one Philox
        // per drone less on the reset path, which sets the launch's tail)
        if (do_reset && s.need[lenv] == 2)
          reset_candidate(P, orig, d, s.win_try[lenv], genv, (uint32_t)episode, init[0], init[1], init[2]);
      }
    } else {
      if (do_reset) { init[0] = orig[0]; init[1] = orig[1]; init[2] = orig[2]; }
    }
    if (do_reset) {
      // BaseAviary._housekeeping (BaseAviary.py:458-477): PID state and the
      // action history are NOT reset (reference quirk).
#pragma unroll
      for (int i = 0; i < 3; ++i) { pos[i] = init[i]; vel[i] = 0; w[i] = 0; rpy[i] = 0; angv[i] = 0; }
      q[0] = q[1] = q[2] = 0; q[3] = 1;
#pragma unroll
      for (int m = 0; m < 4; ++m) lrpm[m] = 0;
      tgt[0] = init[0]; tgt[1] = init[1]; tgt[2] = init[2] + T(1.0 / (double)(d + 1));   // MH:106
      step_counter = 0;
      obs_sc = 0;
    }
  }

  QS_STAMP(5);
  // ---------------- obs output
  if (P.obs) {
    if (P.mode == MODE_RESET_MASK) {
      if (valid && do_reset) write_obs_row(P.obs + (size_t)a * O, obs_sc);
    } else {
      // The block's obs rows are one contiguous span of HBM: build them in LDS
      // and store the span with 16-byte coalesced stores (a per-lane row store
      // touches 64 lines per wave instruction and doubled the write traffic).
      const int nvalid = [&] { const int e0 = blockIdx.x * P.EPB; return min(P.EPB, P.E - e0) * D; }();
      float* const blk = P.obs + (size_t)blockIdx.x * P.EPB * D * O;
      for (int p0 = 0; p0 < nvalid; p0 += P.stage_rows) {   // block-uniform
        const int p1 = min(nvalid, p0 + P.stage_rows);
        if (tid >= p0 && tid < p1) write_obs_row(stage + (tid - p0) * O, obs_sc);
        __syncthreads();
        float* const g = blk + (size_t)p0 * O;                 // span start
        const int n = (p1 - p0) * O;                          // floats in the span
        const int head = min(n, (int)((4 - (((uintptr_t)g >> 2) & 3)) & 3));   // floats to 16-B alignment
        if (tid < head) nt_store(g + tid, stage[tid]);
        const int nv = (n - head) >> 2;
        if ((head & 3) == 0) {
          for (int i = tid; i < nv; i += kBlock)
            obs_store4(reinterpret_cast<float4*>(g + 4 * i), *reinterpret_cast<const float4*>(stage + 4 * i));
        } else {
          for (int i = tid; i < nv; i += kBlock) {
            const float* src = stage + head + 4 * i;
            obs_store4(reinterpret_cast<float4*>(g + head + 4 * i), make_float4(src[0], src[1], src[2], src[3]));
          }
        }
        for (int i = head + 4 * nv + tid; i < n; i += kBlock) nt_store(g + i, stage[i]);
        __syncthreads();
      }
    }
  }
  QS_STAMP(6);
  // ---------------- per-env records: staged in LDS, stored as one span
  if (valid && d == 0) {
    int32_t* r = &s.rec[lenv * kEnvRec];
    const unsigned long long rb = __builtin_bit_cast(unsigned long long, ep_ret_out);
    r[QS_E_STEP_COUNTER] = step_counter; r[QS_E_EPISODE] = episode; r[QS_E_TOTAL_STEPS] = total;
    r[QS_E_EP_LEN] = ep_len_out;
    r[kEnvRetWord] = (int32_t)(unsigned)rb; r[kEnvRetWord + 1] = (int32_t)(unsigned)(rb >> 32);
    // (a reset voids the precomputed word by its tag: the next search is for
    // the episode after this one)
    r[kEnvLogWord] = log_n; r[kEnvPreWord] = 0;
  }
  __syncthreads();
  {
    const int nrec = min(P.EPB, P.E - (int)blockIdx.x * P.EPB) * kEnvRec;
    int32_t* const g = P.env + (size_t)blockIdx.x * P.EPB * kEnvRec;
    for (int i = tid; i < nrec; i += kBlock) __builtin_nontemporal_store(s.rec[i], g + i);
  }
  if (!valid) return;

  // ---------------- store state of the envs that (auto-)reset
  if (do_reset) {
    store_kin();
    if constexpr (kHover) {
#pragma unroll
      for (int i = 0; i < 3; ++i) SA.st(QS_F_TARGET + i, tgt[i]);
    }
  }
}


// ------------------------------------------------- deferred reset search
// MultiHoverAviary.reset's rejection loop (MH:83-102) for the envs the step
// kernel queued (no precomputed try, and try 0 rejected; rare once the
// precomputed resets below run).  Per queue slot (kRq* above): a claim word
// holding the number of chunks claimed (low half) and the best accepted try
// so far (high half), the env id and the number of workgroups searching the
// slot (gang), on a 128-B line of its own, so one returning 64-bit atomicAdd
// both claims a chunk and reads the best try.  The step kernel initialises a
// slot when it queues an env.
//
// An env's tries are cut into chunks of kResetChunk (chunk c holds tries
// 1 + kResetChunk·c + t, thread t; the claims start past the tries the
// precomputed search already rejected).  Workgroup b works on slot b mod n (so up
// to kResetGang workgroups share an env; with more envs than workgroups, slots
// b, b + G, … in turn): it claims the slot's next chunk (issued one chunk
// ahead, so the atomic's round trip runs under the Philox work), tests it,
// publishes its smallest accepted try (rq_publish), and leaves once its
// claimed chunk starts above the best try (every chunk below it is claimed)
// or above the cap.  The last workgroup to leave writes the env (position,
// target, obs row): by then every chunk below the best try has been tested,
// so the best try is the first accepted try of the sequential loop.
// (Workgroups that scanned for open envs to help needed coherent reads of
// other XCDs' atomics — uncached memory — and piled onto single envs: 1 000
// claimants on one line cost ~50 µs; the precomputed resets made the queue
// small instead.)  D <= kResetMaxD.
constexpr int kResetBlock = 256;
constexpr int kResetChunk = kResetBlock;   // tries per chunk, one per thread
constexpr int kResetMaxD = 8;
#ifndef QS_RESET_GANG   // (dev builds may override the three search sizes)
#define QS_RESET_GANG 32
#endif
constexpr int kResetGang = QS_RESET_GANG;
constexpr int kResetNone = kResetNoneDev;  // "no accepted try yet"

__device__ __forceinline__ unsigned long long rq_claim(unsigned long long* w) {
  return atomicAdd(w, 1ull);   // low half: chunks claimed; high half: best try
}
// Publishes accepted try t: one 64-bit atomicMin.  The word becomes {win t,
// chunks claimed 0x7fffffff} when t is the best so far: every chunk below t's
// chunk was claimed before t's, so no chunk needs claiming any more, and every
// later claim returns a base far above t (a compare-and-swap that kept the
// count lost to the ~16 claimants' traffic on the word and starved).
__device__ __forceinline__ void rq_publish(unsigned long long* w, int t) {
  atomicMin(w, ((unsigned long long)(unsigned)t << 32) | 0x7fffffffull);
}

// One chunk of an env's tries, [base, base + kResetChunk), one per thread:
// returns the smallest accepted try of the chunk (kResetNone if none;
// workgroup-uniform) — with the chunks taken in order, the sequential loop's
// first accepted try.  Drones 0-1 and their pair test first; the tries that
// pass it (18.6 % for C2's layout) are compacted into the first lanes (their
// two draws kept in LDS) and draw drones 2.. there, so a try the first pair
// rejects costs two Philox draws instead of D: every wave kept drawing all D
// while any of its 64 tries was alive, which is nearly always.  The accept
// test is the same conjunction of z and pair tests in either order.  claim_in
// (thread 0's value) comes back to every thread in *claim_out after the
// chunk, for the queue loop's claim issued one chunk ahead.
template <class T> struct ResetLds {
  T p[kResetChunk][6];   // the compacted tries' drone 0-1 positions
  int t[kResetChunk];
  int cnt, win;
  unsigned long long claim;
};
template <class T>
__device__ int reset_chunk(const Params<T>& P, const T (&orig)[kResetMaxD][3], uint32_t base, uint32_t genv,
                           uint32_t ep, ResetLds<T>& L, unsigned long long claim_in = 0,
                           unsigned long long* claim_out = nullptr) {
  const int D = P.D, tid = threadIdx.x;
  const uint32_t t = base + (uint32_t)tid;
  if (tid == 0) { L.cnt = 0; L.win = kResetNone; }
  bool ok = t < kMaxResetTries;
  T a[3] = {T(0), T(0), T(0)}, b[3] = {T(0), T(0), T(0)};
  if (ok) {
    reset_candidate(P, orig[0], 0, t, genv, ep, a[0], a[1], a[2]);
    if (a[2] < T(0.1)) ok = false;
  }
  if (D > 1 && ok) {
    reset_candidate(P, orig[1], 1, t, genv, ep, b[0], b[1], b[2]);
    if (b[2] < T(0.1) || too_close(a[0], a[1], a[2], b[0], b[1], b[2])) ok = false;
  }
  __syncthreads();   // L.cnt / L.win initialised
  if (D <= 2) {
    if (ok) atomicMin(&L.win, (int)t);
  } else {
    // wave-aggregated slots: one LDS add per wave, the lanes' ranks from mbcnt
    const unsigned long long m = __ballot(ok);
    const int lane = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    int wb = 0;
    if ((tid & 63) == 0 && m) wb = atomicAdd(&L.cnt, __popcll(m));
    wb = __shfl(wb, 0);
    if (ok) {
      const int s = wb + lane;
      L.t[s] = (int)t;
      L.p[s][0] = a[0]; L.p[s][1] = a[1]; L.p[s][2] = a[2];
      L.p[s][3] = b[0]; L.p[s][4] = b[1]; L.p[s][5] = b[2];
    }
    __syncthreads();
    if (tid < L.cnt) {
      const uint32_t tt = (uint32_t)L.t[tid];
      T px[kResetMaxD], py[kResetMaxD], pz[kResetMaxD];
      px[0] = L.p[tid][0]; py[0] = L.p[tid][1]; pz[0] = L.p[tid][2];
      px[1] = L.p[tid][3]; py[1] = L.p[tid][4]; pz[1] = L.p[tid][5];
      bool ok2 = true;
#pragma unroll
      for (int d = 2; d < kResetMaxD; ++d) {
        if (d < D && ok2) {
          reset_candidate(P, orig[d], d, tt, genv, ep, px[d], py[d], pz[d]);
          if (pz[d] < T(0.1)) ok2 = false;
#pragma unroll
          for (int i = 0; i < d; ++i)
            if (too_close(px[i], py[i], pz[i], px[d], py[d], pz[d])) ok2 = false;
        }
      }
      if (ok2) atomicMin(&L.win, (int)tt);
    }
  }
  if (tid == 0) L.claim = claim_in;
  __syncthreads();
  const int w = L.win;
  if (claim_out) *claim_out = L.claim;
  __syncthreads();   // L is rewritten by the next chunk
  return w;
}

// The precomputed resets: an env's next-episode reset draw depends only on
// (seed, env, episode), so the search for it need not wait for the reset.
// The search launch's workgroups past the queue's, grid-strided over the
// envs, one workgroup at a time: an env whose
// reset_pre word holds no try for its next episode gets kPreChunks chunks of
// 256 tries (chunk c: tries 256·c + t, try 0 included), continuing at the
// word's chunk count when its tag is that episode's; the first accepted try
// goes into the word with kPreFound, and the step kernel that resets the env
// into that episode draws it instead of testing try 0 — the first accepted
// try of MH:83-102, as the queue search finds it.  No atomics, and nothing
// for the step to clear: a reset voids the word by its tag (the search for the
// episode after it starts at chunk 0), so a precompute running beside the step
// could not race it either (measured as a parallel graph branch on a second
// stream: no overlap — 28.1 against 28.8 µs per C2 step serial).
// An env that resets before
// its search ends takes the step kernel's own path (try 0, then the queue,
// whose claims start past the chunks tested here).  (One wave per env, 64
// tries a step: the serial Philox chain of a lone wave made 8 steps cost
// 25 µs a launch.)
#ifndef QS_PRE_CHUNKS
#define QS_PRE_CHUNKS 2
#endif
#ifndef QS_QUEUE_WG
#define QS_QUEUE_WG 256
#endif
constexpr int kPreChunks = QS_PRE_CHUNKS;
constexpr int kQueueWG = QS_QUEUE_WG;   // workgroups of the queue search launch
#ifndef QS_PRE_ENVS
#define QS_PRE_ENVS 1   // measured: 2 / 4 envs per workgroup made C2 23.5 / 26.9 µs per step (1: 22.2)
#endif
constexpr int kPreEnvs = QS_PRE_ENVS;   // envs per precompute workgroup

template <class T>
__device__ __forceinline__ void reset_orig(const Params<T>& P, T (&orig)[kResetMaxD][3]) {
#pragma unroll
  for (int d = 0; d < kResetMaxD; ++d)
#pragma unroll
    for (int k = 0; k < 3; ++k) orig[d][k] = d < P.D ? P.orig_xyz[d * 3 + k] : T(0);
}

template <class T>
__device__ void reset_precompute(const Params<T>& P, ResetLds<T>& L, int first, int stride) {
  const int tid = threadIdx.x;
  T orig[kResetMaxD][3];
  reset_orig(P, orig);
  // kPreEnvs envs per workgroup (first + j·stride), their episode and word
  // loaded together (one env per workgroup measured fastest: the launch is
  // bound by its slowest workgroup's chunks, not by the dispatch)
  for (int e0 = first; e0 < P.E; e0 += stride * kPreEnvs) {   // workgroup-uniform
    uint32_t ep[kPreEnvs];
    int32_t w0[kPreEnvs];
#pragma unroll
    for (int j = 0; j < kPreEnvs; ++j) {
      const int e = e0 + j * stride;
      ep[j] = e < P.E ? (uint32_t)P.env[(size_t)e * kEnvRec + QS_E_EPISODE] + 1u : 0u;
      w0[j] = e < P.E ? P.reset_pre[e] : 0;
    }
#pragma unroll
    for (int j = 0; j < kPreEnvs; ++j) {
      const int e = e0 + j * stride;
      const bool mine = pre_tag_is(w0[j], ep[j]);   // else void: the search starts at chunk 0
      if (e >= P.E || (mine && w0[j] < 0)) continue;   // found already
      int c = mine ? (w0[j] & 0xffffff) : 0;
      const uint32_t genv = (uint32_t)(P.env_offset + e), tag = (ep[j] & 0x7fu) << 24;
      int found = kResetNone;
      for (int k = 0; k < kPreChunks; ++k, ++c) {
        if ((uint32_t)c * kResetChunk >= kMaxResetTries) break;   // none below the cap: the step's own path flags it
        found = reset_chunk(P, orig, (uint32_t)c * kResetChunk, genv, ep[j], L);
        if (found != kResetNone) break;
      }
      if (tid == 0)
        P.reset_pre[e] = (int32_t)(found != kResetNone ? kPreFound | tag | (uint32_t)found : tag | (uint32_t)c);
    }
  }
}

// The search launch: its first kQueueWG workgroups serve the queue (G of
// them), the others precompute (with reset_pre), so neither waits for the other.
template <class T>
__global__ void __launch_bounds__(kResetBlock) reset_search_kernel(Params<T> P) {
  __shared__ ResetLds<T> L;
  __shared__ unsigned long long s_claim;
  __shared__ int s_fin;
  const int G = P.reset_pre ? min((int)gridDim.x, kQueueWG) : (int)gridDim.x;
  if ((int)blockIdx.x >= G) {
    reset_precompute(P, L, (int)blockIdx.x - G, (int)gridDim.x - G);
    return;
  }
  int* const rq = P.reset_queue;
  const int n = rq[0];
  const int D = P.D;
  const int tid = threadIdx.x;
  if (n == 0) return;   // nothing queued: the usual step
  T orig[kResetMaxD][3];
  reset_orig(P, orig);
  const int home = (int)(blockIdx.x % (unsigned)n);
  // More envs than queue workgroups (a reset of every env): workgroup b takes
  // envs b, b + G, b + 2G, … in turn.
  int idx = (int)blockIdx.x < min(G, n * kResetGang) ? home : -1;
  QS_RS_BEGIN();
  while (idx >= 0) {
    int* const r = rq + kRqLine * (1 + idx);
    int* const gang = r + kRqGang;
    unsigned long long* const cwp = reinterpret_cast<unsigned long long*>(r);
    const int e = r[kRqEnv];
    const uint32_t genv = (uint32_t)(P.env_offset + e);
    const uint32_t episode = (uint32_t)P.env[(size_t)e * kEnvRec + QS_E_EPISODE];
    if (tid == 0) {
      // returning: the gang count is raised before the claim is made.  A slot
      // already written (gang >= kRqDone) is left at once: a claim that cannot
      // be below its best try stands in
      const int g0 = atomicAdd(gang, 1);
      const unsigned long long c0 = rq_claim(cwp);   // in flight with the gang add (a claim
      s_claim = g0 >= kRqDone ? 0x7fffffffull : c0;  // after the env closed is above its best try)
    }
    __syncthreads();
    unsigned long long cw = s_claim;
    __syncthreads();
    QS_RS_JOIN(1 + (long long)(cw & 0xffffffffull) * kResetChunk > (long long)(int)(cw >> 32));
    int found = kResetNone;   // this workgroup's accepted try (workgroup-uniform)
    for (;;) {
      const long long base = 1 + (long long)(cw & 0xffffffffull) * kResetChunk;   // workgroup-uniform
      if (base > (long long)min((int)(cw >> 32), found)) break;
      if (base >= (long long)kMaxResetTries) break;
      unsigned long long cw_next = 0;
      if (tid == 0) cw_next = rq_claim(cwp);   // one chunk ahead: used after this chunk's tries
      const int w = reset_chunk(P, orig, (uint32_t)base, genv, episode, L, cw_next, &cw);
      if (w != kResetNone) {
        found = w;       // the claim ahead is above w: the loop test leaves
        if (tid == 0) rq_publish(cwp, w);
      }
      QS_RS_CHUNK(w != kResetNone);
    }
    // The last workgroup to leave writes the env: every leave happens once the
    // env's claims have passed its best try (or the cap), and a workgroup leaves
    // only after testing its chunks and publishing its accepted try, so at gang
    // 0 every chunk below the best try has been tested.  The compare-and-swap to
    // kRqDone makes the write exclusive (a late joiner, raising gang again after
    // 1 -> 0, leaves and takes the turn instead).
    if (tid == 0) {
      s_fin = 0;
      // the publish above is performed before the leave (returning atomics below)
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (atomicSub(gang, 1) == 1 && atomicCAS(gang, 0, kRqDone) == 0) {
        s_fin = 1;
        s_claim = atomicAdd(cwp, 0ull);   // read-modify-write: the coherent best try
      }
    }
    __syncthreads();
    if (s_fin) {
      const int wv = (int)(s_claim >> 32);
      // no accepted try below the cap: flag the error and keep try 0, as the
      // in-kernel search does
      const uint32_t win = wv == kResetNone ? 0u : (uint32_t)wv;
      if (tid < D) {
        T od[3] = {P.orig_xyz[tid * 3 + 0], P.orig_xyz[tid * 3 + 1], P.orig_xyz[tid * 3 + 2]};
        T ix, iy, iz;
        reset_candidate(P, od, tid, win, genv, episode, ix, iy, iz);
        const size_t a = (size_t)e * D + tid, N = (size_t)P.N;
        P.st[(QS_F_POS + 0) * N + a] = ix; P.st[(QS_F_POS + 1) * N + a] = iy; P.st[(QS_F_POS + 2) * N + a] = iz;
        P.st[(QS_F_TARGET + 0) * N + a] = ix; P.st[(QS_F_TARGET + 1) * N + a] = iy;
        P.st[(QS_F_TARGET + 2) * N + a] = iz + T(1.0 / (double)(tid + 1));   // MH:106
        if (P.obs) {
          float* o = P.obs + a * (size_t)P.O;
          o[0] = (float)ix; o[1] = (float)iy; o[2] = (float)iz;
        }
      }
      if (tid == 0) {
        if (wv == kResetNone) atomicExch(P.err, 1);
        // the last env written empties the queue (one same-address atomic per
        // queued env); a workgroup that reads the count after that has nothing to do
        if (atomicAdd(&rq[1], 1) == n - 1) { rq[0] = 0; rq[1] = 0; }
      }
    }
    __syncthreads();   // s_fin / s_claim are rewritten by the next slot
    idx = idx + G < n ? idx + G : -1;
    QS_RS_PICK();
  }
  QS_RS_END(n);
}

}  // namespace qs
