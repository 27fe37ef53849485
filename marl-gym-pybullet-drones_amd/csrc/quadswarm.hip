// quadswarm.hip — host side of the MI355X quadrotor-swarm step: the C-ABI of
// include/quadswarm.h (handle, state buffers, launches).  The device code is
// csrc/step_kernel.h; the kernels are instantiated per task family in
// step_mh.hip / step_spiral.hip / step_generic.hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <string>
#include <vector>
#include <new>

#include "quadswarm.h"
#include "step_launch.h"

namespace qs {
// Calibration kernel: dword per lane, grid-stride (MI355X_MICROARCH §HBM).
__global__ void calib_copy_kernel(float* __restrict__ dst, const float* __restrict__ src, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = src[i];
}

// ------------------------------------------------------------ episode log query
// qs_episode_log selects the newest `cap` records of the per-env rings on the
// device, so that O(cap) records — not the E·R ring slots — cross to the host.
// An env's ring holds its last min(n, R) episodes (n = its logged count) in
// slots (n − min(n, R)) … (n − 1) mod R.
constexpr int kLogBins = 4096;   // seq-distance bins below the newest seq (the last one: ≥ 4095)
struct LogWork {
  unsigned long long total;      // Σ_e n_e
  long long maxseq;              // newest seq over every ring
  unsigned int nsel;             // records compacted by log_select_kernel
  unsigned int pad;
  unsigned int hist[kLogBins];   // live ring slots per (maxseq − seq) bin
};

__device__ __forceinline__ long long env_logged(const int32_t* env, int e) {
  return env[(size_t)e * kEnvRec + kEnvLogWord];
}

// total and newest seq: block sums / maxima, then one global atomic per block
__global__ void __launch_bounds__(256) log_scan_kernel(const int32_t* __restrict__ env,
                                                       const qs_episode_rec* __restrict__ log, int E, int R,
                                                       LogWork* w) {
  __shared__ unsigned long long ssum[4];
  __shared__ long long smax[4];
  const int e = blockIdx.x * 256 + threadIdx.x;
  unsigned long long n = 0;
  long long mx = -1;
  if (e < E) {
    const long long c = env_logged(env, e);
    n = (unsigned long long)c;
    // every live slot (seq grows along a ring, but qs_state_io may rewrite the counters)
    for (long long i = c > R ? c - R : 0; i < c; ++i) mx = max(mx, log[(size_t)e * R + (size_t)(i % R)].seq);
  }
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o, 64);
    mx = max(mx, __shfl_xor(mx, o, 64));
  }
  if ((threadIdx.x & 63) == 0) { ssum[threadIdx.x >> 6] = n; smax[threadIdx.x >> 6] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = ssum[0] + ssum[1] + ssum[2] + ssum[3];
    const long long m = max(max(smax[0], smax[1]), max(smax[2], smax[3]));
    if (t) atomicAdd(&w->total, t);
    if (m >= 0) atomicMax(&w->maxseq, m);
  }
}

// histogram of (maxseq − seq) over the live ring slots: LDS bins, only the
// non-empty ones flushed
__global__ void __launch_bounds__(256) log_hist_kernel(const int32_t* __restrict__ env,
                                                       const qs_episode_rec* __restrict__ log, int E, int R,
                                                       LogWork* w) {
  __shared__ unsigned int h[kLogBins];
  for (int b = threadIdx.x; b < kLogBins; b += 256) h[b] = 0;
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;
  const long long top = w->maxseq;
  if (e < E) {
    const long long n = env_logged(env, e);
    for (long long i = n > R ? n - R : 0; i < n; ++i) {
      const long long d = max(0LL, top - log[(size_t)e * R + (size_t)(i % R)].seq);
      atomicAdd(&h[d < kLogBins - 1 ? (int)d : kLogBins - 1], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kLogBins; b += 256)
    if (h[b]) atomicAdd(&w->hist[b], h[b]);
}

// every live record with seq ≥ thr, in no particular order (the host orders them)
__global__ void __launch_bounds__(256) log_select_kernel(const int32_t* __restrict__ env,
                                                         const qs_episode_rec* __restrict__ log, int E, int R,
                                                         long long thr, qs_episode_rec* __restrict__ out,
                                                         unsigned int out_cap, LogWork* w) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const long long n = env_logged(env, e);
  for (long long i = n > R ? n - R : 0; i < n; ++i) {
    const qs_episode_rec r = log[(size_t)e * R + (size_t)(i % R)];
    if (r.seq < thr) continue;
    const unsigned int k = atomicAdd(&w->nsel, 1u);
    if (k < out_cap) out[k] = r;
  }
}

}  // namespace qs

// ===========================================================================
// Host side: the C-ABI.
// ===========================================================================
namespace {
thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }
#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return fail(QS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// cf2x.urdf + BaseAviary.py:117-128 (same values as the oracle's Consts).
struct HostConsts {
  double G = 9.8, M = 0.027, L = 0.0397, T2W = 2.25, IXX = 1.4e-5, IYY = 1.4e-5, IZZ = 2.17e-5;
  double KF = 3.16e-10, KM = 7.94e-12, COLL_H = 0.025, COLL_Z_OFF = 0.0, MAX_SPEED_KMH = 30.0;
  double GND_EFF_COEFF = 11.36859, PROP_RADIUS = 2.31348e-2, DRAG_XY = 9.1785e-7, DRAG_Z = 10.311e-7;
  double DW1 = 2267.18, DW2 = 0.16, DW3 = -0.11;
};
}  // namespace

struct qs_handle {
  qs_spec spec;
  qs_dims dims;
  int device = 0;
  void* st = nullptr;          // agent SoA (real)
  int32_t* env = nullptr;      // per-env records [E][qs::kEnvRec] (counters + episode return)
  float* hist = nullptr;
  void* orig = nullptr;        // [D][3] real
  qs_episode_rec* log = nullptr;
  int log_per_env = 0;
  int* err = nullptr;
  unsigned long long* stamps = nullptr;   // dev-only (QS_STAMPS)
  int* rq = nullptr;            // deferred reset-search queue (header + one 128-B record per env), MultiHover layouts that can reject
  int32_t* rpre = nullptr;      // [E] each env's precomputed next-episode reset search (qs::kPreFound)
  bool reject_free = false;     // MultiHover layout whose reset draws can never be rejected
  int num_cu = 256;             // compute units of the device (LDS residency plan)
  qs::LogWork* logw = nullptr;  // qs_episode_log's device scratch
  qs_episode_rec* log_sel = nullptr;   // its compacted records (log_sel_cap slots, grown on demand)
  size_t log_sel_cap = 0;
  uint64_t seed = 0;
  bool reset_done = false;
  std::vector<double> orig_host;
};

// Envs per one-wave workgroup: ⌊64/D⌋, a launch parameter (P.EPB).  A dev build
// may halve it while the grid holds fewer than kEpbWaves waves per SIMD (at
// most QS_EPB_HALVINGS times), to overlap more waves' latency chains on an
// under-filled grid (Spiral C4: 683 waves of 12 envs for 1 024 SIMDs) — but
// every wave pays the same load → PID → substeps → reward → store chain, and
// one halving made C4 11.6 → 18.2 µs (as round 2's probe found), so the
// default is none.  Results do not depend on it: every per-env quantity is
// formed inside the env's own lanes.
#ifndef QS_EPB_HALVINGS
#define QS_EPB_HALVINGS 0   // measured: one halving made Spiral C4 11.6 -> 18.2 µs; dev builds probe it
#endif
#ifndef QS_EPB_WAVES
#define QS_EPB_WAVES 2   // (dev builds: the waves per SIMD below which a halving applies)
#endif
static constexpr int kEpbWaves = QS_EPB_WAVES;
static int envs_per_wave(const qs_handle* h) {
  const int E = h->spec.num_envs, simds = 4 * h->num_cu;
  int epb = qs::kBlock / h->spec.num_drones;
  for (int k = 0; k < QS_EPB_HALVINGS && epb > 1 && (E + epb - 1) / epb < kEpbWaves * simds; ++k) epb = (epb + 1) / 2;
  return epb;
}

template <class T> static void fill_params(const qs_handle* h, qs::Params<T>& P) {
  const qs_spec& s = h->spec;
  std::memset(&P, 0, sizeof(P));
  P.E = s.num_envs; P.D = s.num_drones; P.N = h->dims.num_agents; P.O = h->dims.obs_dim;
  P.H = h->dims.hist_len; P.S = h->dims.substeps;
  P.EPB = envs_per_wave(h);
  P.aux = s.aux_forces; P.flags = s.flags; P.pyb_freq = s.pyb_freq; P.task = s.task;
  P.ep_len_sec = s.episode_len_sec;
  P.k0 = (uint32_t)h->seed; P.k1 = (uint32_t)(h->seed >> 32);
  P.env_offset = s.env_offset;
  P.reset_queue = h->rq;
  P.reset_pre = h->rpre;
  P.reject_free = h->reject_free ? 1 : 0;
  const double dt = 1.0 / s.pyb_freq;
  P.dt = T(dt); P.hdt = T(dt / 2); P.hdt2 = T((dt / 2) * (dt / 2)); P.ctrl_dt = T(1.0 / s.ctrl_freq); P.ctrl_hz = T(s.ctrl_freq);
  P.sp_R = T(s.spiral_radius); P.sp_OMEGA = T(2 * M_PI / s.spiral_period); P.sp_VZ = T(s.height_rate);
  P.sp_cx = T(s.target_center[0]); P.sp_cy = T(s.target_center[1]); P.sp_cz = T(s.target_center[2]);
  P.st = (T*)h->st; P.env = h->env; P.hist = h->hist; P.orig_xyz = (const T*)h->orig;
  P.log = h->log; P.log_per_env = h->log_per_env; P.err = h->err;
  P.stamps = h->stamps;
}

// LDS per workgroup: the history prefetch image plus obs rows staged per pass.
// The staging is sized so that the launch's workgroups are resident at once:
// `resident` = ⌈grid / CUs⌉ of them must share a CU's 160 KB (else the grid runs
// in rounds, each paying the whole per-wave latency again: Spiral C4's 683
// one-wave workgroups at 61 KB each ran as 512 + 171, 17.5 µs → 12.0 µs).  When
// the whole grid cannot be resident even with fewer staged rows (MultiHover VEL:
// 15 KB of history per workgroup), full staging is kept — more passes of fewer
// rows cost more than the partial residency returns (C3-VEL 22.3 → 26.0 µs).
static constexpr size_t kLdsBytes = 160 * 1024, kLdsStatic = 8192, kLdsGrain = 512, kStageBudget = 48 * 1024;
static int lds_plan(const qs_dims& d, int epb, int resident, int* stage_rows, size_t* bytes) {
  const size_t hist = (size_t)d.hist_len * qs::kBlock * d.act_dim * sizeof(float);
  const size_t row = (size_t)d.obs_dim * sizeof(float);
  if (hist + row + kLdsStatic > kLdsBytes) return QS_E_INVALID;
  const int rows = epb * d.num_drones;
  size_t per = kLdsBytes / (size_t)std::max(1, std::min(resident, 32));   // a workgroup's share at full residency
  if (per < kLdsStatic + kLdsGrain + hist + row) per = kLdsBytes;          // unreachable: plain staging
  const size_t budget = std::min(kStageBudget, per - kLdsStatic - kLdsGrain - hist);
  *stage_rows = (int)std::max<size_t>(1, std::min<size_t>(rows, budget / row));
  *bytes = hist + (size_t)*stage_rows * row;
  return QS_OK;
}

template <class T> static int launch(qs_handle* h, qs::Params<T>& P, hipStream_t st) {
  const int grid = (P.E + P.EPB - 1) / P.EPB;
  size_t lds = 0;
  if (lds_plan(h->dims, P.EPB, (grid + h->num_cu - 1) / h->num_cu, &P.stage_rows, &lds) != QS_OK)
    return fail(QS_E_INVALID, "launch: action history does not fit in LDS (ctrl_freq too high)");
  const qs_spec& s = h->spec;
  bool ok;
  if (s.task == QS_TASK_MULTIHOVER)
    ok = qs::launch_task<T, QS_TASK_MULTIHOVER>(s.act_type, grid, lds, st, P, s.ctrl_freq, s.pyb_freq, s.physics);
  else if (s.task == QS_TASK_SPIRAL)
    ok = qs::launch_task<T, QS_TASK_SPIRAL>(s.act_type, grid, lds, st, P, s.ctrl_freq, s.pyb_freq, s.physics);
  else
    ok = qs::launch_task<T, qs::kTaskMarl>(s.act_type, grid, lds, st, P, s.ctrl_freq, s.pyb_freq, s.physics);
  if (!ok) return fail(QS_E_INVALID, "launch: bad act_type");
  HIP_TRY(hipGetLastError());
  if (P.reset_queue) {   // the envs whose try 0 was rejected (usually none)
    // Workgroups claim chunks of the queued envs' tries dynamically; kQueueWG
    // workgroups for the queue, then one per kPreEnvs envs (up to 4 096 envs,
    // grid-strided beyond) for the precomputed resets
    const int rgrid = qs::kQueueWG + std::min(4096 / qs::kPreEnvs, (P.E + qs::kPreEnvs - 1) / qs::kPreEnvs);
    hipLaunchKernelGGL(qs::reset_search_kernel<T>, dim3(rgrid), dim3(qs::kResetBlock), 0, st, P);
    HIP_TRY(hipGetLastError());
  }
  return QS_OK;
}

// The device code folds the CF2X constants as literals (qs::cf2x); re-derive
// them here from the URDF values exactly as the oracle does and refuse to run
// if any literal is not the correctly rounded value.
static int check_consts() {
  const HostConsts C;
  namespace K = qs::cf2x;
  const bool ok = K::G == C.G && K::M == C.M && K::L == C.L && K::KF == C.KF && K::KM == C.KM &&
                  K::IXX == C.IXX && K::IYY == C.IYY && K::IZZ == C.IZZ &&
                  K::L_SQRT2 == C.L / std::sqrt(2.0) &&
                  K::HOVER_RPM == std::sqrt(C.G * C.M / (4 * C.KF)) &&
                  K::SPEED_LIMIT == 0.03 * C.MAX_SPEED_KMH * (1000.0 / 3600.0) &&
                  K::DRAG_XY == C.DRAG_XY && K::DRAG_Z == C.DRAG_Z && K::GND_COEFF == C.GND_EFF_COEFF &&
                  K::PROP_R == C.PROP_RADIUS && K::DW1 == C.DW1 && K::DW2 == C.DW2 && K::DW3 == C.DW3;
  const double max_rpm = std::sqrt((C.T2W * C.G * C.M) / (4 * C.KF));
  const double max_thrust = 4 * C.KF * max_rpm * max_rpm;
  const double gnd_clip = 0.25 * C.PROP_RADIUS * std::sqrt((15 * max_rpm * max_rpm * C.KF * C.GND_EFF_COEFF) / max_thrust);
  if (!ok || K::GND_CLIP != gnd_clip) return fail(QS_E_INVALID, "qs_create: CF2X device constants disagree with the URDF derivation");
  // CF2P (QS_FLAG_CF2P): cf2p.urdf:12 inertia, props on the body axes at L (cf2p.urdf:42-79)
  using MP = qs::Model<true>;
  const bool okp = MP::IXX == 2.3951e-5 && MP::IYY == 2.3951e-5 && MP::IZZ == 3.2347e-5 && MP::PX[0] == C.L &&
                   MP::PY[1] == C.L && MP::PX[2] == -C.L && MP::PY[3] == -C.L && MP::PX[1] == 0 && MP::PY[0] == 0;
  if (!okp) return fail(QS_E_INVALID, "qs_create: CF2P device constants disagree with cf2p.urdf");
  return QS_OK;
}

extern "C" {

const char* qs_last_error(void) { return g_err.c_str(); }
int qs_abi_version(void) { return QS_ABI_VERSION; }

int qs_create(const qs_spec* spec, int device, qs_handle** out) {
  if (!spec || !out) return fail(QS_E_INVALID, "qs_create: null argument");
  const qs_spec& s = *spec;
  if (s.task < QS_TASK_MULTIHOVER || s.task > QS_TASK_LEADERFOLLOWER) return fail(QS_E_INVALID, "qs_create: bad task");
  if (s.num_drones < 1 || s.num_drones > 64) return fail(QS_E_INVALID, "qs_create: num_drones must be in 1..64");
  if (s.num_envs < 1) return fail(QS_E_INVALID, "qs_create: num_envs must be >= 1");
  if (s.physics != QS_PHYS_DYN && s.physics != QS_PHYS_PYB) return fail(QS_E_INVALID, "qs_create: bad physics");
  if (s.aux_forces & ~7u) return fail(QS_E_INVALID, "qs_create: bad aux_forces");
  if (s.flags & ~(QS_FLAG_NO_AUTORESET | QS_FLAG_INKERNEL_RESET_SEARCH | QS_FLAG_CF2P))
    return fail(QS_E_INVALID, "qs_create: bad flags");
  if (s.pyb_freq <= 0 || s.ctrl_freq <= 0 || s.pyb_freq % s.ctrl_freq)
    return fail(QS_E_INVALID, "qs_create: pyb_freq is not divisible by env_freq");  // BaseAviary.py:79-80
  if (s.ctrl_freq < 2) return fail(QS_E_INVALID, "qs_create: ctrl_freq must be >= 2 (action history length ctrl_freq//2)");
  if (s.precision != 4 && s.precision != 8) return fail(QS_E_INVALID, "qs_create: precision must be 4 or 8");
  if (check_consts() != QS_OK) return QS_E_INVALID;
  if (s.task == QS_TASK_MULTIHOVER && !s.initial_xyzs && s.num_drones >= 6)
    return fail(QS_E_INVALID, "qs_create: MultiHover reset with the default diagonal layout cannot complete for "
                              "D >= 6 (SURVEY §7 hard-2); pass initial_xyzs");
  int A;
  switch (s.act_type) {
    case QS_ACT_RPM: case QS_ACT_VEL: A = 4; break;
    case QS_ACT_PID: A = 3; break;
    case QS_ACT_ONE_D_RPM: case QS_ACT_ONE_D_PID: A = 1; break;
    default: return fail(QS_E_INVALID, "qs_create: bad act_type");
  }
  {
    // The kernels address every buffer through 32-bit buffer-resource ranges and
    // offsets (step_kernel.h: state, history, obs rows, env records): refuse a
    // shard whose largest buffer would not fit below 2^31 bytes instead of
    // letting the offsets wrap.  (C3 at 16 384 envs uses 15 MB.)
    const int64_t Nn = (int64_t)s.num_envs * s.num_drones;
    const int64_t H = s.ctrl_freq / 2;
    const int64_t O = 12 + H * A + (s.task == QS_TASK_SPIRAL ? 11 : 0);
    const int64_t biggest = std::max({(int64_t)QS_AGENT_FIELDS * Nn * s.precision, H * Nn * A * 4, Nn * O * 4,
                                      (int64_t)qs::kEnvRec * s.num_envs * 4});
    if (biggest >= (int64_t(1) << 31))
      return fail(QS_E_INVALID, "qs_create: num_envs * num_drones too large for one handle (a state buffer would "
                                "exceed 2^31 bytes); shard the envs over more handles");
  }
  HIP_TRY(hipSetDevice(device));
  auto* h = new (std::nothrow) qs_handle();
  if (!h) return fail(QS_E_NOMEM, "qs_create: host allocation failed");
  h->spec = s;
  h->spec.initial_xyzs = nullptr;
  h->device = device;
  {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
      h->num_cu = cu;
  }
  qs_dims& d = h->dims;
  d.num_envs = s.num_envs; d.num_drones = s.num_drones; d.num_agents = s.num_envs * s.num_drones;
  d.act_dim = A; d.hist_len = s.ctrl_freq / 2; d.substeps = s.pyb_freq / s.ctrl_freq;
  d.obs_dim = 12 + d.hist_len * A + (s.task == QS_TASK_SPIRAL ? 11 : 0);
  d.precision = s.precision; d.agent_fields = QS_AGENT_FIELDS; d.env_fields = QS_ENV_FIELDS;
  {
    int rows; size_t bytes;
    if (lds_plan(d, qs::kBlock / s.num_drones, 1, &rows, &bytes) != QS_OK) {
      delete h;
      return fail(QS_E_INVALID, "qs_create: action history (ctrl_freq // 2 entries) does not fit in LDS");
    }
  }
  // initial layout (BaseAviary.py:194-197 / SpiralAviary.py:47-53)
  const HostConsts C;
  h->orig_host.resize(3 * s.num_drones);
  for (int i = 0; i < s.num_drones; ++i) {
    double xyz[3];
    if (s.initial_xyzs) { for (int k = 0; k < 3; ++k) xyz[k] = s.initial_xyzs[i * 3 + k]; }
    else if (s.task == QS_TASK_SPIRAL) {
      xyz[0] = s.spiral_radius * std::cos(2 * M_PI * i / s.num_drones);
      xyz[1] = s.spiral_radius * std::sin(2 * M_PI * i / s.num_drones);
      xyz[2] = 0.3;
    } else {
      xyz[0] = i * 4 * C.L; xyz[1] = i * 4 * C.L; xyz[2] = C.COLL_H / 2 - C.COLL_Z_OFF + .1;
    }
    for (int k = 0; k < 3; ++k) h->orig_host[i * 3 + k] = xyz[k];
  }
  // MultiHover reset draws are rejected when two drones come within 0.5 m
  // (MH:96-101).  The U(±0.25) noise moves a pair by < 0.5 per axis, so a layout
  // whose every pair is >= 1 m apart in x or y never rejects (the bench's grid);
  // otherwise (the reference's default diagonal layout) rejected envs are queued
  // for reset_search_kernel instead of being searched inside the step.
  bool can_reject = false;
  for (int i = 0; i < s.num_drones; ++i)
    for (int j = i + 1; j < s.num_drones; ++j)
      if (std::fabs(h->orig_host[i * 3] - h->orig_host[j * 3]) < 1.0 &&
          std::fabs(h->orig_host[i * 3 + 1] - h->orig_host[j * 3 + 1]) < 1.0)
        can_reject = true;
  // (z is clipped to [0.1, 1], so MH:96's z < 0.1 test never rejects either)
  h->reject_free = s.task == QS_TASK_MULTIHOVER && !can_reject;
  const bool may_reject = s.task == QS_TASK_MULTIHOVER && s.num_drones <= qs::kResetMaxD && can_reject;
  const size_t rs = (size_t)s.precision;
  const size_t N = d.num_agents;
  // per-env episode rings: at least 8 slots each, 65 536 records in all for small batches
  h->log_per_env = (int)std::max<int64_t>(8, ((int64_t)1 << 16) / std::max(1, s.num_envs));
  auto cleanup = [&]() { qs_destroy(h); };
  hipError_t e1 = hipMalloc(&h->st, rs * QS_AGENT_FIELDS * N);
  hipError_t e2 = hipMalloc((void**)&h->env, sizeof(int32_t) * qs::kEnvRec * s.num_envs);
  hipError_t e3 = hipMalloc((void**)&h->hist, sizeof(float) * d.hist_len * N * A);
  hipError_t e5 = hipMalloc(&h->orig, rs * 3 * s.num_drones);
  hipError_t e6 = hipMalloc((void**)&h->log, sizeof(qs_episode_rec) * h->log_per_env * (size_t)s.num_envs);
  hipError_t e7 = hipSuccess;
  hipError_t e8 = hipMalloc((void**)&h->err, sizeof(int));
  if (e1 || e2 || e3 || e5 || e6 || e7 || e8) { cleanup(); return fail(QS_E_NOMEM, "qs_create: hipMalloc failed"); }
  if (may_reject && !(s.flags & QS_FLAG_INKERNEL_RESET_SEARCH)) {
    // header line {count, envs written}, then one 128-B record per slot
    // (initialised when the step kernel queues an env; qs::reset_search_kernel)
    const size_t qn = (size_t)qs::kRqLine * (1 + (size_t)s.num_envs);
    if (hipMalloc((void**)&h->rq, sizeof(int) * qn) != hipSuccess) { cleanup(); return fail(QS_E_NOMEM, "qs_create: hipMalloc failed"); }
    if (hipMalloc((void**)&h->rpre, sizeof(int32_t) * (size_t)s.num_envs) != hipSuccess) {
      cleanup(); return fail(QS_E_NOMEM, "qs_create: hipMalloc failed");
    }
    if (hipMemset(h->rq, 0, sizeof(int) * qn) ||
        hipMemset(h->rpre, 0, sizeof(int32_t) * (size_t)s.num_envs)) {
      cleanup(); return fail(QS_E_HIP, "qs_create: memset");
    }
  }
  if (s.precision == 8) {
    if (hipMemcpy(h->orig, h->orig_host.data(), 8 * 3 * s.num_drones, hipMemcpyHostToDevice)) { cleanup(); return fail(QS_E_HIP, "qs_create: copy"); }
  } else {
    std::vector<float> of(h->orig_host.begin(), h->orig_host.end());
    if (hipMemcpy(h->orig, of.data(), 4 * 3 * s.num_drones, hipMemcpyHostToDevice)) { cleanup(); return fail(QS_E_HIP, "qs_create: copy"); }
  }
  if (hipMemset(h->st, 0, rs * QS_AGENT_FIELDS * N) || hipMemset(h->env, 0, sizeof(int32_t) * qs::kEnvRec * s.num_envs) ||
      hipMemset(h->hist, 0, sizeof(float) * d.hist_len * N * A) ||
      hipMemset(h->err, 0, sizeof(int))) {
    cleanup(); return fail(QS_E_HIP, "qs_create: memset");
  }
#ifdef QS_STAMPS_BUILD
  if (getenv("QS_STAMPS")) {   // dev-only phase timestamps
    const int grid = (s.num_envs + qs::kBlock / s.num_drones - 1) / (qs::kBlock / s.num_drones);
    if (hipMalloc((void**)&h->stamps, sizeof(unsigned long long) * 8 * grid) == hipSuccess)
      hipMemset(h->stamps, 0, sizeof(unsigned long long) * 8 * grid);
  }
#endif
  *out = h;
  return QS_OK;
}

// dev-only: copy the per-wave phase timestamps (8 per workgroup) to host.
extern "C" int qs_debug_stamps(qs_handle* h, unsigned long long* host, int64_t n) {
  if (!h || !h->stamps) return fail(QS_E_STATE, "QS_STAMPS not enabled");
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(host, h->stamps, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
  return QS_OK;
}

int qs_destroy(qs_handle* h) {
  if (!h) return QS_OK;
  (void)hipSetDevice(h->device);   // teardown: best effort, nothing to report to
  void* ptrs[] = {h->st, h->env, h->hist, h->orig, h->log, h->err, h->stamps, h->rq, h->rpre, h->logw, h->log_sel};
  for (void* p : ptrs) if (p) (void)hipFree(p);
  delete h;
  return QS_OK;
}

int qs_get_dims(const qs_handle* h, qs_dims* out) {
  if (!h || !out) return fail(QS_E_INVALID, "qs_get_dims: null argument");
  *out = h->dims;
  return QS_OK;
}

int qs_reset(qs_handle* h, uint64_t seed, float* obs, void* stream) {
  if (!h) return fail(QS_E_INVALID, "qs_reset: null handle");
  hipStream_t st = (hipStream_t)stream;
  const qs_dims& d = h->dims;
  const size_t N = d.num_agents, rs = d.precision;
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemsetAsync(h->st, 0, rs * QS_AGENT_FIELDS * N, st));
  HIP_TRY(hipMemsetAsync(h->env, 0, sizeof(int32_t) * qs::kEnvRec * d.num_envs, st));
  HIP_TRY(hipMemsetAsync(h->hist, 0, sizeof(float) * d.hist_len * N * d.act_dim, st));
  HIP_TRY(hipMemsetAsync(h->err, 0, sizeof(int), st));
  // the precomputed reset searches belong to the old (seed, episode) tags: restart
  // them, or a queued search would skip the new episode's first chunks (MH:83-102
  // takes the FIRST accepted try)
  if (h->rpre) HIP_TRY(hipMemsetAsync(h->rpre, 0, sizeof(int32_t) * d.num_envs, st));
  h->seed = seed;
  int rc;
  if (d.precision == 8) {
    qs::Params<double> P; fill_params(h, P); P.mode = qs::MODE_RESET_ALL; P.obs = obs;
    rc = launch(h, P, st);
  } else {
    qs::Params<float> P; fill_params(h, P); P.mode = qs::MODE_RESET_ALL; P.obs = obs;
    rc = launch(h, P, st);
  }
  if (rc == QS_OK) h->reset_done = true;
  return rc;
}

int qs_reset_envs(qs_handle* h, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail(QS_E_INVALID, "qs_reset_envs: null handle");
  if (!h->reset_done) return fail(QS_E_STATE, "qs_reset_envs: call qs_reset first");
  hipStream_t st = (hipStream_t)stream;
  if (h->dims.precision == 8) {
    qs::Params<double> P; fill_params(h, P); P.mode = qs::MODE_RESET_MASK; P.reset_mask = mask; P.obs = obs;
    return launch(h, P, st);
  }
  qs::Params<float> P; fill_params(h, P); P.mode = qs::MODE_RESET_MASK; P.reset_mask = mask; P.obs = obs;
  return launch(h, P, st);
}

int qs_step(qs_handle* h, const float* actions, const qs_step_out* out, void* stream) {
  if (!h) return fail(QS_E_INVALID, "qs_step: null handle");
  if (!h->reset_done) return fail(QS_E_STATE, "qs_step: call qs_reset first");
  hipStream_t st = (hipStream_t)stream;
  qs_step_out o{};
  if (out) o = *out;
  if (h->dims.precision == 8) {
    qs::Params<double> P; fill_params(h, P); P.mode = qs::MODE_STEP;
    P.act_in = actions; P.obs = o.obs; P.rew = (double*)o.reward; P.term = o.terminated; P.trunc = o.truncated;
    P.tobs = o.terminal_obs; P.reasons = o.reasons; P.act_out = o.actions_out;
    return launch(h, P, st);
  }
  qs::Params<float> P; fill_params(h, P); P.mode = qs::MODE_STEP;
  P.act_in = actions; P.obs = o.obs; P.rew = (float*)o.reward; P.term = o.terminated; P.trunc = o.truncated;
  P.tobs = o.terminal_obs; P.reasons = o.reasons; P.act_out = o.actions_out;
  return launch(h, P, st);
}

// qs_state_io's view of the per-env records: counters as [QS_ENV_FIELDS][E]
// int32 (counters = true) or the episode returns as [E] f64.
// Written counters (the episode number among them) void the env's precomputed
// reset search: word 7 and its chunk counter start over.
__global__ void env_io_kernel(int32_t* rec, void* ext, int E, bool counters, bool to_rec, int32_t* pre) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  int32_t* r = rec + (size_t)e * qs::kEnvRec;
  if (counters) {
    int32_t* x = (int32_t*)ext;
    for (int f = 0; f < QS_ENV_FIELDS; ++f) {
      if (to_rec) r[f] = x[(size_t)f * E + e];
      else x[(size_t)f * E + e] = r[f];
    }
    if (to_rec) {
      r[qs::kEnvPreWord] = 0;
      if (pre) pre[e] = 0;
    }
  } else {
    double* x = (double*)ext;
    double* rr = reinterpret_cast<double*>(r + qs::kEnvRetWord);
    if (to_rec) *rr = x[e];
    else x[e] = *rr;
  }
}

int qs_state_io(qs_handle* h, int block, void* buf, int dir, void* stream) {
  if (!h || !buf) return fail(QS_E_INVALID, "qs_state_io: null argument");
  hipStream_t st = (hipStream_t)stream;
  const qs_dims& d = h->dims;
  void* src = nullptr;
  size_t bytes = 0;
  switch (block) {
    case QS_STATE_AGENT: src = h->st; bytes = (size_t)d.precision * QS_AGENT_FIELDS * d.num_agents; break;
    case QS_STATE_ENV:
    case QS_STATE_EP_RETURN: {   // the external layouts [4][E] int32 / [E] f64, from the records
      HIP_TRY(hipSetDevice(h->device));
      const int E = d.num_envs;
      env_io_kernel<<<(E + 255) / 256, 256, 0, st>>>(h->env, buf, E, block == QS_STATE_ENV, dir != 0, h->rpre);
      HIP_TRY(hipGetLastError());
      if (dir) h->reset_done = true;
      return QS_OK;
    }
    case QS_STATE_HISTORY: src = h->hist; bytes = sizeof(float) * d.hist_len * d.num_agents * d.act_dim; break;
    default: return fail(QS_E_INVALID, "qs_state_io: bad block");
  }
  HIP_TRY(hipSetDevice(h->device));
  if (dir) HIP_TRY(hipMemcpyAsync(src, buf, bytes, hipMemcpyDeviceToDevice, st));
  else HIP_TRY(hipMemcpyAsync(buf, src, bytes, hipMemcpyDeviceToDevice, st));
  if (dir) h->reset_done = true;
  return QS_OK;
}

int qs_episode_log(qs_handle* h, qs_episode_rec* dst, int64_t cap, int64_t* total, int64_t* written, void* stream) {
  if (!h || !total) return fail(QS_E_INVALID, "qs_episode_log: null argument");
  if (written) *written = 0;
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(h->device));
  const int E = h->dims.num_envs, R = h->log_per_env;
  const unsigned grid = (unsigned)((E + 255) / 256);
  if (!h->logw) HIP_TRY(hipMalloc((void**)&h->logw, sizeof(qs::LogWork)));
  qs::LogWork* w = h->logw;
  // 1. total and the newest seq (one 16-byte read back)
  HIP_TRY(hipMemsetAsync(w, 0, sizeof(qs::LogWork), st));
  HIP_TRY(hipMemsetAsync(&w->maxseq, 0xff, sizeof(long long), st));   // −1: nothing logged
  hipLaunchKernelGGL(qs::log_scan_kernel, dim3(grid), dim3(256), 0, st, h->env, h->log, E, R, w);
  HIP_TRY(hipGetLastError());
  struct { unsigned long long total; long long maxseq; } head;
  HIP_TRY(hipMemcpyAsync(&head, w, sizeof(head), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *total = (int64_t)head.total;
  if (!dst || cap <= 0 || head.total == 0) return QS_OK;
  // 2. how far below the newest seq the newest `cap` live records reach
  hipLaunchKernelGGL(qs::log_hist_kernel, dim3(grid), dim3(256), 0, st, h->env, h->log, E, R, w);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned int> hist(qs::kLogBins);
  HIP_TRY(hipMemcpyAsync(hist.data(), w->hist, hist.size() * sizeof(unsigned int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  uint64_t live = 0, cum = 0;
  for (unsigned int c : hist) live += c;
  long long thr = -1;   // every live record, unless the newest `cap` lie within the binned window
  uint64_t want = live;
  for (int b = 0; b < qs::kLogBins - 1; ++b) {
    cum += hist[b];
    if (cum >= (uint64_t)cap) {   // bin b = seq maxseq − b holds the cap-th newest
      thr = head.maxseq - b;
      want = cum;
      break;
    }
  }
  // 3. compact the records at or above the threshold (the cap newest plus the rest
  // of the threshold seq's ties) and order them on the host: (seq, env) is the
  // order the reference's env loop logs them
  if (h->log_sel_cap < want) {
    if (h->log_sel) HIP_TRY(hipFree(h->log_sel));
    h->log_sel = nullptr;
    h->log_sel_cap = std::max<size_t>((size_t)want, 1024);
    HIP_TRY(hipMalloc((void**)&h->log_sel, h->log_sel_cap * sizeof(qs_episode_rec)));
  }
  hipLaunchKernelGGL(qs::log_select_kernel, dim3(grid), dim3(256), 0, st, h->env, h->log, E, R, thr, h->log_sel,
                     (unsigned)want, w);
  HIP_TRY(hipGetLastError());
  std::vector<qs_episode_rec> sel((size_t)want);
  HIP_TRY(hipMemcpyAsync(sel.data(), h->log_sel, sel.size() * sizeof(qs_episode_rec), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const size_t k = std::min<size_t>(sel.size(), (size_t)cap);
  auto older = [](const qs_episode_rec& a, const qs_episode_rec& b) {
    return a.seq != b.seq ? a.seq < b.seq : a.env < b.env;
  };
  // the k newest, oldest first
  std::nth_element(sel.begin(), sel.begin() + (sel.size() - k), sel.end(), older);
  std::sort(sel.begin() + (sel.size() - k), sel.end(), older);
  HIP_TRY(hipMemcpyAsync(dst, sel.data() + (sel.size() - k), k * sizeof(qs_episode_rec), hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (written) *written = (int64_t)k;
  return QS_OK;
}

int qs_reset_error(qs_handle* h, int* out) {
  if (!h || !out) return fail(QS_E_INVALID, "qs_reset_error: null argument");
  HIP_TRY(hipMemcpy(out, h->err, sizeof(int), hipMemcpyDeviceToHost));
  return QS_OK;
}

int qs_calib_copy(float* dst, const float* src, int64_t n, void* stream) {
  if (!dst || !src || n < 0) return fail(QS_E_INVALID, "qs_calib_copy: bad argument");
  long long blocks = std::min<long long>((n + 255) / 256, 256LL * 8);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(qs::calib_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dst, src, (long long)n);
  HIP_TRY(hipGetLastError());
  return QS_OK;
}

}  // extern "C"
