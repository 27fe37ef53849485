// normalizer.hip — the observation normaliser of the MAPPO rollout on gfx950
// (include/qs_learner.h: qs_rms_update, qs_rms_normalize).
//
// safe_control_gym/math_and_models/normalization.py:13-120: MeanStdNormalizer
// updates a RunningMeanStd with the batch's per-column moments (np.mean /
// np.var over axis 0, float64) and returns clip((x − mean) / sqrt(var + eps)).
// The rollout calls it once per control step on the (E, D, O) obs
// (env_select_learn_mappo.py:265-283 runs norm_obs), so torch's generic
// float64 column reductions (a Welford reduce_kernel of ~200 µs and a mean of
// ~90 µs at C4's 8 192 × 135) were most of a C4 rollout step.
//
// Here the moments are two launches: each 64-row tile's columns are held in
// registers (16 rows per wave) and give the tile's column means and sums of
// squared deviations (two passes, float64); then a workgroup per 16 columns
// merges the tiles (the batch mean first, then the parallel-variance sum
// Σ M2_t + n_t·(mean_t − mean)²) and applies normalization.py:42-60's update
// in place in its operation order.  No atomics or fences: an agent-scope
// release per workgroup writes back the XCD's L2 and cost ~40 µs over 1 280
// workgroups when the merge was folded into the tile launch.  Fixed orders
// throughout: a replay is bit-identical.  The normalisation is a third,
// elementwise launch (float64 arithmetic, float32 out).  HBM-bound: 4 B
// read per element for the moments, 4 B read + 4 B written for the
// normalisation.

#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_nerr;
int nfail(int code, const std::string& m) { g_nerr = m; return code; }

constexpr int kRmsBlock = 256;
constexpr int kRmsRows = 64;        // rows per tile
constexpr int kRmsCols = 64;        // columns per workgroup (one per lane)

struct RmsShape {
  long long R;
  int C, GR, NCB;   // tiles of kRmsRows rows, blocks of kRmsCols columns
};

__host__ __device__ inline RmsShape rms_shape(long long R, int C) {
  RmsShape s;
  s.R = R;
  s.C = C;
  s.GR = (int)((R + kRmsRows - 1) / kRmsRows);
  s.NCB = (C + kRmsCols - 1) / kRmsCols;
  return s;
}

// work: [the running count before this update (one double, 64 B)]
//       [mean_b: GR·C] [m2_b: GR·C]   (tile t has min(64, R − 64t) rows)
inline long long rms_work_bytes(const RmsShape& s) { return 64 + 16LL * s.GR * s.C; }

// Σ over the four waves' values of one lane in wave order (float64)
__device__ __forceinline__ double rms_wave_sum(double (*red)[64], double v, int w, int lane) {
  red[w][lane] = v;
  __syncthreads();
  const double r = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
  __syncthreads();
  return r;
}

// Launch 1: a workgroup per (64-row tile, 64 columns).  Wave w holds rows
// 16w .. 16w+15 of the lane's column in registers (every load issued before
// the first use; a wave's load is 64 consecutive columns of one row), then the
// tile's column mean and its sum of squared deviations from that mean (two
// passes over the registers, float64, the waves combined in order).  Block
// (0, 0) also saves the running count for launch 2 (which rewrites it).
__global__ void __launch_bounds__(kRmsBlock) rms_tile_kernel(RmsShape s, const float* __restrict__ x,
                                                             const double* __restrict__ count,
                                                             unsigned* __restrict__ work) {
  __shared__ double red[4][64];
  constexpr int RW = kRmsRows / 4;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * kRmsCols + lane, b = blockIdx.x;
  const bool cv = c < s.C;
  const long long r0 = (long long)b * kRmsRows;
  const int nr = (int)min((long long)kRmsRows, s.R - r0);
  const int rw = RW * w;
  const float* src = x + (r0 + rw) * s.C + (cv ? c : 0);
  float v[RW];
  if (nr == kRmsRows) {
#pragma unroll
    for (int r = 0; r < RW; ++r) v[r] = cv ? __builtin_nontemporal_load(src + (long long)r * s.C) : 0.0f;
  } else {
#pragma unroll
    for (int r = 0; r < RW; ++r) v[r] = cv && rw + r < nr ? src[(long long)r * s.C] : 0.0f;
  }
  double a = 0.0;
#pragma unroll
  for (int r = 0; r < RW; ++r)
    if (rw + r < nr) a += (double)v[r];
  const double m = rms_wave_sum(red, a, w, lane) / (double)nr;
  double q = 0.0;
#pragma unroll
  for (int r = 0; r < RW; ++r)
    if (rw + r < nr) {
      const double d = (double)v[r] - m;
      q += d * d;
    }
  q = rms_wave_sum(red, q, w, lane);
  double* mean_b = reinterpret_cast<double*>(reinterpret_cast<char*>(work) + 64);
  double* m2_b = mean_b + (size_t)s.GR * s.C;
  if (w == 0 && cv) {
    mean_b[(size_t)b * s.C + c] = m;
    m2_b[(size_t)b * s.C + c] = q;
  }
  if (count && b == 0 && blockIdx.y == 0 && threadIdx.x == 0) *reinterpret_cast<double*>(work) = *count;
}

// Launch 2: a workgroup per 16 columns merges the tiles: 16 slices of the
// workgroup's threads take the tiles t ≡ slice (mod 16), eight loads in flight,
// and the slices are added in order through LDS: the batch mean Σ n_t·mean_t / R,
// then M2 = Σ (M2_t + n_t·(mean_t − mean)²) (the parallel-variance merge with
// the mean known), then normalization.py:42-60's update of the running
// statistics in its operation order, from the count launch 1 saved; block 0
// writes the new count.  No atomics, no fences (the launch boundary orders
// launch 1's writes), every order fixed: a replay is bit-identical.
constexpr int kRmsMergeCols = 16, kRmsSlices = kRmsBlock / kRmsMergeCols;
__device__ __forceinline__ double rms_slice_sum(double (*red)[kRmsMergeCols], double v, int sl, int cl) {
  red[sl][cl] = v;
  __syncthreads();
  double r = red[0][cl];
#pragma unroll
  for (int k = 1; k < kRmsSlices; ++k) r += red[k][cl];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kRmsBlock) rms_merge_kernel(RmsShape s, double* __restrict__ mean,
                                                              double* __restrict__ var, double* __restrict__ count,
                                                              double* __restrict__ sums,
                                                              const unsigned* __restrict__ work) {
  __shared__ double red[kRmsSlices][kRmsMergeCols];
  const int cl = threadIdx.x % kRmsMergeCols, sl = threadIdx.x / kRmsMergeCols;
  const int c = blockIdx.x * kRmsMergeCols + cl;
  const bool cv = c < s.C;
  const int cc = cv ? c : 0;
  const double* mean_b = reinterpret_cast<const double*>(reinterpret_cast<const char*>(work) + 64);
  const double* m2_b = mean_b + (size_t)s.GR * s.C;
  const double cnt = sums ? 0.0 : *reinterpret_cast<const double*>(work);   // (the multi-rank form has no statistics)
  auto nrows = [&](int tt) { return (double)min((long long)kRmsRows, s.R - (long long)tt * kRmsRows); };
  constexpr int kMergeU = 8;
  double ma = 0.0;
  for (int t0 = sl; t0 < s.GR; t0 += kRmsSlices * kMergeU) {
    double mv[kMergeU];
#pragma unroll
    for (int u = 0; u < kMergeU; ++u) {
      const int tt = t0 + kRmsSlices * u;
      mv[u] = tt < s.GR ? mean_b[(size_t)tt * s.C + cc] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kMergeU; ++u)
      if (t0 + kRmsSlices * u < s.GR) ma += nrows(t0 + kRmsSlices * u) * mv[u];
  }
  const double na = (double)s.R;
  const double bm = rms_slice_sum(red, ma, sl, cl) / na;
  double mq = 0.0;
  for (int t0 = sl; t0 < s.GR; t0 += kRmsSlices * kMergeU) {
    double mv[kMergeU], qv[kMergeU];
#pragma unroll
    for (int u = 0; u < kMergeU; ++u) {
      const int tt = t0 + kRmsSlices * u;
      mv[u] = tt < s.GR ? mean_b[(size_t)tt * s.C + cc] : 0.0;
      qv[u] = tt < s.GR ? m2_b[(size_t)tt * s.C + cc] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kMergeU; ++u)
      if (t0 + kRmsSlices * u < s.GR) {
        const double d = mv[u] - bm;
        mq += qv[u] + nrows(t0 + kRmsSlices * u) * (d * d);
      }
  }
  const double qa = rms_slice_sum(red, mq, sl, cl);
  if (sl == 0 && cv) {
    const double bv = qa / na;   // np.mean, np.var (ddof 0)
    if (sums) {   // several ranks: this rank's Σx and Σx² (merged across ranks by the caller)
      sums[c] = bm * na;
      sums[s.C + c] = qa + bm * bm * na;
    } else {
      // normalization.py:42-60, in its operation order
      const double delta = bm - mean[c];
      const double tot = cnt + na;
      const double new_mean = mean[c] + delta * na / tot;
      const double m_a = var[c] * cnt;
      const double m_b = bv * na;
      const double M2 = m_a + m_b + delta * delta * cnt * na / (cnt + na);
      var[c] = M2 / (cnt + na);
      mean[c] = new_mean;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (sums) sums[2 * s.C] = na;
    else *count = na + cnt;
  }
}

// out = clip((x − mean) / sqrt(var + eps), −clip, clip) in float64, stored as
// float32 (MeanStdNormalizer.__call__, normalization.py:110-113); NaN passes
// through like torch.clamp.  Each workgroup first forms sqrt(var + eps) of
// every column once into LDS (with the means), then walks the flat [R·C]
// array four consecutive elements per thread (one 16-byte load and store
// where x and out allow it), their columns from one division.
constexpr int kRmsNormLdsCols = 2048;   // columns staged in LDS (wider: read from global)

__device__ __forceinline__ float rms_norm1(float xv, double m, double sd, double clip) {
  double y = ((double)xv - m) / sd;
  y = y < -clip ? -clip : (y > clip ? clip : y);
  return (float)y;
}

typedef float rms_f4 __attribute__((ext_vector_type(4)));

template <bool VEC, bool LDS>
__global__ void __launch_bounds__(kRmsBlock) rms_normalize_kernel(long long N, int C, const float* __restrict__ x,
                                                                   const double* __restrict__ mean,
                                                                   const double* __restrict__ var, double eps,
                                                                   double clip, float* __restrict__ out) {
  __shared__ double smean[LDS ? kRmsNormLdsCols : 1], ssd[LDS ? kRmsNormLdsCols : 1];
  if constexpr (LDS) {
    for (int c = threadIdx.x; c < C; c += kRmsBlock) {
      smean[c] = mean[c];
      ssd[c] = sqrt(var[c] + eps);
    }
    __syncthreads();
  }
  auto mu = [&](int c) { return LDS ? smean[c] : mean[c]; };
  auto sd = [&](int c) { return LDS ? ssd[c] : sqrt(var[c] + eps); };
  const long long nq = (N + 3) / 4;
  for (long long q = (long long)blockIdx.x * kRmsBlock + threadIdx.x; q < nq; q += (long long)gridDim.x * kRmsBlock) {
    const long long i0 = q * 4;
    int c = (int)(i0 % C);
    if (VEC && i0 + 4 <= N) {
      const rms_f4 v = __builtin_nontemporal_load(reinterpret_cast<const rms_f4*>(x) + q);
      rms_f4 o;
      o.x = rms_norm1(v.x, mu(c), sd(c), clip);
      c = c + 1 == C ? 0 : c + 1;
      o.y = rms_norm1(v.y, mu(c), sd(c), clip);
      c = c + 1 == C ? 0 : c + 1;
      o.z = rms_norm1(v.z, mu(c), sd(c), clip);
      c = c + 1 == C ? 0 : c + 1;
      o.w = rms_norm1(v.w, mu(c), sd(c), clip);
      __builtin_nontemporal_store(o, reinterpret_cast<rms_f4*>(out) + q);
    } else {
      for (long long i = i0; i < N && i < i0 + 4; ++i) {
        out[i] = rms_norm1(x[i], mu(c), sd(c), clip);
        c = c + 1 == C ? 0 : c + 1;
      }
    }
  }
}
}  // namespace

extern "C" {

const char* qs_rms_last_error(void) { return g_nerr.c_str(); }

int64_t qs_rms_work_bytes(int64_t R, int32_t C) {
  if (R <= 0 || C <= 0) return 0;
  return rms_work_bytes(rms_shape(R, C));
}

int qs_rms_update(int64_t R, int32_t C, const float* x, double* mean, double* var, double* count, double* sums,
                  void* work, void* stream) {
  if (R <= 0 || C <= 0 || !x || !work || (!sums && (!mean || !var || !count)))
    return nfail(QS_E_INVALID, "qs_rms_update: bad argument");
  if (R > (1LL << 40) || (long long)R * C > (1LL << 46) || C > 65535 * kRmsCols || (R + kRmsRows - 1) / kRmsRows > (1LL << 31) - 1)
    return nfail(QS_E_INVALID, "qs_rms_update: batch too large");
  const RmsShape s = rms_shape(R, C);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(rms_tile_kernel, dim3((unsigned)s.GR, (unsigned)s.NCB), dim3(kRmsBlock), 0, st, s, x,
                     sums ? nullptr : count, (unsigned*)work);
  hipLaunchKernelGGL(rms_merge_kernel, dim3((unsigned)((C + kRmsMergeCols - 1) / kRmsMergeCols)), dim3(kRmsBlock), 0, st,
                     s, mean, var, count, sums,
                     (const unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_update: ") + hipGetErrorString(e));
}

int qs_rms_normalize(int64_t R, int32_t C, const float* x, const double* mean, const double* var, double eps,
                     double clip, float* out, void* stream) {
  if (R <= 0 || C <= 0 || !x || !mean || !var || !out) return nfail(QS_E_INVALID, "qs_rms_normalize: bad argument");
  const long long N = (long long)R * C, nq = (N + 3) / 4;
  // a grid of at most 1 024 workgroups: each stages the columns' statistics once
  const unsigned grid = (unsigned)std::min<long long>((nq + kRmsBlock - 1) / kRmsBlock, 1024);
  const bool vec = ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0), lds = C <= kRmsNormLdsCols;
  hipStream_t st = (hipStream_t)stream;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kRmsBlock), 0, st, N, (int)C, x, mean, var, eps, clip, out);
  };
  if (vec) lds ? go(rms_normalize_kernel<true, true>) : go(rms_normalize_kernel<true, false>);
  else lds ? go(rms_normalize_kernel<false, true>) : go(rms_normalize_kernel<false, false>);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_normalize: ") + hipGetErrorString(e));
}

}  // extern "C"
