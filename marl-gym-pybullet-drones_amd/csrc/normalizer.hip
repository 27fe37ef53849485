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
// Here the moments are two launches: one workgroup per 16-row tile reads its
// contiguous span once into LDS and forms every column's tile mean and sum of
// squared deviations (two passes from LDS, float64); then the tiles are merged
// per column by 64 threads and a fixed LDS tree (the batch mean first, then
// the parallel-variance sum Σ M2_t + n_t·(mean_t − mean)²) and
// normalization.py:42-60's update applied in place in its operation order.
// Fixed orders throughout: a replay is bit-identical.  The normalisation is a
// third, elementwise launch (float64 arithmetic, float32 out).  HBM-bound: 4 B
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
constexpr int kRmsRows = 16;        // rows per tile (one workgroup each)
constexpr int kRmsMergeCols = 4;    // columns per merge workgroup (64 threads each)

struct RmsShape {
  long long R;
  int C, GR;   // tiles of kRmsRows rows
};

__host__ __device__ inline RmsShape rms_shape(long long R, int C) {
  RmsShape s;
  s.R = R;
  s.C = C;
  s.GR = (int)((R + kRmsRows - 1) / kRmsRows);
  return s;
}

// work: [counter (64 B)] [mean_b: GR·C] [m2_b: GR·C]   (tile t has min(16, R − 16t) rows)
inline long long rms_work_bytes(const RmsShape& s) { return 64 + 16LL * s.GR * s.C; }

// Launch 1: one workgroup per 16-row tile; the tile's rows are one contiguous
// span of x, read once (coalesced) into LDS, then every column's mean and sum
// of squared deviations over the tile's rows (two passes from LDS, float64).
__global__ void __launch_bounds__(kRmsBlock) rms_tile_kernel(RmsShape s, const float* __restrict__ x,
                                                             unsigned* __restrict__ work) {
  extern __shared__ float tile[];   // [rows][C]
  const int t = threadIdx.x, b = blockIdx.x;
  const long long r0 = (long long)b * kRmsRows;
  const int nr = (int)min((long long)kRmsRows, s.R - r0);
  const float* src = x + r0 * s.C;
  const int n = nr * s.C;
  for (int i = t; i < n; i += kRmsBlock) tile[i] = src[i];
  __syncthreads();
  double* mean_b = reinterpret_cast<double*>(reinterpret_cast<char*>(work) + 64);
  double* m2_b = mean_b + (size_t)s.GR * s.C;
  for (int c = t; c < s.C; c += kRmsBlock) {
    double a = 0.0;
    for (int r = 0; r < nr; ++r) a += (double)tile[r * s.C + c];
    const double m = a / (double)nr;
    double q = 0.0;
    for (int r = 0; r < nr; ++r) {
      const double d = (double)tile[r * s.C + c] - m;
      q += d * d;
    }
    mean_b[(size_t)b * s.C + c] = m;
    m2_b[(size_t)b * s.C + c] = q;
  }
}

// Launch 2: kRmsMergeCols columns per workgroup, 64 threads per column, each
// thread over the tiles t ≡ lane (mod 64) in order, the lanes combined by a
// fixed LDS tree: the batch mean Σ n_t·mean_t / R first, then M2 = Σ (M2_t +
// n_t·(mean_t − mean)²) (the parallel-variance merge with the mean known), then
// normalization.py:42-60's update of the running statistics in its operation
// order.  Every workgroup reads the running count before arriving; the last to
// arrive writes the new count.
__device__ __forceinline__ double rms_lane_sum(double v, double* red, int col, int lane) {
  red[col * 64 + lane] = v;
  __syncthreads();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    if (lane < o) red[col * 64 + lane] += red[col * 64 + lane + o];
    __syncthreads();
  }
  const double r = red[col * 64];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kRmsBlock) rms_merge_kernel(RmsShape s, double* __restrict__ mean,
                                                              double* __restrict__ var, double* __restrict__ count,
                                                              double* __restrict__ sums, unsigned* __restrict__ work) {
  __shared__ double red[kRmsMergeCols * 64];
  __shared__ bool last;
  const int t = threadIdx.x, col = t >> 6, lane = t & 63;
  const int c = blockIdx.x * kRmsMergeCols + col;
  const bool cv = c < s.C;
  const double* mean_b = reinterpret_cast<const double*>(reinterpret_cast<const char*>(work) + 64);
  const double* m2_b = mean_b + (size_t)s.GR * s.C;
  const double cnt = sums ? 0.0 : *count;   // (the multi-rank form has no statistics)
  auto nrows = [&](int tt) { return (double)min((long long)kRmsRows, s.R - (long long)tt * kRmsRows); };
  double a = 0.0;
  if (cv)
    for (int tt = lane; tt < s.GR; tt += 64) a += nrows(tt) * mean_b[(size_t)tt * s.C + c];
  const double na = (double)s.R;
  const double bm = rms_lane_sum(a, red, col, lane) / na;
  double q = 0.0;
  if (cv)
    for (int tt = lane; tt < s.GR; tt += 64) {
      const double d = mean_b[(size_t)tt * s.C + c] - bm;
      q += m2_b[(size_t)tt * s.C + c] + nrows(tt) * (d * d);
    }
  const double qa = rms_lane_sum(q, red, col, lane);
  if (cv && lane == 0) {
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
  __syncthreads();
  if (t == 0) {
    __threadfence();
    last = atomicAdd(work, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && t == 0) {
    if (sums) sums[2 * s.C] = na;
    else *count = na + cnt;
    *work = 0u;
  }
}

// out = clip((x − mean) / sqrt(var + eps), −clip, clip) in float64, stored as
// float32 (MeanStdNormalizer.__call__, normalization.py:110-113); NaN passes
// through like torch.clamp
__global__ void __launch_bounds__(kRmsBlock) rms_normalize_kernel(long long R, int C, const float* __restrict__ x,
                                                                   const double* __restrict__ mean,
                                                                   const double* __restrict__ var, double eps,
                                                                   double clip, float* __restrict__ out) {
  // one row per workgroup step (no per-element modulo): threads over its columns
  for (long long r = blockIdx.x; r < R; r += gridDim.x) {
    const float* xr = x + r * C;
    float* orow = out + r * C;
    for (int c = threadIdx.x; c < C; c += kRmsBlock) {
      double y = ((double)xr[c] - mean[c]) / sqrt(var[c] + eps);
      y = y < -clip ? -clip : (y > clip ? clip : y);
      orow[c] = (float)y;
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
  if (R > (1LL << 40) || (long long)R * C > (1LL << 46) || (long long)C * kRmsRows * 4 > 64 * 1024)
    return nfail(QS_E_INVALID, "qs_rms_update: batch too large (at most 1 024 columns)");
  const RmsShape s = rms_shape(R, C);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(rms_tile_kernel, dim3((unsigned)s.GR), dim3(kRmsBlock), (size_t)C * kRmsRows * 4, st, s, x,
                     (unsigned*)work);
  hipLaunchKernelGGL(rms_merge_kernel, dim3((unsigned)((C + kRmsMergeCols - 1) / kRmsMergeCols)), dim3(kRmsBlock), 0,
                     st, s, mean, var, count, sums, (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_update: ") + hipGetErrorString(e));
}

int qs_rms_normalize(int64_t R, int32_t C, const float* x, const double* mean, const double* var, double eps,
                     double clip, float* out, void* stream) {
  if (R <= 0 || C <= 0 || !x || !mean || !var || !out) return nfail(QS_E_INVALID, "qs_rms_normalize: bad argument");
  const long long grid = std::min<long long>(R, 8192);
  hipLaunchKernelGGL(rms_normalize_kernel, dim3((unsigned)grid), dim3(kRmsBlock), 0, (hipStream_t)stream, (long long)R,
                     (int)C, x, mean, var, eps, clip, out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_normalize: ") + hipGetErrorString(e));
}

}  // extern "C"
