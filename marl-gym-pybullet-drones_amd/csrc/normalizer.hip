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
// Here the moments are one launch: each workgroup owns a row range × up to
// 256 columns, takes its range's mean and sum of squared deviations in two
// passes over rows it re-reads from L2 (float64, lanes of the same column
// combined in lane order through LDS), and the last workgroup to arrive merges
// the range partials in row-range order (the global mean first, then the
// parallel-variance sum Σ M2_b + n_b·(mean_b − mean)²), then applies
// normalization.py:42-60's update in place in its operation order.  Fixed orders throughout: a replay is bit-identical.  The
// normalisation is a second, elementwise launch (float64 arithmetic, float32
// out).  HBM-bound: 4 B read per element for the moments (plus an L2 re-read),
// 4 B read + 4 B written for the normalisation.

#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_nerr;
int nfail(int code, const std::string& m) { g_nerr = m; return code; }

constexpr int kRmsBlock = 256;
constexpr int kRmsRowsMin = 16;     // rows per workgroup at least
constexpr int kRmsRangesMax = 64;   // row ranges at most: the last workgroup's merge walks them per column

struct RmsShape {
  long long R;
  int C, GR, GC;   // row ranges, column blocks of <= 256 columns
};

__host__ __device__ inline RmsShape rms_shape(long long R, int C) {
  RmsShape s;
  s.R = R;
  s.C = C;
  long long gr = (R + kRmsRowsMin - 1) / kRmsRowsMin;
  s.GR = (int)(gr < kRmsRangesMax ? gr : kRmsRangesMax);
  s.GC = (C + kRmsBlock - 1) / kRmsBlock;
  return s;
}

// work: [counter (64 B)] [n_b: GR doubles] [mean_b: GR·C] [m2_b: GR·C]
inline long long rms_work_bytes(const RmsShape& s) { return 64 + 8LL * s.GR * (1 + 2LL * s.C); }

__global__ void __launch_bounds__(kRmsBlock) rms_moments_kernel(RmsShape s, const float* __restrict__ x,
                                                                double* __restrict__ mean, double* __restrict__ var,
                                                                double* __restrict__ count, double* __restrict__ sums,
                                                                unsigned* __restrict__ counter) {
  __shared__ double lds[kRmsBlock];
  __shared__ bool last;
  const int t = threadIdx.x;
  const int rb = blockIdx.x, cb = blockIdx.y;
  const int c0 = cb * kRmsBlock;
  const int CW = min(kRmsBlock, s.C - c0);   // this block's columns
  const int P = kRmsBlock / CW;              // row lanes per column
  const int lane = t / CW, col = c0 + t % CW;
  const bool act = lane < P;
  const long long r0 = s.R * rb / s.GR, r1 = s.R * (rb + 1) / s.GR;
  const double nb = (double)(r1 - r0);
  double* n_b = reinterpret_cast<double*>(reinterpret_cast<char*>(counter) + 64);
  double* mean_b = n_b + s.GR;
  double* m2_b = mean_b + (size_t)s.GR * s.C;

  // pass 1: the range's column sums (lanes in order)
  double a = 0.0;
  if (act)
    for (long long r = r0 + lane; r < r1; r += P) a += (double)x[(size_t)r * s.C + col];
  lds[t] = a;
  __syncthreads();
  double m = 0.0;
  if (act) {
    double sum = 0.0;
    for (int p = 0; p < P; ++p) sum += lds[p * CW + t % CW];
    m = sum / nb;
  }
  __syncthreads();
  // pass 2: Σ (x − m)² of the range (the rows are L2-resident from pass 1)
  double q = 0.0;
  if (act)
    for (long long r = r0 + lane; r < r1; r += P) {
      const double d = (double)x[(size_t)r * s.C + col] - m;
      q += d * d;
    }
  lds[t] = q;
  __syncthreads();
  if (t < CW) {
    double m2 = 0.0;
    for (int p = 0; p < P; ++p) m2 += lds[p * CW + t];
    mean_b[(size_t)rb * s.C + col] = m;
    m2_b[(size_t)rb * s.C + col] = m2;
    if (cb == 0 && t == 0) n_b[rb] = nb;
  }
  __syncthreads();
  if (t == 0) {
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x * gridDim.y - 1;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // the batch moments: the ranges merged in order (parallel variance)
  const double cnt = sums ? 0.0 : *count;   // (the multi-rank form has no statistics)
  // mean = Σ n_b·mean_b / N, then M2 = Σ (M2_b + n_b·(mean_b − mean)²): the
  // parallel-variance merge with the global mean known (no division per range;
  // a sequential Chan merge of 512 ranges with an fp64 division each took
  // ~600 µs in one workgroup), ranges in order
  const double na = (double)s.R;
  for (int c = t; c < s.C; c += kRmsBlock) {
    double sm = 0.0;
#pragma unroll 8
    for (int b = 0; b < s.GR; ++b) sm += n_b[b] * mean_b[(size_t)b * s.C + c];
    const double bm = sm / na;
    double qa = 0.0;
#pragma unroll 8
    for (int b = 0; b < s.GR; ++b) {
      const double d = mean_b[(size_t)b * s.C + c] - bm;
      qa += m2_b[(size_t)b * s.C + c] + n_b[b] * (d * d);
    }
    const double bv = qa / na;   // np.mean, np.var (ddof 0)
    if (sums) {   // several ranks: this rank's Σx and Σx² (merged across ranks by the caller)
      sums[c] = bm * na;
      sums[s.C + c] = qa + bm * bm * na;
      continue;
    }
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
  __syncthreads();   // every column read the old count
  if (t == 0) {
    if (sums) sums[2 * s.C] = (double)s.R;
    else *count = (double)s.R + cnt;
    *counter = 0u;
  }
}

// out = clip((x − mean) / sqrt(var + eps), −clip, clip) in float64, stored as
// float32 (MeanStdNormalizer.__call__, normalization.py:110-113); NaN passes
// through like torch.clamp
__global__ void rms_normalize_kernel(long long n, int C, const float* __restrict__ x, const double* __restrict__ mean,
                                     const double* __restrict__ var, double eps, double clip, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % C);
    double y = ((double)x[i] - mean[c]) / sqrt(var[c] + eps);
    y = y < -clip ? -clip : (y > clip ? clip : y);
    out[i] = (float)y;
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
  if (R > (1LL << 40) || (long long)R * C > (1LL << 46)) return nfail(QS_E_INVALID, "qs_rms_update: batch too large");
  const RmsShape s = rms_shape(R, C);
  hipLaunchKernelGGL(rms_moments_kernel, dim3((unsigned)s.GR, (unsigned)s.GC), dim3(kRmsBlock), 0,
                     (hipStream_t)stream, s, x, mean, var, count, sums, (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_update: ") + hipGetErrorString(e));
}

int qs_rms_normalize(int64_t R, int32_t C, const float* x, const double* mean, const double* var, double eps,
                     double clip, float* out, void* stream) {
  if (R <= 0 || C <= 0 || !x || !mean || !var || !out) return nfail(QS_E_INVALID, "qs_rms_normalize: bad argument");
  const long long n = (long long)R * C;
  const int block = 256;
  const long long grid = std::min<long long>((n + block - 1) / block, 4096);
  hipLaunchKernelGGL(rms_normalize_kernel, dim3((unsigned)grid), dim3(block), 0, (hipStream_t)stream, n, (int)C, x,
                     mean, var, eps, clip, out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : nfail(QS_E_HIP, std::string("qs_rms_normalize: ") + hipGetErrorString(e));
}

}  // extern "C"
