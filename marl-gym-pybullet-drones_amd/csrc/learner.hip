// learner.hip — on-device MAPPO learner kernels for gfx950 (include/qs_learner.h).
//
// qs_gae replaces the reference's host-side numpy loop over E×D×T
// (mappo/buffer.py:428-614) with one thread per sequence walking T backwards;
// loads for step t are independent of the recurrence, so the unrolled loop
// keeps several in flight.  Both kernels are memory/latency-bound elementwise
// work (no contraction ⇒ no MFMA).
//
// qs_adam_gated/qs_adam_commit replace torch.optim.Adam.step behind the
// reference's KL gate (mappo/agent.py:731-734): the gate is evaluated on the
// device from approx_kl, so an update iteration needs no host sync and can be
// replayed from a HIP graph.
//
// qs_ppo_heads forms both PPO losses and their gradients with respect to the
// actor mean, logstd and the critic value in one launch (one thread per agent
// row), replacing some sixty small torch kernels per minibatch; the MLP
// backward stays with autograd.

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }

// The recurrence in float32, as the reference evaluates it: its arrays are
// float32 (buffer.py:346-362) and under its pinned numpy 2.2.6 (NEP 50) a
// float32 scalar op with a Python float (γ, λ) stays float32 with the Python
// float rounded to float32 first, so every line of buffer.py:590-612 is a
// float32 operation in source order (no FMA: -ffp-contract=off).  The results
// are stored to the reference's float64 arrays exactly.
__global__ void gae_kernel(int T, long long N, const float* __restrict__ rews, const float* __restrict__ vals,
                           const float* __restrict__ masks, const float* __restrict__ tvals,
                           const float* __restrict__ last_val, double gamma, double lam, int use_gae,
                           double* __restrict__ rets, double* __restrict__ advs) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float g = (float)gamma, lm = (float)lam;
  const float lv = last_val[n];
  float ret = lv, adv = 0.0f, vnext = lv;
#pragma unroll 4
  for (int t = T - 1; t >= 0; --t) {
    const long long k = (long long)t * N + n;
    const float r = rews[k], m = masks[k];
    const float v = vals ? vals[k] : 0.0f;
    const float tv = tvals ? tvals[k] : 0.0f;
    const float ra = r + g * tv;                            // buffer.py:593
    ret = ra + (g * m) * ret;                               // buffer.py:602
    if (use_gae) {
      const float td = (ra + (g * m) * vnext) - v;          // buffer.py:608
      adv = ((adv * lm) * g) * m + td;                      // buffer.py:609
    } else {
      adv = ret - v;                                        // buffer.py:606
    }
    rets[k] = (double)ret;
    advs[k] = (double)adv;
    vnext = v;
  }
}

__device__ __forceinline__ bool gate_ok(const float* gate_val, float thr) {
  return gate_val == nullptr || *gate_val <= thr;
}

// torch.optim.Adam single step (torch/optim/adam.py, _single_tensor/_multi_tensor
// semantics with amsgrad=False, maximize=False, weight_decay=0):
//   m = lerp(m, g, 1-β1);  v = β2·v + (1-β2)·g²
//   step_size = lr / (1-β1^t);  denom = sqrt(v)/sqrt(1-β2^t) + eps;  p -= step_size·m/denom
__global__ void adam_kernel(long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float* step, float lr, float b1, float b2, float eps,
                            const float* gate_val, float gate_thr) {
  if (!gate_ok(gate_val, gate_thr)) return;    // wave-uniform: the whole update is skipped
  const double t = (double)(*step) + 1.0;
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, t));
  const float step_size = lr / bc1;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const float gi = g[i];
    float mi = m[i];
    mi = mi + (1.0f - b1) * (gi - mi);
    float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

__global__ void adam_commit_kernel(float* step, const float* gate_val, float gate_thr) {
  if (threadIdx.x == 0 && gate_ok(gate_val, gate_thr)) *step = *step + 1.0f;
}

// ------------------------------------------------------------- PPO loss heads
// compute_policy_loss (mappo/agent.py:602-640) and compute_value_loss
// (agent.py:642-683) of one minibatch, forward and backward, in one launch.
// Row r = i·D + d is agent d of env-timestep idx[i].  The arithmetic follows
// the autograd graph of the torch expressions: log_prob of Normal in fp32,
// ratio·adv and clamp(ratio)·adv promoted to f64 (adv is f64), torch.minimum's
// gradient split in half on ties, clamp's gradient inside [lo, hi] inclusive,
// f32 divisions formed in f64 and rounded (correctly rounded, like torch's).
// One thread per row; each workgroup reduces its rows, writes its partial
// sums to the workspace, and the last workgroup to finish adds the partials in
// workgroup order — a fixed order, so a replay gives bit-identical results.
constexpr int kHeadsBlock = 256;
constexpr int kMaxA = 4;
constexpr int kHeadsSums = 3 + kMaxA;   // policy, approx_kl, value, d logstd[A]

// NV block sums at once: one shuffle butterfly per value, one LDS round and one
// barrier for all of them (the per-value order of block_sum: lanes by
// butterfly, then the waves in order); valid in thread 0.
template <int NV>
__device__ __forceinline__ void block_sum_n(double (&x)[NV], double (*lds)[NV]) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < NV; ++k) x[k] += __shfl_xor(x[k], o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[w][k] = x[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double t = 0;
      for (int j = 0; j < (int)(blockDim.x >> 6); ++j) t += lds[j][k];
      x[k] = t;
    }
}


// A (actions per agent) is a template value: the per-action arrays stay in
// registers (a run-time A put them in scratch memory and cost ~70 µs a launch).
template <int A, bool POLICY = true>
__global__ void __launch_bounds__(kHeadsBlock) ppo_heads_kernel(
    int mb, int D, const long long* __restrict__ idx, const float* __restrict__ mean,
    const float* __restrict__ logstd, float scale, const float* __restrict__ act, const float* __restrict__ logp_old,
    const double* __restrict__ adv, const double* __restrict__ ret, const float* __restrict__ v, float clip,
    float ent_coef, float* __restrict__ dmean, float* __restrict__ dlogstd, float* __restrict__ dv,
    float* __restrict__ kl_out, double* __restrict__ acc, double* __restrict__ partial, unsigned* __restrict__ count) {
  __shared__ double ldsn[kHeadsBlock / 64][kHeadsSums];
  __shared__ bool last;
  const int R = mb * D;
  float sd[A], lsd[A], var2[A];
#pragma unroll
  for (int a = 0; a < A; ++a) {
    sd[a] = expf(logstd[a]);          // scale = logstd.exp()
    lsd[a] = logf(sd[a]);             // Normal.log_prob: scale.log()
    var2[a] = 2.0f * (sd[a] * sd[a]); // 2 * scale ** 2
  }
  const float lc = (float)log(sqrt(2.0 * M_PI));
  const float lo = 1.0f - clip, hi = 1.0f + clip;
  const double G = -1.0 / (double)R;  // d(-mean(min(...)))/d min_r
  double sums[kHeadsSums] = {0, 0, 0, 0, 0, 0, 0};
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (POLICY && r < R) {
    const int i = r / D, d = r - i * D;
    const long long g = idx[i];
    const float* x = act + ((size_t)g * D + d) * A;
    float t1[A], logp = 0.0f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float mu = mean[(size_t)r * A + a] * scale;
      t1[a] = x[a] - mu;
      const float t4 = (float)((double)(-(t1[a] * t1[a])) / (double)var2[a]);
      const float lp = (t4 - lsd[a]) - lc;
      logp = a == 0 ? lp : logp + lp;
    }
    const float lpo = logp_old[(size_t)g * D + d];
    const float ratio = expf(logp - lpo);
    const double ad = adv[g];
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const double s1 = (double)ratio * ad, s2 = (double)rc * ad;
    sums[0] = -(s1 < s2 ? s1 : s2);
    sums[1] = (double)(lpo - logp);
    const double g1 = s1 < s2 ? G : (s1 == s2 ? G / 2 : 0.0);
    const double g2 = s2 < s1 ? G : (s1 == s2 ? G / 2 : 0.0);
    float gr = (float)(g1 * ad);
    if (ratio >= lo && ratio <= hi) gr = gr + (float)(g2 * ad);
    const float gl = gr * ratio;                    // d/d logp
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float gt3 = (float)((double)gl / (double)var2[a]);
      const float gt1 = -gt3 * 2.0f * t1[a];
      dmean[(size_t)r * A + a] = -gt1 * scale;
      // d/d logstd_a of log_prob: ((x-mu)²/scale² - 1)·gl
      sums[3 + a] = (double)gl * ((double)(t1[a] * t1[a]) / ((double)sd[a] * sd[a]) - 1.0);
    }
  }
  // value head: 0.5·mean((v - mean_d ret)²) over the mb env-timesteps
  if (r < mb) {
    const double rt = ret[idx[r]];
    double rs = 0;
    for (int d = 0; d < D; ++d) rs += rt;
    const double diff = (double)v[r] - rs / (double)D;
    sums[2] = diff * diff;
    dv[r] = (float)(diff / (double)mb);
  }
  block_sum_n<kHeadsSums>(sums, ldsn);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 3 + A; ++k) partial[(size_t)blockIdx.x * kHeadsSums + k] = sums[k];
    __threadfence();
    last = atomicAdd(count, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: every thread sums a fixed strided subset of the
  // partials in workgroup order, then the same fixed-order block reduction
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double tot[kHeadsSums] = {0, 0, 0, 0, 0, 0, 0};
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x)
#pragma unroll
    for (int k = 0; k < 3 + A; ++k) tot[k] += partial[(size_t)b * kHeadsSums + k];
  block_sum_n<kHeadsSums>(tot, ldsn);
  if (threadIdx.x != 0) return;
  *count = 0;   // ready for the next launch (graph replay)
  if constexpr (!POLICY) {   // qs_value_head: the value loss only
    acc[1] += 0.5 * (tot[2] / (double)mb);
    return;
  }
  float ent = 0.0f;   // Normal.entropy summed over A: 0.5 + 0.5·log(2π) + log(scale)
#pragma unroll
  for (int a = 0; a < A; ++a) ent = a == 0 ? (0.5f + lc) + lsd[a] : ent + ((0.5f + lc) + lsd[a]);
  // d(ent_coef · -mean(entropy))/d logstd_a = -ent_coef
#pragma unroll
  for (int a = 0; a < A; ++a) dlogstd[a] = (float)tot[3 + a] - ent_coef;
  const float akl = (float)(tot[1] / (double)R);
  *kl_out = akl;
  acc[0] += tot[0] / (double)R;
  acc[1] += 0.5 * (tot[2] / (double)mb);
  acc[2] += (double)(-ent);
  acc[3] += (double)akl;
}

// ------------------------------------------------------------- MLP tanh layers
// The elementwise / reduction side of the actor and critic MLPs (MLP with tanh
// hidden layers, safe_control_gym neural_networks.py:18-54) around the GEMMs:
//   qs_mlp_bias_tanh: H = tanh(Z + b) in place of the GEMM output, and for the
//     last hidden layer the linear head out = H·W3ᵀ + b3 in the same pass;
//   qs_mlp_tanh_bwd: dZ = dH ⊙ (1 − H²) with dH given, or formed on the fly as
//     dout·W3 (the head's backward), plus per-block partial sums of the bias
//     gradient Σ_k dZ (and of dW3 = Σ_k dout_k H_k, db3 = Σ_k dout_k);
//   qs_mlp_sum_partials: adds the [G][P] block partials (or the [S][M] split-K
//     weight-gradient partials) in block order into up to three destinations —
//     a fixed order, so a graph replay is bit-identical.
// Rows are 64·C floats (N = hidden size): lane l of a wave owns columns
// [l·C, l·C + C), so every row access is one coalesced wave instruction.
constexpr int kMlpBlock = 256;
constexpr int kMlpMaxA = 4;

template <int C> struct VecC;
template <> struct VecC<1> { typedef float T; };
template <> struct VecC<2> { typedef float2 T; };
template <> struct VecC<4> { typedef float4 T; };

template <int C> __device__ __forceinline__ void ld_row(const float* p, float (&v)[C]) {
  if constexpr (C == 8) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const typename VecC<C>::T t = *reinterpret_cast<const typename VecC<C>::T*>(p);
    __builtin_memcpy(v, &t, sizeof(t));
  }
}
template <int C> __device__ __forceinline__ void st_row(float* p, const float (&v)[C]) {
  if constexpr (C == 8) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    typename VecC<C>::T t;
    __builtin_memcpy(&t, v, sizeof(t));
    *reinterpret_cast<typename VecC<C>::T*>(p) = t;
  }
}

template <int C>
__global__ void __launch_bounds__(kMlpBlock) mlp_bias_tanh_kernel(long long K, const float* __restrict__ z,
                                                                  const float* __restrict__ b, float* __restrict__ h,
                                                                  int A, const float* __restrict__ w3,
                                                                  const float* __restrict__ b3, float* __restrict__ out) {
  constexpr int N = 64 * C;
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * (kMlpBlock / 64);
  float bias[C], w[kMlpMaxA][C];
  ld_row<C>(b + lane * C, bias);
  for (int a = 0; a < A; ++a) ld_row<C>(w3 + (size_t)a * N + lane * C, w[a]);
  for (long long r = (long long)blockIdx.x * (kMlpBlock / 64) + (threadIdx.x >> 6); r < K; r += nw) {
    float v[C];
    ld_row<C>(z + r * N + lane * C, v);
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = tanhf(v[c] + bias[c]);
    st_row<C>(h + r * N + lane * C, v);
    for (int a = 0; a < A; ++a) {
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) t += v[c] * w[a][c];
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0) out[r * A + a] = t + b3[a];
    }
  }
}

// Partial layout per block: [db N | dw3 A·N | db3 A].
// 8 waves per block, one block per 64 rows up to one per CU: every CU streams,
// and the final sum reads at most 256 partials per column.
constexpr int kMlpBwdBlock = 512;
constexpr int kMlpBwdMaxG = 256;
template <int C, int A>
__global__ void __launch_bounds__(kMlpBwdBlock) mlp_tanh_bwd_kernel(long long K, long long rows_per_block,
                                                                 const float* __restrict__ dh,
                                                                 const float* __restrict__ dout,
                                                                 const float* __restrict__ w3,
                                                                 const float* __restrict__ h, float* __restrict__ dz,
                                                                 float* __restrict__ partial) {
  constexpr int N = 64 * C, P = N * (1 + A) + A, W = kMlpBwdBlock / 64;
  __shared__ float lds[W][P];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float w[A > 0 ? A : 1][C];
  for (int a = 0; a < A; ++a) ld_row<C>(w3 + (size_t)a * N + lane * C, w[a]);
  float sdb[C] = {}, sdw[A > 0 ? A : 1][C] = {}, sdb3[A > 0 ? A : 1] = {};
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = r0 + rows_per_block < K ? r0 + rows_per_block : K;
  for (long long r = r0 + wv; r < r1; r += W) {
    float hv[C], g[C];
    ld_row<C>(h + r * N + lane * C, hv);
    float dv[A > 0 ? A : 1];
    if constexpr (A > 0) {
#pragma unroll
      for (int a = 0; a < A; ++a) dv[a] = dout[r * A + a];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float t = 0.f;
#pragma unroll
        for (int a = 0; a < A; ++a) t += dv[a] * w[a][c];
        g[c] = t;
      }
    } else {
      ld_row<C>(dh + r * N + lane * C, g);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      g[c] = g[c] * (1.0f - hv[c] * hv[c]);   // tanh_backward: grad·(1 − y²)
      sdb[c] += g[c];
    }
    st_row<C>(dz + r * N + lane * C, g);
    if constexpr (A > 0) {
#pragma unroll
      for (int a = 0; a < A; ++a) {
#pragma unroll
        for (int c = 0; c < C; ++c) sdw[a][c] += dv[a] * hv[c];
        sdb3[a] += dv[a];
      }
    }
  }
  // waves → block partial, in wave order
#pragma unroll
  for (int c = 0; c < C; ++c) lds[wv][lane * C + c] = sdb[c];
  if constexpr (A > 0) {
#pragma unroll
    for (int a = 0; a < A; ++a) {
#pragma unroll
      for (int c = 0; c < C; ++c) lds[wv][N + a * N + lane * C + c] = sdw[a][c];
      if (lane == 0) lds[wv][N * (1 + A) + a] = sdb3[a];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < P; j += kMlpBwdBlock) {
    float t = lds[0][j];
    for (int k = 1; k < W; ++k) t += lds[k][j];
    partial[(size_t)blockIdx.x * P + j] = t;
  }
}

// dst segments: [0, n0) → d0, [n0, n0+n1) → d1, [n0+n1, P) → d2; d += Σ_g partial[g][j].
// A block owns 64 columns; its 16 waves sum interleaved slices of g (g ≡ w mod 16),
// combined in wave order — a fixed order for a given G.
constexpr int kMlpSumBlock = 1024;
__global__ void __launch_bounds__(kMlpSumBlock) mlp_sum_partials_kernel(int G, long long P,
                                                                        const float* __restrict__ partial, float* d0,
                                                                        long long n0, float* d1, long long n1,
                                                                        float* d2) {
  constexpr int W = kMlpSumBlock / 64;
  __shared__ float lds[W][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long j = (long long)blockIdx.x * 64 + lane;
  float t = 0.f;
  if (j < P) {
    int g = wv;
    for (; g + 3 * W < G; g += 4 * W) {   // four independent loads in flight
      const float a = partial[(size_t)g * P + j], b = partial[(size_t)(g + W) * P + j];
      const float c = partial[(size_t)(g + 2 * W) * P + j], d = partial[(size_t)(g + 3 * W) * P + j];
      t = (((t + a) + b) + c) + d;
    }
    for (; g < G; g += W) t += partial[(size_t)g * P + j];
  }
  lds[wv][lane] = t;
  __syncthreads();
  if (wv != 0 || j >= P) return;
  t = lds[0][lane];
  for (int k = 1; k < W; ++k) t += lds[k][lane];
  float* dst = j < n0 ? d0 + j : (j < n0 + n1 ? d1 + (j - n0) : d2 + (j - n0 - n1));
  *dst += t;
}

// Several partial-sum reductions in one launch (the bias and weight-gradient
// sums of a whole minibatch backward): blocks [start[i], start[i+1]) serve task i.
constexpr int kMlpMaxTasks = 16;
struct MlpSumTask {
  const float* partial;
  float* d0;
  float* d1;
  float* d2;
  long long P, n0, n1;
  int G;
};
struct MlpSumTasks {
  MlpSumTask t[kMlpMaxTasks];
  int start[kMlpMaxTasks + 1];
  int n;
};
struct SegOf {
  int s[kMlpMaxTasks];   // the Adam segment of each task's destination
};
constexpr int kMlpSumCols = 4;
// a task of at least this many partial rows (the fused kernels' per-tile bias
// rows: 2 048 at C3) takes one column per lane and 32 rows in flight, so its
// slices finish in 4 batches instead of 16 (the same per-column order)
#ifndef QS_SUM_TALL_G
#define QS_SUM_TALL_G 512   // dev builds probe other thresholds
#endif
constexpr int kMlpSumTallG = QS_SUM_TALL_G;
__host__ __device__ __forceinline__ int mlp_sum_cols(int G) { return G >= kMlpSumTallG ? 1 : kMlpSumCols; }
__device__ __forceinline__ int mlp_sum_wg(int G) {
  int w = 1;
  while (w < G && w < 16) w <<= 1;
  return w;
}
// fin(ti, dst, u, pv): the block's result u for a column of task ti (dst its
// destination element); pv = pre(ti, dst), issued by the finishing waves before
// their partial-row loads so that its memory latency overlaps theirs
template <int C, int U, class Fin, class Pre>
__device__ __forceinline__ void mlp_sum_body(const MlpSumTasks& tasks, int ti, float (*lds)[64 * kMlpSumCols], Fin fin,
                                             Pre pre) {
  constexpr int W = kMlpSumBlock / 64;
  const MlpSumTask& T = tasks.t[ti];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int Wg = mlp_sum_wg(T.G), ws = wv % Wg, cg = wv / Wg;
  const long long c0 = ((long long)(blockIdx.x - tasks.start[ti]) * (W / Wg) + cg) * (64 * C) + lane;
  auto dst_of = [&](long long c) {
    return c < T.n0 ? T.d0 + c : (c < T.n0 + T.n1 ? T.d1 + (c - T.n0) : T.d2 + (c - T.n0 - T.n1));
  };
  decltype(pre(0, (float*)nullptr)) pv[C];
  if (ws == 0)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const long long c = c0 + 64 * j;
      if (c < T.P) pv[j] = pre(ti, dst_of(c));
    }
  float t[C];
#pragma unroll
  for (int j = 0; j < C; ++j) t[j] = 0.f;
  int g = ws;
  for (; g + (U - 1) * Wg < T.G; g += U * Wg) {   // U rows' loads in flight per column
    float v[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const long long c = c0 + 64 * j;
        v[u][j] = c < T.P ? T.partial[(size_t)(g + u * Wg) * T.P + c] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j) t[j] += v[u][j];
  }
  for (; g < T.G; g += Wg)
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const long long c = c0 + 64 * j;
      if (c < T.P) t[j] += T.partial[(size_t)g * T.P + c];
    }
#pragma unroll
  for (int j = 0; j < C; ++j) lds[wv][lane + 64 * j] = t[j];
  __syncthreads();
  if (ws != 0) return;
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const long long c = c0 + 64 * j;
    if (c >= T.P) continue;
    float u = lds[cg * Wg][lane + 64 * j];
    for (int k = 1; k < Wg; ++k) u += lds[cg * Wg + k][lane + 64 * j];
    fin(ti, dst_of(c), u, pv[j]);
  }
}

// A block is 16 waves; a task's G partial rows are split over Wg = min(16,
// pow2 ≥ G) wave slices (wave slice w sums rows g ≡ w mod Wg in order), and
// the 16 / Wg wave groups of the block take 64·C-column spans (lane l: columns
// l + 64j, j < C — every load a coalesced 256-B wave access).  The slices are
// combined in slice order: per column the same fixed order as
// mlp_sum_partials_kernel (rows g ≡ w mod 16 in order, then w = 0..15), so
// both give the same bits.
template <class Fin, class Pre>
__device__ __forceinline__ void mlp_sum_block(const MlpSumTasks& tasks, Fin fin, Pre pre) {
  __shared__ float lds[kMlpSumBlock / 64][64 * kMlpSumCols];
  int ti = 0;
  while (ti + 1 < tasks.n && (int)blockIdx.x >= tasks.start[ti + 1]) ++ti;
  if (mlp_sum_cols(tasks.t[ti].G) == 1) mlp_sum_body<1, 32>(tasks, ti, lds, fin, pre);
  else mlp_sum_body<kMlpSumCols, 8>(tasks, ti, lds, fin, pre);
}

__global__ void __launch_bounds__(kMlpSumBlock) mlp_sum_multi_kernel(MlpSumTasks tasks) {
  mlp_sum_block(tasks, [](int, float* dst, float u, float pv) { *dst = pv + u; },
                [](int, float* dst) { return *dst; });
}

// torch.optim.Adam step and its step-count commit in one launch: every block
// reads the count first; the last block to finish increments it (gate permitting).
__global__ void adam_step_kernel(long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, float* step, float lr, float b1, float b2, float eps,
                                 const float* gate_val, float gate_thr, unsigned* done) {
  __shared__ bool last;
  if (gate_ok(gate_val, gate_thr)) {
    const double t = (double)(*step) + 1.0;
    const float bc1 = (float)(1.0 - pow((double)b1, t));
    const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, t));
    const float step_size = lr / bc1;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
      const float gi = g[i];
      float mi = m[i];
      mi = mi + (1.0f - b1) * (gi - mi);
      float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      const float denom = sqrtf(vi) / bc2_sqrt + eps;
      p[i] = p[i] - step_size * (mi / denom);
    }
  }
  __syncthreads();
  // no fence: nothing is handed over but the arrival count (every block read
  // *step before counting itself; p/m/v are read by later launches only)
  if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *done = 0;
    if (gate_ok(gate_val, gate_thr)) *step = *step + 1.0f;
  }
}

// ------------------------------------------------ fused 256-wide tanh MLP (MFMA)
// The reference MLP (neural_networks.py:18-54) with two tanh hidden layers of
// N = 256 and a linear head of A <= 4 outputs, on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32 FMA chains at the fp32 rate), for the
// large batches of the actor update (>= 512 tiles of 32 rows).
//
// Transposed, register-resident formulation.  A tile is 32 rows (batch
// samples) r; the kernels compute Zᵀ = W·Xᵀ so that a 32×32 accumulator holds
// hidden units m on its 16 registers and samples r on its lanes (C/D map:
// lane l = 32h + c holds column c and rows (i & 3) + 8 (i >> 2) + 4h of
// register i).  That is exactly the B-operand map of the next product, which
// sums over the hidden index (B[k][col]: lane 32h + c supplies column c and
// k-slot h), so tanh(Z1ᵀ + b1) feeds layer 2 straight from registers: no LDS
// round trip for the activations, no transposes.  The weights are the A
// operands: qs_mlp3_pack lays them out in MFMA-step order (lane-contiguous
// float4 = 4 steps), and a workgroup of 4 waves (4 tiles) streams them through
// a double-buffered 16-KB LDS window, one chunk = 64 MFMA steps of every wave.
// Hᵀ and dZᵀ are stored [N][K] (a register store is two 128-B row segments).
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kM3N = 256;       // hidden width of the fused path
constexpr int kM3NB = 8;        // 32-wide hidden blocks
constexpr int kM3Steps2 = 128;  // MFMA steps of a 256-deep contraction (2 k per step)
constexpr int kM3ChunkF = 8192; // floats per streamed chunk (32 KB = 128 steps x 64 lanes)
constexpr int kM3Waves = 4;     // waves (tiles) per workgroup
constexpr int kM3Block = 64 * kM3Waves;

__device__ __forceinline__ int m3_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }   // C/D row of reg i
__device__ __forceinline__ int m3_ip(int I) { return (I + 31) & ~31; }   // padded input width: whole groups of 4 k-quads

// Raw buffer access: lanes past the batch get offset kM3OOB, which the
// hardware drops on stores and reads as 0 — no per-element branches.
constexpr unsigned kM3OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t m3_rsrc(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float m3_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void m3_st(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, 0);
}

// tanh as 1 − 2/(e^{2x} + 1) with the hardware exp2 and rcp: five VALU
// instructions, no branches, saturates to ±1; absolute error a few 1e-7
// (fp32 rounding level of the activations).
__device__ __forceinline__ float m3_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);   // e^{2x}
  return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

// Σ over the 32 lanes of each half-wave, for each of the 16 registers:
// returns in lane 32h + c the sum of register j = 8b4 + 4b3 + 2b2 + b1 (b = bits of c).
__device__ __forceinline__ float m3_lane_sum16(const float* v) {
  const int c = threadIdx.x & 31;
  float a8[8], a4[4], a2[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool up = c & 16;
    const float keep = up ? v[j + 8] : v[j], send = up ? v[j] : v[j + 8];
    a8[j] = keep + __shfl_xor(send, 16, 64);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool up = c & 8;
    const float keep = up ? a8[j + 4] : a8[j], send = up ? a8[j] : a8[j + 4];
    a4[j] = keep + __shfl_xor(send, 8, 64);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool up = c & 4;
    const float keep = up ? a4[j + 2] : a4[j], send = up ? a4[j] : a4[j + 2];
    a2[j] = keep + __shfl_xor(send, 4, 64);
  }
  const bool up = c & 2;
  const float t = (up ? a2[1] : a2[0]) + __shfl_xor(up ? a2[0] : a2[1], 2, 64);
  return t + __shfl_xor(t, 1, 64);
}
__device__ __forceinline__ int m3_lane_sum16_reg() {
  const int c = threadIdx.x & 31;
  return 8 * ((c >> 4) & 1) + 4 * ((c >> 3) & 1) + 2 * ((c >> 2) & 1) + ((c >> 1) & 1);
}

// Packed weights (float offsets; qs_mlp3_pack_floats):
//   W1p  [Ip/8 q][8 mb][64 lane][4]: step s = 4q + e, lane 32h + c → W1[32mb + c][2s + h]
//   W2p  [8 mb][32 q][64][4]:  step s = 16 nb + i → W2[32mb + c][32nb + row(i, h)]
//   W2Tp [8 nb][32 q][64][4]:  step s = 16 mb + i → W2[32mb + row(i, h)][32nb + c]
__device__ __forceinline__ size_t m3_w1p_floats(int Ip) { return (size_t)(Ip / 8) * kM3NB * 256; }
__device__ __forceinline__ size_t m3_w2_floats() { return (size_t)kM3NB * 32 * 256; }

__global__ void mlp3_pack_kernel(int I, const float* __restrict__ W1, const float* __restrict__ W2,
                                 float* __restrict__ pack) {
  const int Ip = m3_ip(I);
  const size_t n1 = m3_w1p_floats(Ip), n2 = m3_w2_floats();
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n1 + 2 * n2; t += (size_t)gridDim.x * blockDim.x) {
    const size_t u = t < n1 ? t : (t < n1 + n2 ? t - n1 : t - n1 - n2);
    const int e = u & 3, lane = (u >> 2) & 63, c = lane & 31, h = lane >> 5;
    const size_t rest = u >> 8;
    float v;
    if (t < n1) {
      const int mb = rest % kM3NB, q = rest / kM3NB, k = 2 * (4 * q + e) + h;
      v = k < I ? W1[(size_t)(32 * mb + c) * I + k] : 0.f;
    } else {
      const int q = rest % 32, blk = rest / 32, st = 4 * q + e, i = st & 15, other = st >> 4;
      if (t < n1 + n2) v = W2[(size_t)(32 * blk + c) * kM3N + 32 * other + m3_row(i, h)];   // blk = mb, other = nb
      else v = W2[(size_t)(32 * other + m3_row(i, h)) * kM3N + 32 * blk + c];               // blk = nb, other = mb
    }
    pack[t] = v;
  }
}

// Double-buffered chunk stream: the workgroup's 256 threads load a 32-KB chunk
// of `src` into registers one chunk ahead of its LDS write, and every wave
// consumes chunk c from buf[c & 1] after the barrier that makes it visible.
struct M3Stream {
  const float4* src;
  float4* buf;   // LDS [2][kM3ChunkF / 4]
  float4 st[kM3ChunkF / 4 / kM3Block];
  __device__ __forceinline__ void load(int c) {
#pragma unroll
    for (int j = 0; j < kM3ChunkF / 4 / kM3Block; ++j) st[j] = src[(size_t)c * (kM3ChunkF / 4) + j * kM3Block + threadIdx.x];
  }
  __device__ __forceinline__ void store(int c) {
#pragma unroll
    for (int j = 0; j < kM3ChunkF / 4 / kM3Block; ++j) buf[(c & 1) * (kM3ChunkF / 4) + j * kM3Block + threadIdx.x] = st[j];
  }
  // LDS-only fences around a plain barrier: the LDS writes are complete and
  // ordered, but the next chunk's global loads stay in flight (a full
  // __syncthreads would drain vmcnt)
  __device__ __forceinline__ static void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
};

// Stream `n` chunks: body(c, chunk) with chunk = the LDS float4 window of chunk c.
template <class Body>
__device__ __forceinline__ void m3_stream(M3Stream& S, int n, Body body) {
  S.load(0);
  S.store(0);
  if (n > 1) S.load(1);
  for (int c = 0; c < n; ++c) {
    M3Stream::sync();
    if (c + 1 < n) S.store(c + 1);
    if (c + 2 < n) S.load(c + 2);
    body(c, S.buf + (c & 1) * (kM3ChunkF / 4));
  }
  M3Stream::sync();
}

// GATHER: batch row r is X row rows[r / G]·G + r % G (the minibatch's agent
// rows read straight from the rollout table, which may exceed a buffer
// descriptor's 4-GB range: plain 64-bit loads)
template <int A, bool GATHER = false>
__global__ void __launch_bounds__(kM3Block) mlp3_fwd_kernel(long long K, int I, const float* __restrict__ X,
                                                            const float* __restrict__ pack, const float* __restrict__ b1,
                                                            const float* __restrict__ b2, const float* __restrict__ W3,
                                                            const float* __restrict__ b3, float* __restrict__ H1T,
                                                            float* __restrict__ H2T, float* __restrict__ out,
                                                            const long long* __restrict__ rows = nullptr, int G = 1) {
  __shared__ float4 wbuf[2 * kM3ChunkF / 4];
  __shared__ float sb1[kM3N], sb2[kM3N], sw3[A * kM3N];   // biases and head weights, read in the epilogues
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long long r = ((long long)blockIdx.x * kM3Waves + w) * 32 + c;
  const bool rv = r < K;
  const int Ip = m3_ip(I);
  for (int j = threadIdx.x; j < kM3N; j += kM3Block) { sb1[j] = b1[j]; sb2[j] = b2[j]; }
  for (int j = threadIdx.x; j < A * kM3N; j += kM3Block) sw3[j] = W3[j];
  // H1T / H2T may be NULL (inference): a zero-size descriptor drops every store
  const float* xrow = X;
  if constexpr (GATHER) xrow = rv ? X + (rows[r / G] * G + r % G) * (long long)I : X;
  const __amdgpu_buffer_rsrc_t xr = m3_rsrc(X, GATHER ? 0 : (size_t)K * I * 4),
                               h1r = m3_rsrc(H1T, H1T ? (size_t)K * kM3N * 4 : 0),
                               h2r = m3_rsrc(H2T, H2T ? (size_t)K * kM3N * 4 : 0);
  const unsigned xoff = rv ? (unsigned)(r * I * 4) : kM3OOB, roff = rv ? (unsigned)(r * 4) : kM3OOB;
  const unsigned kstride = (unsigned)(K * 4);
  M3Stream S{reinterpret_cast<const float4*>(pack), wbuf};
  // layer 1: Z1ᵀ = W1·Xᵀ; chunk = 4 k-quads x 8 blocks; B = X[r][2s + h]
  f32x16 acc[kM3NB];
#pragma unroll
  for (int mb = 0; mb < kM3NB; ++mb) acc[mb] = f32x16{};
  m3_stream(S, Ip / 32, [&](int ch, const float4* wc) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int q = 4 * ch + qq;
      if (q >= Ip / 8) break;
      float xb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 2 * (4 * q + e) + h;
        if constexpr (GATHER) xb[e] = rv && k < I ? xrow[k] : 0.f;
        else xb[e] = m3_ld(xr, k < I ? xoff + 4u * k : kM3OOB);
      }
#pragma unroll
      for (int mb = 0; mb < kM3NB; ++mb) {
        const float4 wv = wc[(qq * kM3NB + mb) * 64 + lane];
        acc[mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, xb[0], acc[mb], 0, 0, 0);
        acc[mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, xb[1], acc[mb], 0, 0, 0);
        acc[mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, xb[2], acc[mb], 0, 0, 0);
        acc[mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, xb[3], acc[mb], 0, 0, 0);
      }
    }
  });
  // bias + tanh in the accumulators → H1ᵀ registers (the B operand of layer 2) and HBM
  float hb[kM3Steps2];
#pragma unroll
  for (int nb = 0; nb < kM3NB; ++nb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 32 * nb + m3_row(i, h);
      const float v = m3_tanh(acc[nb][i] + sb1[m]);
      hb[nb * 16 + i] = v;
      m3_st(h1r, roff + (unsigned)m * kstride, v);
    }
  // layer 2: Z2ᵀ[mb] = W2[mb]·H1ᵀ, one chunk (128 steps) per block; the
  // epilogue of block mb − 1 (bias + tanh, H2ᵀ store, head) sits in block mb's
  // basic block, beside its MFMAs
  S.src = reinterpret_cast<const float4*>(pack + m3_w1p_floats(Ip));
  float hs[A];
#pragma unroll
  for (int a = 0; a < A; ++a) hs[a] = 0.f;
  f32x16 zp = f32x16{};
  auto epi2 = [&](int mb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 32 * mb + m3_row(i, h);
      const float v = m3_tanh(zp[i] + sb2[m]);
      m3_st(h2r, roff + (unsigned)m * kstride, v);
#pragma unroll
      for (int a = 0; a < A; ++a) hs[a] += v * sw3[a * kM3N + m];
    }
  };
  m3_stream(S, kM3NB, [&](int mb, const float4* wc) {
    f32x16 z = f32x16{};
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const float4 wv = wc[q * 64 + lane];
      z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, hb[4 * q + 0], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, hb[4 * q + 1], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, hb[4 * q + 2], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, hb[4 * q + 3], z, 0, 0, 0);
      if (q == 0 && mb > 0) epi2(mb - 1);
    }
    zp = z;
  });
  epi2(kM3NB - 1);
  // head: out[r][a] = Σ_m H2ᵀ[m][r]·W3[a][m] + b3[a] (the two halves hold the two m sets)
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float t = hs[a] + __shfl_xor(hs[a], 32, 64);
    if (h == 0 && rv) out[r * A + a] = t + b3[a];
  }
}

// partA[tile][N + A·N + A] = [Σ_r dZ2ᵀ | Σ_r dout_a·H2ᵀ | Σ_r dout_a], partB[tile][N] = Σ_r dZ1ᵀ.
template <int A>
__global__ void __launch_bounds__(kM3Block) mlp3_bwd_kernel(long long K, const float* __restrict__ dout,
                                                            const float* __restrict__ H1T, const float* __restrict__ H2T,
                                                            const float* __restrict__ pack, int Ip,
                                                            const float* __restrict__ W3, float* __restrict__ dZ2T,
                                                            float* __restrict__ dZ1T, float* __restrict__ partA,
                                                            float* __restrict__ partB) {
  constexpr int N = kM3N, PA = N + A * N + A;
  __shared__ float4 wbuf[2 * kM3ChunkF / 4];
  __shared__ float sw3[A * kM3N];
  __shared__ float spa[kM3Waves][PA], spb[kM3Waves][N];   // per-wave (tile) partials, combined per workgroup
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long long tile = (long long)blockIdx.x * kM3Waves + w;
  const long long r = tile * 32 + c;
  const bool rv = r < K;
  for (int j = threadIdx.x; j < A * kM3N; j += kM3Block) sw3[j] = W3[j];
  const size_t hbytes = (size_t)K * kM3N * 4;
  const __amdgpu_buffer_rsrc_t h1r = m3_rsrc(H1T, hbytes), h2r = m3_rsrc(H2T, hbytes), z2r = m3_rsrc(dZ2T, hbytes),
                               z1r = m3_rsrc(dZ1T, hbytes);
  const unsigned roff = rv ? (unsigned)(r * 4) : kM3OOB, kstride = (unsigned)(K * 4);
  float dv[A];
#pragma unroll
  for (int a = 0; a < A; ++a) dv[a] = rv ? dout[r * A + a] : 0.f;
  float* pa = spa[w];
  const int jr = m3_lane_sum16_reg();
#pragma unroll
  for (int a = 0; a < A; ++a) {   // Σ_r dout_a over the tile (half 0 holds the 32 rows)
    float t = h == 0 ? dv[a] : 0.f;
    for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) pa[N + A * N + a] = t;
  }
  // 1. dZ2ᵀ = (W3ᵀ·doutᵀ) ⊙ (1 − H2ᵀ²) in registers (the B operand of dH1ᵀ); bias / head partials
  float zb[kM3Steps2];
#pragma unroll
  for (int mb = 0; mb < kM3NB; ++mb) {
    float hw[A][16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 32 * mb + m3_row(i, h);
      const float hv = m3_ld(h2r, roff + (unsigned)m * kstride);
      float g = 0.f;
#pragma unroll
      for (int a = 0; a < A; ++a) { g += dv[a] * sw3[a * N + m]; hw[a][i] = dv[a] * hv; }
      const float zz = g * (1.f - hv * hv);
      zb[mb * 16 + i] = zz;
      m3_st(z2r, roff + (unsigned)m * kstride, zz);
    }
    const float sdb = m3_lane_sum16(zb + mb * 16);
    float sdw[A];
#pragma unroll
    for (int a = 0; a < A; ++a) sdw[a] = m3_lane_sum16(hw[a]);
    if ((c & 1) == 0) {   // tiles past K write zeros: every partial row is defined
      const int m = 32 * mb + m3_row(jr, h);
      pa[m] = sdb;
#pragma unroll
      for (int a = 0; a < A; ++a) pa[N + a * N + m] = sdw[a];
    }
  }
  // 2. dH1ᵀ[nb] = (W2ᵀ)[nb]·dZ2ᵀ, one chunk per block; the epilogue of block
  // nb − 1 (dZ1ᵀ = dH1ᵀ ⊙ (1 − H1ᵀ²), store, Σ_r) beside block nb's MFMAs
  M3Stream S{reinterpret_cast<const float4*>(pack + m3_w1p_floats(Ip) + m3_w2_floats()), wbuf};
  // H1ᵀ of block nb is loaded at the start of block nb and used one block later
  // (the epilogue's loads never stall the MFMA chain)
  f32x16 dp = f32x16{};
  float h1p[16], h1n[16];
  auto epi1 = [&](int nb) {
    float z1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = 32 * nb + m3_row(i, h);
      z1[i] = dp[i] * (1.f - h1p[i] * h1p[i]);
      m3_st(z1r, roff + (unsigned)n * kstride, z1[i]);
    }
    const float sdb = m3_lane_sum16(z1);
    if ((c & 1) == 0) spb[w][32 * nb + m3_row(jr, h)] = sdb;
  };
  m3_stream(S, kM3NB, [&](int nb, const float4* wc) {
#pragma unroll
    for (int i = 0; i < 16; ++i) h1n[i] = m3_ld(h1r, roff + (unsigned)(32 * nb + m3_row(i, h)) * kstride);
    f32x16 d = f32x16{};
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const float4 wv = wc[q * 64 + lane];
      d = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, zb[4 * q + 0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, zb[4 * q + 1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, zb[4 * q + 2], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, zb[4 * q + 3], d, 0, 0, 0);
      if (q == 16 && nb > 0) epi1(nb - 1);
    }
    dp = d;
#pragma unroll
    for (int i = 0; i < 16; ++i) h1p[i] = h1n[i];
  });
  epi1(kM3NB - 1);
  // the workgroup's four tiles → one partial row, waves in order (a fixed summation order)
  __syncthreads();
  for (int j = threadIdx.x; j < PA; j += kM3Block)
    partA[(size_t)blockIdx.x * PA + j] = ((spa[0][j] + spa[1][j]) + spa[2][j]) + spa[3][j];
  for (int j = threadIdx.x; j < N; j += kM3Block)
    partB[(size_t)blockIdx.x * N + j] = ((spb[0][j] + spb[1][j]) + spb[2][j]) + spb[3][j];
}


// ---------------------------------------------------------------- fused actor
// One launch per PPO minibatch for the shared actor (MLPActor AG:87-148 with
// the PPO policy loss AG:602-640): forward, the per-row loss head and the
// backward of every 16-row tile, with the activations of a tile kept in
// registers from the first layer to the last gradient.
//
// Tiles of 16 batch rows on v_mfma_f32_16x16x4_f32, activations transposed
// (hidden × rows): lane (g, j) of a wave (j = lane & 15, g = lane >> 4) holds
// hidden units 16·b + 4g + r (r = 0..3) of row j in the C registers of block b.
// Those registers are exactly the B operand of the next contraction over the
// hidden index (step (b, r): lane group g supplies hidden 16b + 4g + r), so
// tanh(Z1ᵀ) feeds layer 2, H2ᵀ feeds the head and dZ2ᵀ feeds dH1ᵀ = W2ᵀ·dZ2ᵀ
// without an LDS round trip.  A wave holds H1ᵀ (64 VGPRs) and H2ᵀ → dZ2ᵀ (64)
// of its tile: under 256 registers, so two waves share each SIMD — one wave's
// epilogues, loss head and barrier waits hide behind the other's MFMAs.
//
// A workgroup = 8 waves = 128 rows.  The weights (packed in MFMA-step order by
// qs_mlp3f_pack: W1f, W2f, W2b) stream through a double-buffered 32-KB LDS
// window shared by the 8 waves.  The loss head is ppo_heads_kernel's
// arithmetic per row; per-row inputs are read by index (the minibatch's
// env-timesteps, D agent rows each, straight from the rollout table).
// Outputs: H1, dZ2, dZ1 row-major [K][256] (the weight-gradient GEMMs' operands,
// written as 16-byte stores: four times fewer store instructions than a
// transposed [256][K] image, whose stores bound the epilogues),
// the gathered inputs Xa [K][I], per-workgroup partial rows of the bias / head
// gradients, and — from the last workgroup, in workgroup order — approx_kl,
// d logstd and the loss statistics.
constexpr int kFWaves = 8;
constexpr int kFBlock = 64 * kFWaves;
constexpr int kFChunkF = 8192;                   // floats per streamed chunk (32 KB)
constexpr int kFStage = kFChunkF / 4 / kFBlock;  // float4 per thread per chunk
constexpr int kFMaxIp = 128;                     // input width bound of the fused path
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int f16_ip(int I) { return (I + 31) & ~31; }
__host__ __device__ constexpr long long f16_w1_floats(int Ip) { return 256LL * Ip; }
constexpr long long kFW2Floats = 65536;

// pack positions: W1f[q][ob][lane][e] = W1[16ob + (l&15)][16q + 4e + (l>>4)],
// W2f[ob][ib][lane][e] = W2[16ob + (l&15)][16ib + 4(l>>4) + e],
// W2b[ib][ob][lane][e] = W2[16ob + 4(l>>4) + e][16ib + (l&15)]
__device__ __forceinline__ long long f16_pos_w1(int m, int k) {
  const int kk = k & 15;
  return ((((long long)(k >> 4) * 16 + (m >> 4)) * 64 + 16 * (kk & 3) + (m & 15)) << 2) + (kk >> 2);
}
__device__ __forceinline__ long long f16_pos_w2f(int m, int n) {
  const int nn = n & 15;
  return ((((long long)(m >> 4) * 16 + (n >> 4)) * 64 + 16 * (nn >> 2) + (m & 15)) << 2) + (nn & 3);
}
__device__ __forceinline__ long long f16_pos_w2b(int m, int n) {
  const int mm = m & 15;
  return ((((long long)(n >> 4) * 16 + (m >> 4)) * 64 + 16 * (mm >> 2) + (n & 15)) << 2) + (mm & 3);
}

__global__ void mlp3f_pack_kernel(int I, const float* __restrict__ W1, const float* __restrict__ W2,
                                  float* __restrict__ pack) {
  const int Ip = f16_ip(I);
  const long long n1 = f16_w1_floats(Ip);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n1 + 2 * kFW2Floats;
       t += (long long)gridDim.x * blockDim.x) {
    // invert the position maps: t → (lane, e, block indices)
    const long long u = t < n1 ? t : (t < n1 + kFW2Floats ? t - n1 : t - n1 - kFW2Floats);
    const int e = (int)(u & 3), l = (int)((u >> 2) & 63), jl = l & 15, gl = l >> 4;
    const long long rest = u >> 8;
    float v;
    if (t < n1) {
      const int ob = (int)(rest & 15), q = (int)(rest >> 4), k = 16 * q + 4 * e + gl;
      v = k < I ? W1[(size_t)(16 * ob + jl) * I + k] : 0.f;
    } else {
      const int lo = (int)(rest & 15), hi = (int)(rest >> 4);
      if (t < n1 + kFW2Floats) v = W2[(size_t)(16 * hi + jl) * kM3N + 16 * lo + 4 * gl + e];   // W2f: hi = ob, lo = ib
      else v = W2[(size_t)(16 * lo + 4 * gl + e) * kM3N + 16 * hi + jl];                      // W2b: hi = ib, lo = ob
    }
    pack[t] = v;
  }
}

// Double-buffered chunk stream for 512 threads (M3Stream's scheme: register
// staging one chunk ahead of its LDS write, LDS-only fences around the barrier)
struct FStream {
  const float4* src;
  float4* buf;   // LDS [2][kFChunkF / 4]
  float4 st[kFStage];
  __device__ __forceinline__ void load(int c) {
#pragma unroll
    for (int j = 0; j < kFStage; ++j) st[j] = src[(size_t)c * (kFChunkF / 4) + j * kFBlock + threadIdx.x];
  }
  __device__ __forceinline__ void store(int c) {
#pragma unroll
    for (int j = 0; j < kFStage; ++j) buf[(c & 1) * (kFChunkF / 4) + j * kFBlock + threadIdx.x] = st[j];
  }
};

// n chunks (compile-time N when > 0, so that the body's register arrays are
// indexed statically); body(c, chunk window)
template <int N, class Body>
__device__ __forceinline__ void f_stream(FStream& S, int n, Body body) {
  if constexpr (N > 0) n = N;
  S.load(0);
  S.store(0);
  if (n > 1) S.load(1);
  auto step = [&](int c) {
    M3Stream::sync();
    if (c + 1 < n) S.store(c + 1);
    if (c + 2 < n) S.load(c + 2);
    body(c, S.buf + (c & 1) * (kFChunkF / 4));
  };
  if constexpr (N > 0) {
#pragma unroll
    for (int c = 0; c < N; ++c) step(c);
  } else {
#pragma unroll 1
    for (int c = 0; c < n; ++c) step(c);
  }
  M3Stream::sync();
}

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Σ over the 16 lanes of each lane group of 64 values v[x] (x = 4·b + r):
// a transposing butterfly (60 shuffles); lane j of the group ends with the
// sums of x = 4j + i in out[i], i = 0..3.  Fixed order: replays are bit-identical.
template <class V>
__device__ __forceinline__ void f_lane_sum64(V v, float (&out)[4]) {
  const int j = threadIdx.x & 15;
  float a[32], b[16], c[8];
  {
    const bool up = j & 8;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const float keep = up ? v(i + 32) : v(i), send = up ? v(i) : v(i + 32);
      a[i] = keep + __shfl_xor(send, 8, 64);
    }
  }
  {
    const bool up = j & 4;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float keep = up ? a[i + 16] : a[i], send = up ? a[i] : a[i + 16];
      b[i] = keep + __shfl_xor(send, 4, 64);
    }
  }
  {
    const bool up = j & 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float keep = up ? b[i + 8] : b[i], send = up ? b[i] : b[i + 8];
      c[i] = keep + __shfl_xor(send, 2, 64);
    }
  }
  const bool up = j & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float keep = up ? c[i + 4] : c[i], send = up ? c[i] : c[i + 4];
    out[i] = keep + __shfl_xor(send, 1, 64);
  }
}

// Σ over the 16 lanes of a lane group of a block's four C registers v[r] (hidden
// 16b + 4g + r): a transposing butterfly (5 shuffles); lane j gets the sum for
// r = 2·bit3(j) + bit2(j) (lanes differing in bits 0-1 hold the same value).
// Fixed order: replays are bit-identical.
// Lane exchanges within a 16-lane DPP row (VALU moves, no LDS pipe): the value of
// lane j ^ 8, j ^ 4 (row_shl:4 into banks 0 and 2, row_shr:4 into banks 1 and 3),
// j ^ 2, j ^ 1 (quad permutes).
template <int CTRL, int BANKS = 0xF>
__device__ __forceinline__ float f_dpp(float v, float old = 0.f) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, BANKS, false));
}
__device__ __forceinline__ float f_x8(float v) { return f_dpp<0x128>(v); }   // row_ror:8
__device__ __forceinline__ float f_x4(float v) { return f_dpp<0x114, 0xA>(v, f_dpp<0x104, 0x5>(v)); }
__device__ __forceinline__ float f_x2(float v) { return f_dpp<0x4E>(v); }    // quad_perm [2,3,0,1]
__device__ __forceinline__ float f_x1(float v) { return f_dpp<0xB1>(v); }    // quad_perm [1,0,3,2]
// Σ over the 16 lanes of a row, in every lane
__device__ __forceinline__ float f_row_sum(float t) {
  t += f_x8(t);
  t += f_x4(t);
  t += f_x2(t);
  return t + f_x1(t);
}

__device__ __forceinline__ float f_blk_sum(const float (&v)[4]) {
  const int j = threadIdx.x & 15;
  const bool u8 = j & 8, u4 = j & 4;
  const float a0 = (u8 ? v[2] : v[0]) + f_x8(u8 ? v[0] : v[2]);
  const float a1 = (u8 ? v[3] : v[1]) + f_x8(u8 ? v[1] : v[3]);
  float b = (u4 ? a1 : a0) + f_x4(u4 ? a0 : a1);
  b += f_x2(b);
  return b + f_x1(b);
}

// LDS layout (floats) of the fused actor kernel; dynamic shared memory
__host__ __device__ constexpr int f_pa(int A) { return kM3N + A * kM3N + A; }   // b2 | W3[A] | b3[A]
__host__ __device__ constexpr int f_lds_floats(int A) {
  return 2 * kFChunkF + (2 + A) * kM3N + kFWaves * (f_pa(A) + kM3N);
}

// a lane's four C registers of one block (hidden 16b + 4g + r, r = 0..3, of its
// row) into a row-major [K][256] buffer: one 16-byte store, the lane's part in
// the VGPR offset and the block's 64·b bytes in soffset
typedef unsigned f_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void f_st4(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, const float (&v)[4]) {
#ifndef QS_F_NOSTORE   // dev probe: the kernel without its activation stores
  const f_u4 u = {__builtin_bit_cast(unsigned, v[0]), __builtin_bit_cast(unsigned, v[1]),
                  __builtin_bit_cast(unsigned, v[2]), __builtin_bit_cast(unsigned, v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, (int)voff, (int)soff, 0);
#endif
}

#ifdef QS_F_STAMP   // dev probe: per-wave phase timestamps (s_memtime) of the fused actor kernel
__device__ unsigned long long g_fstamp[4096 * 8];
#define F_STAMP(k) do { if ((threadIdx.x & 63) == 0) g_fstamp[((size_t)blockIdx.x * kFWaves + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define F_STAMP(k) do { } while (0)
#endif

template <int A>
__global__ void __launch_bounds__(kFBlock) mlp3f_actor_kernel(
    long long K, int I, int D, const float* __restrict__ X, const long long* __restrict__ idx,
    const float* __restrict__ pack, const float* __restrict__ b1, const float* __restrict__ b2,
    const float* __restrict__ W3, const float* __restrict__ b3, const float* __restrict__ logstd, float scale,
    const float* __restrict__ act, const float* __restrict__ logp_old, const double* __restrict__ adv, float clip,
    float ent_coef, float* __restrict__ Xa, float* __restrict__ H1T, float* __restrict__ dZ2T,
    float* __restrict__ dZ1T, float* __restrict__ partA, float* __restrict__ partB, double* __restrict__ lossp,
    float* __restrict__ dlogstd, float* __restrict__ kl_out, double* __restrict__ acc, unsigned* __restrict__ count,
    float* __restrict__ mean_out, float* __restrict__ partW1) {
  constexpr int N = kM3N, PA = f_pa(A), NL = 2 + A;   // loss sums: policy, approx_kl, d logstd[A]
  extern __shared__ float4 f_lds[];
  float* lf = reinterpret_cast<float*>(f_lds);
  float* sb1 = lf + 2 * kFChunkF;
  float* sb2 = sb1 + N;
  float* sw3 = sb2 + N;                 // [A][N]
  float* spa = sw3 + A * N;             // [waves][PA]
  float* spb = spa + kFWaves * PA;      // [waves][N]
  __shared__ double ldsn[kFWaves][NL];
  __shared__ bool last;
  F_STAMP(0);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, j = l & 15, g = l >> 4;
  const long long row = ((long long)blockIdx.x * kFWaves + w) * 16 + j;
  const bool rv = row < K;
  const int Ip = f16_ip(I);
  for (int t = tid; t < N; t += kFBlock) { sb1[t] = b1[t]; sb2[t] = b2[t]; }
  for (int t = tid; t < A * N; t += kFBlock) sw3[t] = W3[t];
  // the row's agent obs in the rollout table: env-timestep idx[row / D], agent row % D
  const long long ei = rv ? row / D : 0;
  const float* xrow = X + (rv ? (idx[ei] * D + (row - ei * D)) * (long long)I : 0);
  const size_t hbytes = (size_t)K * N * 4;
  const __amdgpu_buffer_rsrc_t h1r = m3_rsrc(H1T, hbytes), z2r = m3_rsrc(dZ2T, hbytes),
                               z1r = m3_rsrc(dZ1T, dZ1T ? hbytes : 0);   // NULL with partW1: no dZ1 stores
  // H1, dZ2, dZ1 are row-major [K][256]: a lane's block of four hidden units is 16 contiguous bytes
  const unsigned voff = rv ? (unsigned)((row * N + 4 * g) * 4) : kM3OOB;
  // One continuous chunk stream over the whole pack (W1f | W2f | W2b): chunk c + 2
  // is in flight while chunk c is consumed, across the phase boundaries too
  const int nW1 = Ip / 32, nC = nW1 + 16;
  FStream S{reinterpret_cast<const float4*>(pack), f_lds};
  auto next = [&](int c) -> const float4* {
    M3Stream::sync();
    if (c + 1 < nC) S.store(c + 1);
    if (c + 2 < nC) S.load(c + 2);
    return S.buf + (c & 1) * (kFChunkF / 4);
  };
  auto xload = [&](int ch, float (&xb)[8]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = 32 * ch + 4 * t + g;   // q = 2ch + (t >> 2), e = t & 3
      xb[t] = rv && k < I ? xrow[k] : 0.f;
    }
  };
  float xb[8];
  S.load(0);
  xload(0, xb);
  S.store(0);
  S.load(1);

  // ---- layer 1: Z1ᵀ = W1·Xᵀ, all 16 hidden blocks at once; step (q, e) contracts k = 16q + 4e + g
  f32x4 acc1[16];
#pragma unroll
  for (int b = 0; b < 16; ++b) acc1[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ch = 0; ch < nW1; ++ch) {
    const float4* wc = next(ch);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = 32 * ch + 4 * t + g;
      if (rv && k < I) Xa[row * I + k] = xb[t];
    }
    float xn[8];
    if (ch + 1 < nW1) xload(ch + 1, xn);
    float4 wv = wc[l];
#pragma unroll
    for (int u = 0; u < 32; ++u) {   // u = 16·qq + b
      const int qq = u >> 4, b = u & 15;
      float4 nx = wv;
      if (u + 1 < 32) nx = wc[(u + 1) * 64 + l];
      __builtin_amdgcn_sched_barrier(0);   // the next operand read stays one step ahead of these MFMAs
      acc1[b] = mfma16(wv.x, xb[4 * qq + 0], acc1[b]);
      acc1[b] = mfma16(wv.y, xb[4 * qq + 1], acc1[b]);
      acc1[b] = mfma16(wv.z, xb[4 * qq + 2], acc1[b]);
      acc1[b] = mfma16(wv.w, xb[4 * qq + 3], acc1[b]);
      wv = nx;
    }
    if (ch + 1 < nW1)
#pragma unroll
      for (int t = 0; t < 8; ++t) xb[t] = xn[t];
  }
  F_STAMP(1);
  // ---- layer 2: Z2ᵀ = W2·H1ᵀ, two output blocks per chunk (independent accumulators).
  // H1 = tanh(Z1ᵀ + b1) of block ib + 1 is formed and stored during step ib of the
  // first chunk: the epilogue runs beside the MFMAs instead of before them
  float h1[16][4];
  auto epi1 = [&](int b) {
#pragma unroll
    for (int r = 0; r < 4; ++r) h1[b][r] = m3_tanh(acc1[b][r] + sb1[16 * b + 4 * g + r]);
    f_st4(h1r, voff, 64u * b, h1[b]);
  };
  epi1(0);
  F_STAMP(2);
  float h2[16][4];
  float hs[A];
#pragma unroll
  for (int a = 0; a < A; ++a) hs[a] = 0.f;
  // the epilogue of chunk c's two blocks (bias + tanh, the head's partial dots) runs
  // during the first two steps of chunk c + 1
  f32x4 zp0 = f32x4{0.f, 0.f, 0.f, 0.f}, zp1 = zp0;
  auto epi2 = [&](int c, int half) {
    const f32x4& z = half ? zp1 : zp0;
    const int b = 2 * c + half;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hh = 16 * b + 4 * g + r;
      h2[b][r] = m3_tanh(z[r] + sb2[hh]);
#pragma unroll
      for (int a = 0; a < A; ++a) hs[a] += h2[b][r] * sw3[a * N + hh];
    }
  };
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float4* wc = next(nW1 + c);
    f32x4 z0 = f32x4{0.f, 0.f, 0.f, 0.f}, z1 = z0;
    float4 w0 = wc[l], w1 = wc[16 * 64 + l];
#pragma unroll
    for (int ib = 0; ib < 16; ++ib) {
      float4 n0 = w0, n1 = w1;
      if (ib + 1 < 16) { n0 = wc[(ib + 1) * 64 + l]; n1 = wc[(17 + ib) * 64 + l]; }
      __builtin_amdgcn_sched_barrier(0);
      if (c == 0 && ib + 1 < 16) epi1(ib + 1);
      if (c > 0 && ib < 2) epi2(c - 1, ib);
      z0 = mfma16(w0.x, h1[ib][0], z0);
      z1 = mfma16(w1.x, h1[ib][0], z1);
      z0 = mfma16(w0.y, h1[ib][1], z0);
      z1 = mfma16(w1.y, h1[ib][1], z1);
      z0 = mfma16(w0.z, h1[ib][2], z0);
      z1 = mfma16(w1.z, h1[ib][2], z1);
      z0 = mfma16(w0.w, h1[ib][3], z0);
      z1 = mfma16(w1.w, h1[ib][3], z1);
      w0 = n0;
      w1 = n1;
    }
    zp0 = z0;
    zp1 = z1;
  }
  epi2(7, 0);
  epi2(7, 1);

  F_STAMP(3);
  // ---- the loss head of row j (every lane group forms the same values; group 0 counts them)
  float dout[A];
  double ls[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) ls[k] = 0.0;
  {
    float sd[A], lsd[A], var2[A], mu[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      float t = hs[a] + __shfl_xor(hs[a], 16, 64);
      t = t + __shfl_xor(t, 32, 64);
      mu[a] = t + b3[a];
      sd[a] = expf(logstd[a]);
      lsd[a] = logf(sd[a]);
      var2[a] = 2.0f * (sd[a] * sd[a]);
    }
    if (mean_out && rv && g == 0)
#pragma unroll
      for (int a = 0; a < A; ++a) mean_out[row * A + a] = mu[a];
    const float lc = (float)log(sqrt(2.0 * M_PI));
    const float lo = 1.0f - clip, hi = 1.0f + clip;
    const double G = -1.0 / (double)K;
    const long long gi = rv ? idx[ei] * D + (row - ei * D) : 0;
    float t1[A], logp = 0.0f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float m = mu[a] * scale;
      t1[a] = (rv ? act[gi * A + a] : 0.f) - m;
      const float t4 = (float)((double)(-(t1[a] * t1[a])) / (double)var2[a]);
      const float lp = (t4 - lsd[a]) - lc;
      logp = a == 0 ? lp : logp + lp;
    }
    const float lpo = rv ? logp_old[gi] : 0.f;
    const float ratio = expf(logp - lpo);
    const double ad = rv ? adv[idx[ei]] : 0.0;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const double s1 = (double)ratio * ad, s2 = (double)rc * ad;
    const double g1 = s1 < s2 ? G : (s1 == s2 ? G / 2 : 0.0);
    const double g2 = s2 < s1 ? G : (s1 == s2 ? G / 2 : 0.0);
    float gr = (float)(g1 * ad);
    if (ratio >= lo && ratio <= hi) gr = gr + (float)(g2 * ad);
    const float gl = gr * ratio;
    const bool cnt = rv && g == 0;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float gt3 = (float)((double)gl / (double)var2[a]);
      const float gt1 = -gt3 * 2.0f * t1[a];
      dout[a] = rv ? -gt1 * scale : 0.f;
      if (cnt) ls[2 + a] = (double)gl * ((double)(t1[a] * t1[a]) / ((double)sd[a] * sd[a]) - 1.0);
    }
    if (cnt) {
      ls[0] = -(s1 < s2 ? s1 : s2);
      ls[1] = (double)(lpo - logp);
    }
  }

#ifdef QS_F_NOHEAD   // dev probe: a constant output gradient, no loss head
#pragma unroll
  for (int a = 0; a < A; ++a) dout[a] = 1e-3f;
#endif
  // ---- head and second-tanh backward, one hidden block at a time: its W3 partials
  // Σ_rows dout·H2, dZ2 = (dout·W3) ⊙ (1 − H2²) in place of H2 (stored), its b2
  // partial Σ_rows dZ2.  Block ob + 1 is prepared during step ob of the first
  // backward chunk, beside its MFMAs.  Row sums within a block: blk_sum.
  float* pa = spa + w * PA;
  const int rsel = 2 * ((j >> 3) & 1) + ((j >> 2) & 1);   // the hidden unit 16b + 4g + rsel a lane's block sum is for
  const bool wsum = (j & 3) == 0;                          // one lane per (g, rsel) writes it
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float t = f_row_sum(dout[a]);   // Σ_rows dout_a (every row holds the same dout)
    if (l == 0) pa[N + A * N + a] = t;
  }
  // W3 partials Σ_rows dout·H2 of every block (they need H2 before dZ2 replaces it)
#ifndef QS_F_NOHEAD
#pragma unroll
  for (int b = 0; b < 16; ++b)
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float p4[4] = {dout[a] * h2[b][0], dout[a] * h2[b][1], dout[a] * h2[b][2], dout[a] * h2[b][3]};
      const float sv = f_blk_sum(p4);
      if (wsum) pa[N + a * N + 16 * b + 4 * g + rsel] = sv;
    }
#endif
  auto prep2 = [&](int b) {   // dZ2 of block b, in place of H2, and its store
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hh = 16 * b + 4 * g + r;
      float gg = 0.f;
#pragma unroll
      for (int a = 0; a < A; ++a) gg += dout[a] * sw3[a * N + hh];
      const float hv = h2[b][r];
      h2[b][r] = gg * (1.f - hv * hv);
    }
    f_st4(z2r, voff, 64u * b, h2[b]);
  };
  prep2(0);

  F_STAMP(4);
  // ---- dH1ᵀ = W2ᵀ·dZ2ᵀ (two hidden blocks per chunk); dZ1ᵀ = dH1ᵀ ⊙ (1 − H1ᵀ²) in place of H1ᵀ
  // (stored at the chunk's end).  Beside the MFMAs: dZ2 of block ob + 1 during step ob of
  // chunk 0, the b2 partial of dZ2 block ob during step ob of chunk 1, the b1 partials of
  // chunk c's dZ1 blocks during the first two steps of chunk c + 1.
  float* pb = spb + w * N;
  auto b1sum = [&](int b) {
    const float sv = f_blk_sum(h1[b]);
    if (wsum) pb[16 * b + 4 * g + rsel] = sv;
  };
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float4* wc = next(nW1 + 8 + c);
    f32x4 d0 = f32x4{0.f, 0.f, 0.f, 0.f}, d1 = d0;
    float4 w0 = wc[l], w1 = wc[16 * 64 + l];
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) {
      float4 n0 = w0, n1 = w1;
      if (ob + 1 < 16) { n0 = wc[(ob + 1) * 64 + l]; n1 = wc[(17 + ob) * 64 + l]; }
      __builtin_amdgcn_sched_barrier(0);
      if (c == 0 && ob + 1 < 16) prep2(ob + 1);
      if (c == 1) {
        const float sb = f_blk_sum(h2[ob]);
        if (wsum) pa[16 * ob + 4 * g + rsel] = sb;
      }
      if (c > 0 && ob < 2) b1sum(2 * (c - 1) + ob);
      d0 = mfma16(w0.x, h2[ob][0], d0);
      d1 = mfma16(w1.x, h2[ob][0], d1);
      d0 = mfma16(w0.y, h2[ob][1], d0);
      d1 = mfma16(w1.y, h2[ob][1], d1);
      d0 = mfma16(w0.z, h2[ob][2], d0);
      d1 = mfma16(w1.z, h2[ob][2], d1);
      d0 = mfma16(w0.w, h2[ob][3], d0);
      d1 = mfma16(w1.w, h2[ob][3], d1);
      w0 = n0;
      w1 = n1;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float u0 = h1[2 * c][r], u1 = h1[2 * c + 1][r];
      h1[2 * c][r] = d0[r] * (1.f - u0 * u0);
      h1[2 * c + 1][r] = d1[r] * (1.f - u1 * u1);
    }
    f_st4(z1r, voff, 64u * (2 * c), h1[2 * c]);
    f_st4(z1r, voff, 64u * (2 * c + 1), h1[2 * c + 1]);
  }
  b1sum(14);
  b1sum(15);
  M3Stream::sync();
  F_STAMP(5);
  // the loss sums of the wave's rows (group 0), then the waves in order
#pragma unroll
  for (int k = 0; k < NL; ++k)
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) ls[k] += __shfl_xor(ls[k], o, 64);
  if (l == 0)
#pragma unroll
    for (int k = 0; k < NL; ++k) ldsn[w][k] = ls[k];
  __syncthreads();
  for (int t = tid; t < PA; t += kFBlock) {
    float s = spa[t];
#pragma unroll
    for (int v = 1; v < kFWaves; ++v) s += spa[v * PA + t];
    partA[(size_t)blockIdx.x * PA + t] = s;
  }
  for (int t = tid; t < N; t += kFBlock) {
    float s = spb[t];
#pragma unroll
    for (int v = 1; v < kFWaves; ++v) s += spb[v * N + t];
    partB[(size_t)blockIdx.x * N + t] = s;
  }
  if (partW1) {   // kernel-uniform
    // ---- dW1 = dZ1ᵀ·X over the workgroup's 128 rows, from the
    // dZ1 still in registers: no dZ1 stores, no separate 27-column GEMM beside
    // dW2.  The LDS is free once the partial rows above are read: the X tile
    // [128][Ip + 16] (staged from this workgroup's own Xa rows), then dZ1 one
    // 128-unit half at a time [128][144]; wave w contracts m-block w of the half
    // against every k-block, 4 rows per 16x16x4 step (A: dZ1[row][m], B:
    // X[row][k]); strides ≡ 16 mod 64 put the four rows of a read on distinct banks.
    constexpr int DZS = 144;
    const int XS = Ip + 16, KB = Ip / 16;   // KB <= kFMaxIp / 16 = 8
    float* const dzs = lf;                  // [128][DZS]
    float* const xs = lf + 128 * DZS;       // [128][XS]
    const long long r0 = (long long)blockIdx.x * kFWaves * 16;
    __syncthreads();   // spa / spb read
    for (int t = tid; t < 128 * Ip; t += kFBlock) {
      const int rr = t / Ip, k = t - rr * Ip;
      xs[rr * XS + k] = (r0 + rr < K && k < I) ? Xa[(r0 + rr) * I + k] : 0.f;
    }
    const int rq = l >> 4, cq = l & 15;
    float* const pw = partW1 + (size_t)blockIdx.x * N * I;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int bb = 0; bb < 8; ++bb)
        *reinterpret_cast<float4*>(dzs + (w * 16 + j) * DZS + 16 * bb + 4 * g) =
            make_float4(h1[8 * p + bb][0], h1[8 * p + bb][1], h1[8 * p + bb][2], h1[8 * p + bb][3]);
      __syncthreads();
      f32x4 a4[kFMaxIp / 16];
#pragma unroll
      for (int kb = 0; kb < kFMaxIp / 16; ++kb) a4[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      // one step's operands read ahead of its MFMAs (unrolled further, the
      // compiler hoisted every read and spilled the kernel's registers)
      float av = dzs[rq * DZS + 16 * w + cq], xv[kFMaxIp / 16];
#pragma unroll
      for (int kb = 0; kb < kFMaxIp / 16; ++kb) xv[kb] = kb < KB ? xs[rq * XS + 16 * kb + cq] : 0.f;
#pragma unroll 1
      for (int s4 = 0; s4 < 32; ++s4) {
        const int rn = 4 * (s4 + 1 < 32 ? s4 + 1 : s4) + rq;
        const float an = dzs[rn * DZS + 16 * w + cq];
        float xn[kFMaxIp / 16];
#pragma unroll
        for (int kb = 0; kb < kFMaxIp / 16; ++kb) xn[kb] = kb < KB ? xs[rn * XS + 16 * kb + cq] : 0.f;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kb = 0; kb < kFMaxIp / 16; ++kb)
          if (kb < KB) a4[kb] = mfma16(av, xv[kb], a4[kb]);
        av = an;
#pragma unroll
        for (int kb = 0; kb < kFMaxIp / 16; ++kb) xv[kb] = xn[kb];
      }
#pragma unroll
      for (int kb = 0; kb < kFMaxIp / 16; ++kb) {
        const int k = 16 * kb + cq;
        if (kb < KB && k < I)
#pragma unroll
          for (int r = 0; r < 4; ++r) pw[(size_t)(128 * p + 16 * w + 4 * rq + r) * I + k] = a4[kb][r];
      }
      __syncthreads();   // dzs is rewritten by the next half
    }
  }
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      double s = ldsn[0][k];
#pragma unroll
      for (int v = 1; v < kFWaves; ++v) s += ldsn[v][k];
      lossp[(size_t)blockIdx.x * NL + k] = s;
    }
    F_STAMP(6);
#ifndef QS_F_NOFENCE   // dev probe: the cost of the agent-scope release (results of the loss sums undefined)
    __threadfence();
#endif
    last = atomicAdd(count, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: fixed-order sums of the loss partials (ppo_heads_kernel's tail)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double tot[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) tot[k] = 0.0;
  for (unsigned bb = tid; bb < gridDim.x; bb += kFBlock)
#pragma unroll
    for (int k = 0; k < NL; ++k) tot[k] += lossp[(size_t)bb * NL + k];
  block_sum_n<NL>(tot, ldsn);
  if (tid != 0) return;
  *count = 0;
  const float lc = (float)log(sqrt(2.0 * M_PI));
  float ent = 0.0f;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float lsd = logf(expf(logstd[a]));
    ent = a == 0 ? (0.5f + lc) + lsd : ent + ((0.5f + lc) + lsd);
  }
#pragma unroll
  for (int a = 0; a < A; ++a) dlogstd[a] = (float)tot[2 + a] - ent_coef;
  const float akl = (float)(tot[1] / (double)K);
  *kl_out = akl;
  acc[0] += tot[0] / (double)K;
  acc[2] += (double)(-ent);
  acc[3] += (double)akl;
}


// torch.optim.Adam over several flat parameter buffers in one launch (the
// actor's, KL-gated, and the critic's): blocks [start[i], start[i+1]) serve
// segment i, kAdamPer elements per thread (all loads issued before the
// arithmetic).  Thread 0 of each block forms the bias corrections once from the
// step count (fp64, as torch's host-side step_size), and the last block of a
// segment to finish commits its step count (gate permitting).  Optionally per
// segment: the gradient is zeroed after it is read (the next minibatch's sums
// accumulate into it), and the updated W1 / W2 of a 256-wide tanh MLP are also
// written into its qs_mlp3_pack image (W1p; W2p and W2Tp), so no pack launch
// runs between the step and the next forward.
constexpr int kAdamMaxSeg = 4;
constexpr int kAdamBlock = 256;
constexpr int kAdamPer = 4;
// A segment gets at most kAdamSegBlocks workgroups (grid-stride): the
// last-block arrival count is one atomic per workgroup on one address, and those
// serialise at the L2 — a hundred cost about a microsecond, a thousand ~10 µs.
constexpr int kAdamSegBlocks = 128;
struct AdamSeg {
  float* p;
  float* g;
  float* m;
  float* v;
  float* step;
  const float* gate;
  float* pack;            // NULL: no pack image
  long long n, w1, w2;    // elements; offsets of W1 [256][I] and W2 [256][256] in p
  float lr, b1, b2, eps, thr;
  int I, zero;
  int kind;               // pack layout: 0 qs_mlp3_pack (32x32 tiles), 1 qs_mlp3f_pack (16x16 tiles), 2 W2ᵀ
};
struct AdamSegs {
  AdamSeg s[kAdamMaxSeg];
  int start[kAdamMaxSeg + 1];
  int n;
};

// pack positions (qs_mlp3_pack layout) of W1[m][k] and W2[m][n]
__device__ __forceinline__ long long m3_pos_w1(int m, int k) {
  const int st = k >> 1, hh = k & 1, q = st >> 2, e = st & 3, mb = m >> 5, c = m & 31;
  return ((((long long)q * kM3NB + mb) * 64 + 32 * hh + c) << 2) + e;
}
// row(i, h) = (i & 3) + 8 (i >> 2) + 4h  ⇔  i = (x & 3) + 4 (x >> 3), h = (x >> 2) & 1 for x in [0, 32)
__device__ __forceinline__ long long m3_pos_w2(int blk, int c, int other, int x) {
  const int i = (x & 3) + 4 * (x >> 3), hh = (x >> 2) & 1, st = 16 * other + i, q = st >> 2, e = st & 3;
  return ((((long long)blk * 32 + q) * 64 + 32 * hh + c) << 2) + e;
}

// One Adam element (torch.optim.Adam, amsgrad=False, weight_decay=0): the new
// moments and parameter, and the parameter's pack-image copies.  bc1 =
// 1 − β1^t, bc2s = sqrt(1 − β2^t).
__device__ __forceinline__ void adam_elem(const AdamSeg& A, long long i, float g, float p, float m, float v,
                                          float bc1, float bc2s) {
  const float m1 = m + (1.0f - A.b1) * (g - m);
  const float v1 = v * A.b2 + (1.0f - A.b2) * g * g;
  A.m[i] = m1;
  A.v[i] = v1;
  const float denom = sqrtf(v1) / bc2s + A.eps;
  const float p1 = p - (A.lr / bc1) * (m1 / denom);
  A.p[i] = p1;
  if (A.pack && A.kind == 1) {
    const long long w2f0 = f16_w1_floats(f16_ip(A.I)), w2b0 = w2f0 + kFW2Floats;
    if (i >= A.w1 && i < A.w1 + (long long)kM3N * A.I) {
      const int mm = (int)((i - A.w1) / A.I), k = (int)((i - A.w1) - (long long)mm * A.I);
      A.pack[f16_pos_w1(mm, k)] = p1;
    } else if (i >= A.w2 && i < A.w2 + (long long)kM3N * kM3N) {
      const int mm = (int)((i - A.w2) >> 8), n = (int)((i - A.w2) & 255);
      A.pack[w2f0 + f16_pos_w2f(mm, n)] = p1;
      A.pack[w2b0 + f16_pos_w2b(mm, n)] = p1;
    }
  } else if (A.pack && A.kind == 2) {   // a W2ᵀ copy (QS_PACK_W2T)
    if (i >= A.w2 && i < A.w2 + (long long)kM3N * kM3N) {
      const int mm = (int)((i - A.w2) >> 8), n = (int)((i - A.w2) & 255);
      A.pack[(size_t)n * kM3N + mm] = p1;
    }
  } else if (A.pack) {
    const int Ip = (A.I + 31) & ~31;
    const long long w2p0 = (long long)(Ip / 8) * kM3NB * 256, w2tp0 = w2p0 + (long long)kM3NB * 32 * 256;
    if (i >= A.w1 && i < A.w1 + (long long)kM3N * A.I) {
      const int mm = (int)((i - A.w1) / A.I), k = (int)((i - A.w1) - (long long)mm * A.I);
      A.pack[m3_pos_w1(mm, k)] = p1;
    } else if (i >= A.w2 && i < A.w2 + (long long)kM3N * kM3N) {
      const int mm = (int)((i - A.w2) >> 8), n = (int)((i - A.w2) & 255);
      A.pack[w2p0 + m3_pos_w2(mm >> 5, mm & 31, n >> 5, n & 31)] = p1;    // W2p:  blk = mb, c = m, other = nb
      A.pack[w2tp0 + m3_pos_w2(n >> 5, n & 31, mm >> 5, mm & 31)] = p1;   // W2Tp: blk = nb, c = n, other = mb
    }
  }
}

__device__ __forceinline__ double powi_d(double b, unsigned t) {
  double r = 1.0;
  while (t) {
    if (t & 1u) r *= b;
    b *= b;
    t >>= 1;
  }
  return r;
}

__global__ void __launch_bounds__(kAdamBlock) adam_multi_kernel(AdamSegs S, unsigned* done) {
  __shared__ float sc[2];
  __shared__ bool last;
  int si = 0;
  while (si + 1 < S.n && (int)blockIdx.x >= S.start[si + 1]) ++si;
  const AdamSeg& A = S.s[si];
  const int nb = S.start[si + 1] - S.start[si];
  const bool open = gate_ok(A.gate, A.thr);
  const long long stride = (long long)nb * kAdamBlock * kAdamPer;
  const long long first = (long long)(blockIdx.x - S.start[si]) * kAdamBlock * kAdamPer + threadIdx.x;
  float gi[kAdamPer], mi[kAdamPer], vi[kAdamPer], pi[kAdamPer];
  auto load = [&](long long i0) {
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const long long i = i0 + (long long)u * kAdamBlock;
      if (i < A.n) { gi[u] = A.g[i]; mi[u] = A.m[i]; vi[u] = A.v[i]; pi[u] = A.p[i]; }
    }
  };
  load(first);   // in flight while thread 0 forms the bias corrections
  if (threadIdx.x == 0) {
    // β^t for the integral step count t by fp64 square-and-multiply (a few
    // dozen dependent multiplies; the libm pow took microseconds on one lane)
    const unsigned t = (unsigned)(*A.step) + 1u;
    sc[0] = (float)(1.0 - powi_d((double)A.b1, t));        // bias_correction1
    sc[1] = (float)sqrt(1.0 - powi_d((double)A.b2, t));   // sqrt(bias_correction2)
  }
  __syncthreads();
  for (long long i0 = first; i0 < A.n; i0 += stride) {
    if (i0 != first) load(i0);
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const long long i = i0 + (long long)u * kAdamBlock;
      if (i >= A.n) break;
      if (A.zero) A.g[i] = 0.f;
      if (open) adam_elem(A, i, gi[u], pi[u], mi[u], vi[u], sc[0], sc[1]);
    }
  }
  __syncthreads();
  // every block read *step before counting itself; p/m/v go to later launches only
  if (threadIdx.x == 0) last = atomicAdd(&done[si], 1u) == (unsigned)nb - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    done[si] = 0;
    if (open) *A.step = *A.step + 1.0f;
  }
}

// The minibatch's partial-sum reduction and the Adam step in one launch (one
// rank: no gradient exchange between them).  Every gradient element of the
// segments is the destination of exactly one task column; the block that
// reduces it applies Adam to it at once (the gradient is never written).  Each
// block forms both segments' bias corrections; the last block to finish
// commits the step counts (gates permitting).  The per-column summation order
// is mlp_sum_multi_kernel's, so the step equals sum-then-Adam bit for bit.
constexpr int kSumAdamGroup = 32;     // blocks per group word of mlp_sum_adam_kernel's arrival count
constexpr int kSumAdamStride = 64;    // words between two counter words (256 B)
constexpr int kSumAdamGroups = 63;    // at most 63 · 32 = 2 016 blocks (qs_mlp_sum_adam_work_bytes)
__global__ void __launch_bounds__(kMlpSumBlock) mlp_sum_adam_kernel(MlpSumTasks tasks, AdamSegs S, SegOf seg,
                                                                   unsigned* done) {
  __shared__ float sc[kAdamMaxSeg][2];
  __shared__ bool last;
#ifndef QS_SA_NOPOW
  if (threadIdx.x < (unsigned)S.n) {
    const AdamSeg& A = S.s[threadIdx.x];
    const unsigned t = (unsigned)(*A.step) + 1u;
    sc[threadIdx.x][0] = (float)(1.0 - powi_d((double)A.b1, t));
    sc[threadIdx.x][1] = (float)sqrt(1.0 - powi_d((double)A.b2, t));
  }
#else
  if (threadIdx.x < (unsigned)S.n) sc[threadIdx.x][0] = sc[threadIdx.x][1] = 1.f;
#endif
  __syncthreads();
  // the element's parameter and moments are loaded with the partial rows
  mlp_sum_block(tasks, [&](int ti, float* dst, float u, float3 pmv) {
    const int si = seg.s[ti];
    const AdamSeg& A = S.s[si];
#ifdef QS_SA_NOADAM
    *dst = u + pmv.x;
    return;
#endif
    if (!gate_ok(A.gate, A.thr)) return;
    adam_elem(A, dst - A.g, u, pmv.x, pmv.y, pmv.z, sc[si][0], sc[si][1]);
  }, [&](int ti, float* dst) {
    const AdamSeg& A = S.s[seg.s[ti]];
    const long long i = dst - A.g;
    return make_float3(A.p[i], A.m[i], A.v[i]);
  });
#ifdef QS_SA_NOTAIL
  return;
#endif
  __syncthreads();
  // every block read the step counts before counting itself.  Two-level count:
  // a block arrives at its group's word (kSumAdamGroup blocks a group), a group's
  // last block at the top word; the words lie kSumAdamStride apart, in separate
  // L2 channels (same-address atomics serialise: one word for ~400 blocks was
  // ~3 µs of tail)
  if (threadIdx.x == 0) {
    const unsigned grp = blockIdx.x / kSumAdamGroup, ngrp = (gridDim.x + kSumAdamGroup - 1) / kSumAdamGroup;
    const unsigned gsz = min((unsigned)kSumAdamGroup, gridDim.x - grp * kSumAdamGroup);
    unsigned* gw = done + (size_t)kSumAdamStride * (1 + grp);
    last = false;
    if (atomicAdd(gw, 1u) == gsz - 1) {
      *gw = 0;
      last = atomicAdd(done, 1u) == ngrp - 1;
    }
  }
  __syncthreads();
  if (last && threadIdx.x < (unsigned)S.n) {
    const AdamSeg& A = S.s[threadIdx.x];
    if (gate_ok(A.gate, A.thr)) *A.step = *A.step + 1.0f;
    if (threadIdx.x == 0) *done = 0;
  }
}

// ---- weight gradients dW = Aᵀ·B over a long batch, as fixed-order partials.
// partial[c][n][m] = Σ_{b in chunk c} AT[n][b]·B(b, m), B(b, m) = B[b][m]
// (BT = false: the layer input X, row-major [K][M]) or BT[m][b] (BT = true: a
// transposed activation [M][K]).  One wave per 32×32 output tile and batch
// chunk: each MFMA step contracts two batch rows, a lane's float4 of AT (BT)
// holds four consecutive rows of its n (m), so every operand load is one
// 16-B vector per lane and no LDS or transpose is needed.  The chunk partials
// are summed in chunk order by the minibatch's reduction (qs_mlp_sum_adam).
constexpr int kWgWaves = 4;
template <bool BT>
__global__ void __launch_bounds__(64 * kWgWaves) mlp_wgrad_kernel(long long K, int N, int M, int R,
                                                                  const float* __restrict__ AT,
                                                                  const float* __restrict__ B,
                                                                  float* __restrict__ partial) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c32 = lane & 31, hf = lane >> 5;
  const int nb = blockIdx.x * kWgWaves + w;   // 32-row block of N
  if (nb * 32 >= N) return;                   // (no barriers below)
  const int mb = blockIdx.y, ch = blockIdx.z;
  const int m = mb * 32 + c32;
  const bool mv = m < M;
  const long long b0 = (long long)ch * R;
  const float* ap = AT + (size_t)(nb * 32 + c32) * K + b0 + 4 * hf;
  const float* bp = BT ? B + (size_t)(mv ? m : 0) * K + b0 + 4 * hf : B + (size_t)(b0 + 4 * hf) * M + (mv ? m : 0);
  // batches of U 8-row steps; the next batch's loads are issued before this
  // batch's MFMAs (one wave per SIMD: the loads' latency must hide under MFMAs)
  constexpr int U = 8;
  f32x16 acc = f32x16{};
  float4 av[2][U];
  float bv[2][U][4];
  auto load = [&](int buf, int r) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      av[buf][u] = *reinterpret_cast<const float4*>(ap + r + 8 * u);
      if constexpr (BT) {
        const float4 t = *reinterpret_cast<const float4*>(bp + r + 8 * u);
        bv[buf][u][0] = t.x; bv[buf][u][1] = t.y; bv[buf][u][2] = t.z; bv[buf][u][3] = t.w;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[buf][u][q] = mv ? bp[(size_t)(r + 8 * u + q) * M] : 0.f;
      }
    }
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[buf][u].x, mv ? bv[buf][u][0] : 0.f, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[buf][u].y, mv ? bv[buf][u][1] : 0.f, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[buf][u].z, mv ? bv[buf][u][2] : 0.f, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[buf][u].w, mv ? bv[buf][u][3] : 0.f, acc, 0, 0, 0);
    }
  };
  // R is a multiple of 8·U (qs_mlp_wgrad): batches r = 0, 8U, … alternate buffers
  load(0, 0);
  for (int r = 0; r < R; r += 16 * U) {
    if (r + 8 * U < R) load(1, r + 8 * U);
    mma(0);
    if (r + 16 * U < R) load(0, r + 16 * U);
    if (r + 8 * U < R) mma(1);
  }
  if (!mv) return;
  float* out = partial + (size_t)ch * N * M + m;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int n = nb * 32 + 8 * (j >> 2) + 4 * hf + (j & 3);
    out[(size_t)n * M] = acc[j];
  }
}

// ---- weight gradient of a first layer: dW[256][M] = Σ_b AT[256][b]·X[b][M]
// (AT = dZ1ᵀ, X the layer input [K][M], M <= 256), as chunk partials
// partial[c][256][M] over row chunks of kWxR rows.  A workgroup owns one chunk
// and one 32-column tile of X (staged once in LDS, shared by its 4 waves);
// wave w owns hidden tiles 2w, 2w + 1 (32x32x2 f32 MFMA).  Every AT operand of
// the chunk is issued before the first MFMA (one memory round trip per wave):
// a lane's float4 holds four consecutive rows of its hidden unit, so the
// contraction index is permuted (step 4u + e, half h ↔ row 8u + 4h + e) on both
// operands alike.  The partials are summed in chunk order by the minibatch's
// reduction (qs_mlp_sum_adam).
constexpr int kWxR = 128;
constexpr int kWxStride = 33;   // LDS row stride of the X tile (conflict-free column reads)
template <bool BLOCKED>
__global__ void __launch_bounds__(256) mlp_wgrad_x_kernel(long long K, int M, const float* __restrict__ AT,
                                                          const float* __restrict__ X, float* __restrict__ partial) {
  __shared__ float xs[kWxR * kWxStride];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long long r0 = (long long)blockIdx.x * kWxR;
  const int m0 = blockIdx.y * 32;
  float4 av[2][kWxR / 8];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if constexpr (BLOCKED) {   // AT [K/8][256][8]: a wave's float4s of one u are 1 KB contiguous
      const float* a = AT + ((size_t)(r0 / 8) * kM3N + 64 * w + 32 * t + c) * 8 + 4 * h;
#pragma unroll
      for (int u = 0; u < kWxR / 8; ++u) av[t][u] = *reinterpret_cast<const float4*>(a + (size_t)u * kM3N * 8);
    } else {
      const float* a = AT + (size_t)(64 * w + 32 * t + c) * K + r0 + 4 * h;
#pragma unroll
      for (int u = 0; u < kWxR / 8; ++u) av[t][u] = *reinterpret_cast<const float4*>(a + 8 * u);
    }
  }
  for (int i = threadIdx.x; i < kWxR * 32; i += 256) {
    const int r = i >> 5, cc = i & 31;
    xs[r * kWxStride + cc] = m0 + cc < M ? X[(size_t)(r0 + r) * M + m0 + cc] : 0.f;
  }
  __syncthreads();
  f32x16 acc0 = f32x16{}, acc1 = f32x16{};
#pragma unroll
  for (int u = 0; u < kWxR / 8; ++u) {
    const float* xr = xs + (8 * u + 4 * h) * kWxStride + c;
    const float b0 = xr[0], b1 = xr[kWxStride], b2 = xr[2 * kWxStride], b3 = xr[3 * kWxStride];
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][u].x, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][u].x, b0, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][u].y, b1, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][u].y, b1, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][u].z, b2, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][u].z, b2, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][u].w, b3, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][u].w, b3, acc1, 0, 0, 0);
  }
  if (m0 + c >= M) return;
  float* out = partial + (size_t)blockIdx.x * kM3N * M + m0 + c;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    out[(size_t)(64 * w + m3_row(i, h)) * M] = acc0[i];
    out[(size_t)(64 * w + 32 + m3_row(i, h)) * M] = acc1[i];
  }
}

// ---- wide variant: one 32-row tile per workgroup of 8 waves, wave w owning
// hidden block w (batches of < 16 384 rows, e.g. the critic's 4 096: 128 tiles
// would leave most SIMDs idle with one wave per tile).  The waves exchange
// their activation blocks through LDS before each contraction over the hidden
// index; each wave streams its own weight block from L2 (no sharing, no LDS).
constexpr int kM3WWaves = 8;
constexpr int kM3WBlock = 64 * kM3WWaves;
// dynamic LDS of the wide forward (floats): the X tile (row stride Ip + 1),
// then the H1ᵀ exchange — sized to the input width so a workgroup can share its
// CU with another kernel's (the actor's, on the other stream)
__host__ __device__ constexpr int m3w_lds_floats(int Ip) {
  return 32 * (Ip + 1) > kM3Steps2 * 64 ? 32 * (Ip + 1) : kM3Steps2 * 64;
}

// The exchange of the waves' activation blocks: wave w's 16 values of lane
// (c, h) are B-operand steps 16w .. 16w + 15 of the 256-deep contraction, kept
// in LDS as one float4 per k-quad and lane (k-quad q = steps 4q .. 4q + 3 at
// xs4[q·64 + lane]) — each lane's four operands of a quad in one ds_read_b128,
// consecutive lanes on consecutive 16 B.  (Held in 128 registers per lane, they
// put the 8-wave kernels at 210 VGPRs: one workgroup per CU, its staging and
// barriers never overlapped by another's MFMAs.)
__device__ __forceinline__ void m3w_share(float4* xs4, const float* mine, int w) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    xs4[(4 * w + i) * 64 + lane] = make_float4(mine[4 * i], mine[4 * i + 1], mine[4 * i + 2], mine[4 * i + 3]);
  __syncthreads();
}

// Σ_k over the 128 MFMA steps of block blk of a [8 blk][32 q][64][4] packed
// matrix (W2p or W2Tp), the B operand from the LDS exchange (m3w_share) one
// k-quad ahead.  A wave's block is private to it, so it streams straight from
// L2 into a ring of eight float4 (eight k-quads = 32 MFMAs ahead), no LDS.
__device__ __forceinline__ f32x16 m3w_contract(const float4* __restrict__ mat, int blk, const float4* xs4) {
  const int lane = threadIdx.x & 63;
  const float4* p = mat + (size_t)blk * 32 * 64 + lane;
  const float4* b = xs4 + lane;
  float4 ring[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) ring[u] = p[u * 64];
  float4 bn = b[0];
  f32x16 z = f32x16{};
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const float4 wv = ring[q & 7], bv = bn;
    if (q + 8 < 32) ring[q & 7] = p[(q + 8) * 64];
    if (q + 1 < 32) bn = b[(q + 1) * 64];
    __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead (the scheduler would sink them)
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, bv.x, z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, bv.y, z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, bv.z, z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, bv.w, z, 0, 0, 0);
  }
  return z;
}

// The register-held exchange (round 4): every lane holds the 128 B-operand
// steps of the contraction.  Kept for the backward, where the LDS exchange
// measured slower beside the fused actor (the C3 update: the critic's 8-wave
// backward shares the CUs with the actor chain's kernels); dev builds select
// either per kernel (QS_M3W_FWD_REGS / QS_M3W_BWD_LDS).
__device__ __forceinline__ void m3w_share_regs(float* xs, const float* mine, float* all, int w) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 16; ++i) xs[(w * 16 + i) * 64 + lane] = mine[i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kM3Steps2; ++k) all[k] = xs[k * 64 + lane];
}
__device__ __forceinline__ f32x16 m3w_contract_regs(const float4* __restrict__ mat, int blk, const float* bv) {
  const float4* p = mat + (size_t)blk * 32 * 64 + (threadIdx.x & 63);
  float4 ring[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) ring[b] = p[b * 64];
  f32x16 z = f32x16{};
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const float4 wv = ring[q & 7];
    if (q + 8 < 32) ring[q & 7] = p[(q + 8) * 64];
    __builtin_amdgcn_sched_barrier(0);   // keep the load eight k-quads ahead (the scheduler would sink it)
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, bv[4 * q + 0], z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, bv[4 * q + 1], z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, bv[4 * q + 2], z, 0, 0, 0);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, bv[4 * q + 3], z, 0, 0, 0);
  }
  return z;
}
#ifdef QS_M3W_FWD_REGS
constexpr bool kM3wFwdLds = false;
#else
constexpr bool kM3wFwdLds = true;
#endif
#ifdef QS_M3W_BWD_LDS
constexpr bool kM3wBwdLds = true;
#else
constexpr bool kM3wBwdLds = false;
#endif

// The centralized critic's value head folded into its forward (qs_mlp3_fwd_rows_value):
// compute_value_loss (AG:642-683) per row as qs_value_head does it, its loss sum
// from the last workgroup.  dv == NULL: the plain forward.
struct M3ValueHead {
  const double* ret;   // [T·E] returns; row r's is ret[rows[r]]
  float* dv;           // [K] d(value loss)/dv
  double* lossp;       // [grid] per-workgroup Σ (v − ret)²
  double* acc;         // acc[1] += ½·mean
  unsigned* count;     // arrival counter (left zero)
  int D, mb;
};

template <int A>
__global__ void __launch_bounds__(kM3WBlock) mlp3w_fwd_kernel(long long K, int I, const float* __restrict__ X,
                                                              const float* __restrict__ pack,
                                                              const float* __restrict__ b1,
                                                              const float* __restrict__ b2,
                                                              const float* __restrict__ W3,
                                                              const float* __restrict__ b3, float* __restrict__ H1T,
                                                              float* __restrict__ H2T, float* __restrict__ out,
                                                              const long long* __restrict__ rows,
                                                              float* __restrict__ Xg, int G, M3ValueHead vh) {
  // LDS: the X tile during layer 1, then the H1ᵀ exchange
  extern __shared__ __attribute__((aligned(16))) float lds[];   // m3w_lds_floats(Ip)
  __shared__ float hp[kM3WWaves][A][64];
  float* xs = lds;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long long r0 = (long long)blockIdx.x * 32, r = r0 + c;
  const bool rv = r < K;
  const int Ip = m3_ip(I), S = Ip + 1;   // odd row stride: the 32 rows of a read hit 32 banks
  const __amdgpu_buffer_rsrc_t h1r = m3_rsrc(H1T, H1T ? (size_t)K * kM3N * 4 : 0),
                               h2r = m3_rsrc(H2T, H2T ? (size_t)K * kM3N * 4 : 0);
  const unsigned roff = rv ? (unsigned)(r * 4) : kM3OOB;
  const unsigned kstride = (unsigned)(K * 4);
  // the tile's 32 rows are contiguous in X: every wave reads them coalesced,
  // once, instead of each of the 8 waves gathering every lane's row
  // (rows != NULL: tile row r is X row rows[r] — the minibatch gather — and is
  // also written to Xg[r], the gathered copy the weight gradients read).  Each
  // wave stages 4 rows; every load of a 256-column pass is issued before the
  // first LDS write, so the pass costs one memory latency, not sixteen.
  constexpr int RPW = 32 / kM3WWaves;
  long long src[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) {
    const long long rr = r0 + w + kM3WWaves * j;
    src[j] = rr < K ? (rows ? rows[rr / G] * G + rr % G : rr) : -1;
  }
  for (int k0 = 0; k0 < Ip; k0 += 256) {
    float v[RPW][4];
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + lane + 64 * u;
        v[j][u] = src[j] >= 0 && k < I ? X[src[j] * I + k] : 0.f;
      }
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + lane + 64 * u, row = w + kM3WWaves * j;
        if (k < Ip) lds[row * S + k] = v[j][u];
        if (rows && Xg && src[j] >= 0 && k < I) Xg[(r0 + row) * I + k] = v[j][u];
      }
  }
  __syncthreads();
  // layer 1, block w: W1p (the wave's block, one coalesced float4 per k-quad)
  // from L2, software-pipelined eight k-quads ahead (Ip is a multiple of 32)
  const float4* w1p = reinterpret_cast<const float4*>(pack) + w * 64 + lane;
  const float* xrow = lds + c * S + h;
  f32x16 acc = f32x16{};
  const int nq = Ip / 8;   // a multiple of 4
  float4 wq[8];
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if (b < nq) wq[b] = w1p[(size_t)b * kM3NB * 64];
  for (int q0 = 0; q0 < nq; q0 += 8) {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b >= 4 && q0 + b >= nq) break;
      const float4 wv = wq[b];
      if (q0 + 8 + b < nq) wq[b] = w1p[(size_t)(q0 + 8 + b) * kM3NB * 64];
      __builtin_amdgcn_sched_barrier(0);   // keep the load eight k-quads ahead
      const float* xk = xrow + 8 * (q0 + b);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, xk[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, xk[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, xk[4], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, xk[6], acc, 0, 0, 0);
    }
  }
  __syncthreads();   // the X tile is dead: the LDS is reused below
  float mine[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 32 * w + m3_row(i, h);
    mine[i] = m3_tanh(acc[i] + b1[m]);
    m3_st(h1r, roff + (unsigned)m * kstride, mine[i]);
  }
  // layer 2, block w: Z2ᵀ[w] = W2[w]·H1ᵀ
  f32x16 z;
  if constexpr (kM3wFwdLds) {
    float4* const xs4 = reinterpret_cast<float4*>(xs);
    m3w_share(xs4, mine, w);
    z = m3w_contract(reinterpret_cast<const float4*>(pack + m3_w1p_floats(Ip)), w, xs4);
  } else {
    float hb[kM3Steps2];
    m3w_share_regs(xs, mine, hb, w);
    z = m3w_contract_regs(reinterpret_cast<const float4*>(pack + m3_w1p_floats(Ip)), w, hb);
  }
  float hs[A];
#pragma unroll
  for (int a = 0; a < A; ++a) hs[a] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 32 * w + m3_row(i, h);
    const float v = m3_tanh(z[i] + b2[m]);
    m3_st(h2r, roff + (unsigned)m * kstride, v);
#pragma unroll
    for (int a = 0; a < A; ++a) hs[a] += v * W3[a * kM3N + m];
  }
  // head: halves, then the 8 waves in order
#pragma unroll
  for (int a = 0; a < A; ++a) hp[w][a][lane] = hs[a] + __shfl_xor(hs[a], 32, 64);
  __syncthreads();
  float v0 = 0.f;
  if (w == 0 && h == 0 && rv)
#pragma unroll
    for (int a = 0; a < A; ++a) {
      float t = hp[0][a][lane];
#pragma unroll
      for (int k = 1; k < kM3WWaves; ++k) t += hp[k][a][lane];
      out[r * A + a] = t + b3[a];
      if (a == 0) v0 = t + b3[a];
    }
  if (!vh.dv) return;   // (kernel-uniform)
  // the value head (qs_value_head's arithmetic): dv = (v − mean_d ret)/mb, and
  // the tile's Σ (v − mean_d ret)² over its rows in lane order
  __shared__ bool vlast;
  if (w == 0) {
    double sq = 0.0;
    if (h == 0 && rv) {
      const double rt = vh.ret[rows[r]];
      double rs = 0;
      for (int d = 0; d < vh.D; ++d) rs += rt;
      const double diff = (double)v0 - rs / (double)vh.D;
      vh.dv[r] = (float)(diff / (double)vh.mb);
      sq = diff * diff;
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);   // within each half: lanes 0..31 hold the rows
    if (lane == 0) {
      vh.lossp[blockIdx.x] = sq;
      __threadfence();
      vlast = atomicAdd(vh.count, 1u) == gridDim.x - 1;
    }
  }
  __syncthreads();
  if (!vlast || w != 0) return;
  // the last workgroup: the tiles' sums (lane q: tiles q, q + 64, ... in order),
  // then a fixed xor butterfly (every lane the same bits)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double tot = 0.0;
  for (unsigned b = lane; b < gridDim.x; b += 64) tot += vh.lossp[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if (lane == 0) {
    vh.acc[1] += 0.5 * (tot / (double)vh.mb);
    *vh.count = 0u;
  }
}

template <int A>
__global__ void __launch_bounds__(kM3WBlock) __attribute__((amdgpu_waves_per_eu(kM3wBwdLds && A <= 2 ? 4 : 1))) mlp3w_bwd_kernel(long long K, const float* __restrict__ dout,
                                                              const float* __restrict__ H1T,
                                                              const float* __restrict__ H2T,
                                                              const float* __restrict__ pack, int Ip,
                                                              const float* __restrict__ W3, float* __restrict__ dZ2T,
                                                              float* __restrict__ dZ1T, float* __restrict__ partA,
                                                              float* __restrict__ partB) {
  constexpr int N = kM3N, PA = N + A * N + A;
  __shared__ __attribute__((aligned(16))) float xs[kM3Steps2 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  const long long r = (long long)blockIdx.x * 32 + c;
  const bool rv = r < K;
  const size_t hbytes = (size_t)K * kM3N * 4;
  const __amdgpu_buffer_rsrc_t h1r = m3_rsrc(H1T, hbytes), h2r = m3_rsrc(H2T, hbytes), z2r = m3_rsrc(dZ2T, hbytes),
                               z1r = m3_rsrc(dZ1T, hbytes);
  const unsigned roff = rv ? (unsigned)(r * 4) : kM3OOB, kstride = (unsigned)(K * 4);
  float dv[A];
#pragma unroll
  for (int a = 0; a < A; ++a) dv[a] = rv ? dout[r * A + a] : 0.f;
  float* pa = partA + (size_t)blockIdx.x * PA;
  const int jr = m3_lane_sum16_reg();
  float h1v[16];   // H1ᵀ of block w, used after the contraction
#pragma unroll
  for (int i = 0; i < 16; ++i) h1v[i] = m3_ld(h1r, roff + (unsigned)(32 * w + m3_row(i, h)) * kstride);
  if (w == 0)
#pragma unroll
    for (int a = 0; a < A; ++a) {   // Σ_r dout_a over the tile
      float t = h == 0 ? dv[a] : 0.f;
      for (int o = 16; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0) pa[N + A * N + a] = t;
    }
  // dZ2ᵀ block w; its bias / head partials (this wave's 32 hidden units)
  float mine[16], hw[A][16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 32 * w + m3_row(i, h);
    const float hv = m3_ld(h2r, roff + (unsigned)m * kstride);
    float g = 0.f;
#pragma unroll
    for (int a = 0; a < A; ++a) { g += dv[a] * W3[a * N + m]; hw[a][i] = dv[a] * hv; }
    mine[i] = g * (1.f - hv * hv);
    m3_st(z2r, roff + (unsigned)m * kstride, mine[i]);
  }
  const float sdb = m3_lane_sum16(mine);
  float sdw[A];
#pragma unroll
  for (int a = 0; a < A; ++a) sdw[a] = m3_lane_sum16(hw[a]);
  if ((c & 1) == 0) {   // tiles past K write zeros: every partial row is defined
    const int m = 32 * w + m3_row(jr, h);
    pa[m] = sdb;
#pragma unroll
    for (int a = 0; a < A; ++a) pa[N + a * N + m] = sdw[a];
  }
  // dH1ᵀ block w = (W2ᵀ)[w]·dZ2ᵀ; dZ1ᵀ = dH1ᵀ ⊙ (1 − H1ᵀ²)
  const float4* const w2t = reinterpret_cast<const float4*>(pack + m3_w1p_floats(Ip) + m3_w2_floats());
  f32x16 d;
  if constexpr (kM3wBwdLds) {
    float4* const xs4 = reinterpret_cast<float4*>(xs);
    m3w_share(xs4, mine, w);
    d = m3w_contract(w2t, w, xs4);
  } else {
    float zb[kM3Steps2];
    m3w_share_regs(xs, mine, zb, w);
    d = m3w_contract_regs(w2t, w, zb);
  }
  float z1[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = 32 * w + m3_row(i, h);
    z1[i] = d[i] * (1.f - h1v[i] * h1v[i]);
    m3_st(z1r, roff + (unsigned)n * kstride, z1[i]);
  }
  const float s1 = m3_lane_sum16(z1);
  if ((c & 1) == 0) partB[(size_t)blockIdx.x * N + 32 * w + m3_row(jr, h)] = s1;
}
}  // namespace


// ------------------------------------------------- row-major weight gradient
// nn.Linear's dW = dYᵀ·X for the 256-wide layers of a PPO minibatch (dW2 =
// dZ2ᵀ·H1, AG:733 / AG:759) straight from the row-major [K][N] / [K][M]
// activations the fused actor kernel writes, as chunk partials
// partial[c][N][M] (c < C, K/C rows each) summed by qs_mlp_sum_adam.
//
// A workgroup = 8 waves owns one 128×128 output tile of one chunk; waves 0-3
// take the chunk's first half of rows and waves 4-7 the second (a 64×64
// sub-tile each), and the halves are added through LDS at the end, so the
// chip holds two waves per SIMD without doubling the partials.  One k-step =
// 4 rows: lane (g, i) loads A[k + g][n0 + 4i .. +3] and B[k + g][m0 + 4i .. +3]
// as two 16-byte loads (four full 256-B row segments per wave instruction) and
// issues 16 v_mfma_f32_16x16x4_f32: element e of its A float4 is the A operand
// for output rows n0 + 4i' + e, element f of the B float4 the B operand for
// columns m0 + 4j + f, so no operand is shuffled.  Loads run four k-steps
// ahead.  blockIdx → (chunk, tile) keeps the four tiles of a chunk, which read
// the same rows, on one XCD (shared L2).
constexpr int kWrWaves = 8;
constexpr int kWrAhead = 4;
__global__ void __launch_bounds__(64 * kWrWaves) wgrad_rm_kernel(int N, int M, int Kc, int C,
                                                                const float* __restrict__ A,
                                                                const float* __restrict__ B,
                                                                float* __restrict__ partial) {
  __shared__ float4 red[4][16][64];   // the second half's accumulators, [sub-tile][acc][lane]
  const int TN = N / 128, TM = M / 128, T = TN * TM, total = T * C;
  int flat = (int)blockIdx.x;
  if (total % 8 == 0) flat = (flat & 7) * (total / 8) + (flat >> 3);   // XCD = blockIdx % 8
  const int chunk = flat / T, tile = flat - chunk * T;
  const int tn = tile / TM, tm = tile - tn * TM;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, i = l & 15;
  const int wq = w & 3, kh = w >> 2;
  const int nb = 128 * tn + 64 * (wq >> 1), mb = 128 * tm + 64 * (wq & 1);
  const int half = Kc / 2, steps = half / 4;
  const long long k0 = (long long)chunk * Kc + (long long)kh * half + g;
  const float4* pa = reinterpret_cast<const float4*>(A + k0 * N + nb + 4 * i);
  const float4* pb = reinterpret_cast<const float4*>(B + k0 * M + mb + 4 * i);
  const long long sa = (long long)N, sb = (long long)M;   // float4 stride of 4 rows
  f32x4 acc[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[e][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 ra[kWrAhead], rb[kWrAhead];
#pragma unroll
  for (int u = 0; u < kWrAhead; ++u) {
    ra[u] = u < steps ? pa[u * sa] : make_float4(0.f, 0.f, 0.f, 0.f);
    rb[u] = u < steps ? pb[u * sb] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int s0 = 0; s0 < steps; s0 += kWrAhead) {
#pragma unroll
    for (int u = 0; u < kWrAhead; ++u) {
      const int st = s0 + u;
      if (st < steps) {   // uniform
        const float4 a = ra[u], b = rb[u];
        if (st + kWrAhead < steps) {
          ra[u] = pa[(long long)(st + kWrAhead) * sa];
          rb[u] = pb[(long long)(st + kWrAhead) * sb];
        }
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int f = 0; f < 4; ++f) acc[e][f] = mfma16(av[e], bv[f], acc[e][f]);
      }
    }
  }
  if (kh == 1)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        red[wq][4 * e + f][l] = make_float4(acc[e][f][0], acc[e][f][1], acc[e][f][2], acc[e][f][3]);
  __syncthreads();
  if (kh == 1) return;
  // output (n, m) of acc[e][f][r]: n = nb + 4·(4g + r) + e, m = mb + 4i + f; the
  // four f of one (e, r) are one float4 of a partial row
  float* const out = partial + (size_t)chunk * N * M;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v[4][4];   // [r][f]
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float4 o = red[wq][4 * e + f][l];
      v[0][f] = acc[e][f][0] + o.x; v[1][f] = acc[e][f][1] + o.y;
      v[2][f] = acc[e][f][2] + o.z; v[3][f] = acc[e][f][3] + o.w;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + 4 * (4 * g + r) + e;
      *reinterpret_cast<float4*>(out + (size_t)n * M + mb + 4 * i) = make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
    }
  }
}

extern "C" {

const char* qs_learner_last_error(void) { return g_err.c_str(); }

int qs_gae(int32_t T, int64_t N, const float* rews, const float* vals, const float* masks, const float* terminal_vals,
           const float* last_val, double gamma, double gae_lambda, int32_t use_gae, double* rets, double* advs,
           void* stream) {
  if (T <= 0 || N <= 0 || !rews || !masks || !last_val || !rets || !advs)
    return fail(QS_E_INVALID, "qs_gae: bad argument");
  const int block = 256;
  const long long grid = (N + block - 1) / block;
  hipLaunchKernelGGL(gae_kernel, dim3((unsigned)grid), dim3(block), 0, (hipStream_t)stream, (int)T, (long long)N, rews,
                     vals, masks, terminal_vals, last_val, gamma, gae_lambda, (int)use_gae, rets, advs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_gae: ") + hipGetErrorString(e));
}

int qs_adam_gated(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, const float* step,
                  float lr, float beta1, float beta2, float eps, const float* gate_val, float gate_thr, void* stream) {
  if (n <= 0 || !params || !grads || !exp_avg || !exp_avg_sq || !step) return fail(QS_E_INVALID, "qs_adam_gated: bad argument");
  const int block = 256;
  long long grid = (n + block - 1) / block;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)grid), dim3(block), 0, (hipStream_t)stream, (long long)n, params, grads,
                     exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, gate_val, gate_thr);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_adam_gated: ") + hipGetErrorString(e));
}

int qs_adam_commit(float* step, const float* gate_val, float gate_thr, void* stream) {
  if (!step) return fail(QS_E_INVALID, "qs_adam_commit: bad argument");
  hipLaunchKernelGGL(adam_commit_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, gate_val, gate_thr);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_adam_commit: ") + hipGetErrorString(e));
}

int64_t qs_ppo_heads_work_bytes(int32_t mb, int32_t D) {
  const int64_t rows = (int64_t)mb * D;
  const int64_t blocks = (std::max<int64_t>(rows, mb) + kHeadsBlock - 1) / kHeadsBlock;
  return 64 + blocks * kHeadsSums * (int64_t)sizeof(double);
}

int qs_ppo_heads(int32_t mb, int32_t D, int32_t A, const int64_t* idx, const float* mean, const float* logstd,
                 float action_scale, const float* act, const float* logp_old, const double* adv, const double* ret,
                 const float* v, float clip, float ent_coef, float* dmean, float* dlogstd, float* dv, float* kl_out,
                 double* acc, void* work, void* stream) {
  if (mb <= 0 || D <= 0 || A <= 0 || A > kMaxA || !idx || !mean || !logstd || !act || !logp_old || !adv || !ret || !v ||
      !dmean || !dlogstd || !dv || !kl_out || !acc || !work)
    return fail(QS_E_INVALID, "qs_ppo_heads: bad argument");
  const long long rows = (long long)mb * D;
  const unsigned blocks = (unsigned)((std::max<long long>(rows, mb) + kHeadsBlock - 1) / kHeadsBlock);
  unsigned* count = (unsigned*)work;
  double* partial = (double*)((char*)work + 64);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kHeadsBlock), 0, (hipStream_t)stream, (int)mb, (int)D,
                       (const long long*)idx, mean, logstd, action_scale, act, logp_old, adv, ret, v, clip, ent_coef,
                       dmean, dlogstd, dv, kl_out, acc, partial, count);
  };
  switch (A) {
    case 1: go(ppo_heads_kernel<1>); break;
    case 2: go(ppo_heads_kernel<2>); break;
    case 3: go(ppo_heads_kernel<3>); break;
    default: go(ppo_heads_kernel<4>); break;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_ppo_heads: ") + hipGetErrorString(e));
}

static int mlp_c(int32_t N) { return (N % 64 == 0 && (N / 64 == 1 || N / 64 == 2 || N / 64 == 4 || N / 64 == 8)) ? N / 64 : 0; }

int qs_mlp_bias_tanh(int64_t K, int32_t N, const float* z, const float* b, float* h, int32_t A, const float* w3,
                     const float* b3, float* out, void* stream) {
  const int C = mlp_c(N);
  if (K <= 0 || !C || !z || !b || !h || A < 0 || A > kMlpMaxA || (A > 0 && (!w3 || !b3 || !out)))
    return fail(QS_E_INVALID, "qs_mlp_bias_tanh: bad argument (N must be 64, 128, 256 or 512; A <= 4)");
  long long waves = K < 8192 ? K : 8192;
  const unsigned grid = (unsigned)((waves + 3) / 4);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kMlpBlock), 0, (hipStream_t)stream, (long long)K, z, b, h, (int)A, w3, b3, out);
  };
  switch (C) {
    case 1: go(mlp_bias_tanh_kernel<1>); break;
    case 2: go(mlp_bias_tanh_kernel<2>); break;
    case 4: go(mlp_bias_tanh_kernel<4>); break;
    default: go(mlp_bias_tanh_kernel<8>); break;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_bias_tanh: ") + hipGetErrorString(e));
}

int32_t qs_mlp_bwd_blocks(int64_t K) {
  const long long g = (K + 63) / 64;
  return (int32_t)(g < kMlpBwdMaxG ? (g < 1 ? 1 : g) : kMlpBwdMaxG);
}

int qs_mlp_tanh_bwd(int64_t K, int32_t N, const float* dh, const float* dout, int32_t A, const float* w3, const float* h,
                    float* dz, float* partial, void* stream) {
  const int C = mlp_c(N);
  if (K <= 0 || !C || !h || !dz || !partial || A < 0 || A > kMlpMaxA || (A == 0 && !dh) || (A > 0 && (!dout || !w3)) ||
      (C == 8 && A > 1))
    return fail(QS_E_INVALID, "qs_mlp_tanh_bwd: bad argument (N in {64,128,256,512}; A <= 4, A <= 1 at N = 512)");
  const int G = qs_mlp_bwd_blocks(K);
  const long long rpb = (K + G - 1) / G;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(kMlpBwdBlock), 0, (hipStream_t)stream, (long long)K, rpb, dh, dout, w3, h, dz, partial);
  };
#define QS_MLP_BWD_CASE(CC)                                   \
  case CC:                                                    \
    switch (A) {                                              \
      case 0: go(mlp_tanh_bwd_kernel<CC, 0>); break;          \
      case 1: go(mlp_tanh_bwd_kernel<CC, 1>); break;          \
      case 2: if constexpr (CC < 8) go(mlp_tanh_bwd_kernel<CC, 2>); break; \
      case 3: if constexpr (CC < 8) go(mlp_tanh_bwd_kernel<CC, 3>); break; \
      default: if constexpr (CC < 8) go(mlp_tanh_bwd_kernel<CC, 4>); break; \
    }                                                         \
    break;
  switch (C) {
    QS_MLP_BWD_CASE(1)
    QS_MLP_BWD_CASE(2)
    QS_MLP_BWD_CASE(4)
    QS_MLP_BWD_CASE(8)
  }
#undef QS_MLP_BWD_CASE
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_tanh_bwd: ") + hipGetErrorString(e));
}

int qs_mlp_sum_partials(int32_t G, int64_t P, const float* partial, float* d0, int64_t n0, float* d1, int64_t n1,
                        float* d2, void* stream) {
  if (G <= 0 || P <= 0 || !partial || !d0 || n0 <= 0 || n0 > P || (n0 < P && !d1) || (n0 + n1 < P && !d2) ||
      n1 < 0 || n0 + n1 > P)
    return fail(QS_E_INVALID, "qs_mlp_sum_partials: bad argument");
  const unsigned grid = (unsigned)((P + 63) / 64);
  hipLaunchKernelGGL(mlp_sum_partials_kernel, dim3(grid), dim3(kMlpSumBlock), 0, (hipStream_t)stream, (int)G, (long long)P,
                     partial, d0, (long long)n0, d1, (long long)n1, d2);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_sum_partials: ") + hipGetErrorString(e));
}

static int build_sum_tasks(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial,
                           float* const* d0, const int64_t* n0, float* const* d1, const int64_t* n1, float* const* d2,
                           MlpSumTasks& T, int& blocks, const char* name) {
  if (n <= 0 || n > kMlpMaxTasks || !G || !P || !partial || !d0 || !n0 || !d1 || !n1 || !d2)
    return fail(QS_E_INVALID, std::string(name) + ": bad argument (1..16 tasks)");
  T = MlpSumTasks{};
  T.n = n;
  blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (G[i] <= 0 || P[i] <= 0 || !partial[i] || !d0[i] || n0[i] <= 0 || n0[i] > P[i] || n1[i] < 0 ||
        n0[i] + n1[i] > P[i] || (n0[i] < P[i] && !d1[i]) || (n0[i] + n1[i] < P[i] && !d2[i]))
      return fail(QS_E_INVALID, std::string(name) + ": bad task");
    T.t[i] = MlpSumTask{partial[i], d0[i], d1[i], d2[i], (long long)P[i], (long long)n0[i], (long long)n1[i], (int)G[i]};
    T.start[i] = blocks;
    int wg = 1;   // mlp_sum_wg
    while (wg < G[i] && wg < 16) wg <<= 1;
    const int64_t span = (int64_t)(kMlpSumBlock / 64 / wg) * 64 * mlp_sum_cols(G[i]);   // columns per block
    blocks += (int)((P[i] + span - 1) / span);
  }
  T.start[n] = blocks;
  return QS_OK;
}

int qs_mlp_sum_partials_multi(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial,
                              float* const* d0, const int64_t* n0, float* const* d1, const int64_t* n1,
                              float* const* d2, void* stream) {
  MlpSumTasks T;
  int blocks;
  const int rc = build_sum_tasks(n, G, P, partial, d0, n0, d1, n1, d2, T, blocks, "qs_mlp_sum_partials_multi");
  if (rc != QS_OK) return rc;
  hipLaunchKernelGGL(mlp_sum_multi_kernel, dim3(blocks), dim3(kMlpSumBlock), 0, (hipStream_t)stream, T);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_sum_partials_multi: ") + hipGetErrorString(e));
}

// the 8-wave-per-tile kernels below 512 tiles (too few waves otherwise) and for
// wide inputs (their X tile is staged through LDS once, where the 4-tile
// kernel gathers every lane's row per k-quad)
// The 4-wave kernel (128 rows per workgroup, one workgroup per CU) below 16 384
// rows leaves CUs idle; above 64 inputs its per-lane X loads cost more than the
// 8-wave kernel's LDS tile, except with whole rounds of workgroups (measured
// with scripts/mlp3_fwd_probe.py: K 65 536 × I 72 116.5 µs vs 133.6 wide,
// K 40 960 × I 119 127.4 vs 96.7)
static bool m3_wide(int64_t K, int32_t I) { return K < 16384 || I > (K >= 65536 ? 72 : 64); }
// The forward's choice (it leaves no partials, so it need not follow the
// backward's tiles): the 8-wave kernel at every shape since its exchange moved
// to LDS (101 VGPRs, two workgroups per CU) — C3 / C4 / C5 rollout 180 / 82 /
// 111 µs against the 4-wave kernel's 186 / 127 / 115 (scripts/mlp3_fwd_probe.py).
static bool m3_wide_fwd(int64_t K, int32_t I) {
#ifdef QS_M3_FORCE_WIDE   // dev probe: every forward on the 8-wave (1) or the 4-wave (0) kernels
  return QS_M3_FORCE_WIDE || (void(K), void(I), false);
#else
  (void)K; (void)I;
  return true;
#endif
}
int32_t qs_mlp3_tiles(int64_t K, int32_t I) { return (int32_t)(m3_wide(K, I) ? (K + 31) / 32 : (K + 127) / 128); }   // partial rows

int64_t qs_mlp3_pack_floats(int32_t I) {
  const int64_t Ip = (I + 31) & ~31;
  return (Ip / 8) * kM3NB * 256 + 2 * (int64_t)kM3NB * 32 * 256;
}

int qs_mlp3_pack(int32_t I, int32_t N, const float* W1, const float* W2, float* pack, void* stream) {
  if (I <= 0 || I > 1024 || N != kM3N || !W1 || !W2 || !pack) return fail(QS_E_INVALID, "qs_mlp3_pack: bad argument");
  const int64_t n = qs_mlp3_pack_floats(I);
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(mlp3_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int)I, W1, W2, pack);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp3_pack: ") + hipGetErrorString(e));
}

static int mlp3_fwd_launch(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const int64_t* rows, float* Xg,
                           int32_t G, const float* pack, const float* b1, const float* b2, const float* W3,
                           const float* b3, float* H1T, float* H2T, float* out, void* stream, const char* name,
                           M3ValueHead vh = M3ValueHead{}) {
  if (K <= 0 || K * kM3N * 4 >= (int64_t(1) << 31) || K * (int64_t)I * 4 >= (int64_t(1) << 31) || I <= 0 || I > 1024 || N != kM3N || A < 1 || A > 4 || !X || !pack ||
      !b1 || !b2 || !W3 || !b3 || (!H1T) != (!H2T) || !out)
    return fail(QS_E_INVALID, std::string(name) + ": bad argument (N must be 256, 1 <= A <= 4, I <= 1024)");
  if (G < 1 || (G > 1 && Xg)) return fail(QS_E_INVALID, std::string(name) + ": bad group size");
  // the row-gathering form with a gathered copy (G = 1) is the 8-wave kernel's
  const bool wide = (rows && G == 1) || m3_wide_fwd(K, I);
  if (vh.dv && (!wide || A != 1)) return fail(QS_E_INVALID, std::string(name) + ": the value head needs the 8-wave kernel and A = 1");
  const unsigned grid = (unsigned)(wide ? (K + 31) / 32 : qs_mlp3_tiles(K, I));
  const unsigned lds = wide ? (unsigned)(m3w_lds_floats((I + 31) & ~31) * sizeof(float)) : 0u;
  const long long* rr = (const long long*)rows;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kM3Block), 0, (hipStream_t)stream, (long long)K, (int)I, X, pack, b1, b2,
                       W3, b3, H1T, H2T, out, rr, (int)G);
  };
  auto gow = [&](auto kern) {
    if (lds > 65536u) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kM3WBlock), lds, (hipStream_t)stream, (long long)K, (int)I, X, pack, b1,
                       b2, W3, b3, H1T, H2T, out, rr, Xg, (int)G, vh);
  };
  if (rows && !wide) {
    switch (A) {
      case 1: go(mlp3_fwd_kernel<1, true>); break;
      case 2: go(mlp3_fwd_kernel<2, true>); break;
      case 3: go(mlp3_fwd_kernel<3, true>); break;
      default: go(mlp3_fwd_kernel<4, true>); break;
    }
  } else {
    switch (A) {
      case 1: wide ? gow(mlp3w_fwd_kernel<1>) : go(mlp3_fwd_kernel<1>); break;
      case 2: wide ? gow(mlp3w_fwd_kernel<2>) : go(mlp3_fwd_kernel<2>); break;
      case 3: wide ? gow(mlp3w_fwd_kernel<3>) : go(mlp3_fwd_kernel<3>); break;
      default: wide ? gow(mlp3w_fwd_kernel<4>) : go(mlp3_fwd_kernel<4>); break;
    }
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string(name) + ": " + hipGetErrorString(e));
}

int qs_mlp3_fwd(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const float* pack, const float* b1,
                const float* b2, const float* W3, const float* b3, float* H1T, float* H2T, float* out, void* stream) {
  return mlp3_fwd_launch(K, I, N, A, X, nullptr, nullptr, 1, pack, b1, b2, W3, b3, H1T, H2T, out, stream, "qs_mlp3_fwd");
}

int qs_mlp3_fwd_rows(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const int64_t* rows, float* Xg,
                     const float* pack, const float* b1, const float* b2, const float* W3, const float* b3, float* H1T,
                     float* H2T, float* out, void* stream) {
  if (!rows) return fail(QS_E_INVALID, "qs_mlp3_fwd_rows: rows is NULL");
  return mlp3_fwd_launch(K, I, N, A, X, rows, Xg, 1, pack, b1, b2, W3, b3, H1T, H2T, out, stream, "qs_mlp3_fwd_rows");
}

int64_t qs_mlp3_value_work_bytes(int64_t K) { return K > 0 ? 64 + 8 * ((K + 31) / 32) : 0; }

int qs_mlp3_fwd_rows_value(int64_t K, int32_t I, int32_t D, const float* X, const int64_t* rows, float* Xg,
                           const float* pack, const float* b1, const float* b2, const float* W3, const float* b3,
                           float* H1T, float* H2T, float* out, const double* ret, float* dv, double* acc, void* work,
                           void* stream) {
  if (!rows || !ret || !dv || !acc || !work || D <= 0 || K <= 0 || K > (1LL << 31) - 1)
    return fail(QS_E_INVALID, "qs_mlp3_fwd_rows_value: bad argument");
  M3ValueHead vh;
  vh.ret = ret;
  vh.dv = dv;
  vh.count = (unsigned*)work;
  vh.lossp = (double*)((char*)work + 64);
  vh.acc = acc;
  vh.D = D;
  vh.mb = (int)K;
  return mlp3_fwd_launch(K, I, kM3N, 1, X, rows, Xg, 1, pack, b1, b2, W3, b3, H1T, H2T, out, stream,
                         "qs_mlp3_fwd_rows_value", vh);
}

int qs_mlp3_fwd_group_rows(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const int64_t* rows, int32_t G,
                           const float* pack, const float* b1, const float* b2, const float* W3, const float* b3,
                           float* H1T, float* H2T, float* out, void* stream) {
  if (!rows) return fail(QS_E_INVALID, "qs_mlp3_fwd_group_rows: rows is NULL");
  if (G < 1 || K % G) return fail(QS_E_INVALID, "qs_mlp3_fwd_group_rows: K must be a multiple of G >= 1");
  return mlp3_fwd_launch(K, I, N, A, X, rows, nullptr, G, pack, b1, b2, W3, b3, H1T, H2T, out, stream,
                         "qs_mlp3_fwd_group_rows");
}

int qs_mlp3_bwd(int64_t K, int32_t I, int32_t N, int32_t A, const float* dout, const float* H1T, const float* H2T,
                const float* pack, const float* W3, float* dZ2T, float* dZ1T, float* partA, float* partB,
                void* stream) {
  if (K <= 0 || K * kM3N * 4 >= (int64_t(1) << 31) || K * (int64_t)I * 4 >= (int64_t(1) << 31) || I <= 0 || I > 1024 || N != kM3N || A < 1 || A > 4 || !dout ||
      !H1T || !H2T || !pack || !W3 || !dZ2T || !dZ1T || !partA || !partB)
    return fail(QS_E_INVALID, "qs_mlp3_bwd: bad argument (N must be 256, 1 <= A <= 4)");
  const bool wide = m3_wide(K, I);
  const unsigned grid = (unsigned)qs_mlp3_tiles(K, I);
  const int Ip = (I + 31) & ~31;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(wide ? kM3WBlock : kM3Block), 0, (hipStream_t)stream, (long long)K,
                       dout, H1T, H2T, pack, Ip, W3, dZ2T, dZ1T, partA, partB);
  };
  switch (A) {
    case 1: wide ? go(mlp3w_bwd_kernel<1>) : go(mlp3_bwd_kernel<1>); break;
    case 2: wide ? go(mlp3w_bwd_kernel<2>) : go(mlp3_bwd_kernel<2>); break;
    case 3: wide ? go(mlp3w_bwd_kernel<3>) : go(mlp3_bwd_kernel<3>); break;
    default: wide ? go(mlp3w_bwd_kernel<4>) : go(mlp3_bwd_kernel<4>); break;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp3_bwd: ") + hipGetErrorString(e));
}

static int build_adam_segs(int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                           float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr,
                           const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                           const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                           const int32_t* pack_I, int32_t zero_grads, AdamSegs& S, const char* name) {
  if (nseg <= 0 || nseg > kAdamMaxSeg || !params || !grads || !exp_avg || !exp_avg_sq || !step || !n || !lr || !beta1 ||
      !beta2 || !eps || !gate_val || !gate_thr)
    return fail(QS_E_INVALID, std::string(name) + ": bad argument (1..4 segments)");
  S = AdamSegs{};
  S.n = nseg;
  int blocks = 0;
  for (int i = 0; i < nseg; ++i) {
    if (n[i] <= 0 || !params[i] || !grads[i] || !exp_avg[i] || !exp_avg_sq[i] || !step[i])
      return fail(QS_E_INVALID, std::string(name) + ": bad segment");
    float* pk = pack ? pack[i] : nullptr;
    // pack_I: the MLP's input width, | QS_PACK_F16 for a qs_mlp3f_pack image
    const int I = pk ? (pack_I[i] & ~(QS_PACK_F16 | QS_PACK_W2T)) : 0;
    const int kind = !pk ? 0 : (pack_I[i] & QS_PACK_F16) ? 1 : (pack_I[i] & QS_PACK_W2T) ? 2 : 0;
    if (pk && (I <= 0 || I > 1024 || w1_off[i] < 0 || w2_off[i] < 0 || w1_off[i] + (int64_t)kM3N * I > n[i] ||
               w2_off[i] + (int64_t)kM3N * kM3N > n[i]))
      return fail(QS_E_INVALID, std::string(name) + ": bad pack segment");
    S.s[i] = AdamSeg{params[i], grads[i], exp_avg[i], exp_avg_sq[i], step[i], gate_val[i], pk, (long long)n[i],
                     pk ? (long long)w1_off[i] : 0, pk ? (long long)w2_off[i] : 0, lr[i], beta1[i], beta2[i], eps[i],
                     gate_thr[i], I, zero_grads ? 1 : 0, kind};
    S.start[i] = blocks;
    blocks += (int)std::min<int64_t>((n[i] + kAdamBlock * kAdamPer - 1) / (kAdamBlock * kAdamPer), kAdamSegBlocks);
  }
  S.start[nseg] = blocks;
  return QS_OK;
}

static int adam_multi_launch(int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr,
                             const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                             const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                             const int32_t* pack_I, int32_t zero_grads, void* work, void* stream, const char* name) {
  if (!work) return fail(QS_E_INVALID, std::string(name) + ": bad argument (work)");
  AdamSegs S;
  const int rc = build_adam_segs(nseg, params, grads, exp_avg, exp_avg_sq, step, n, lr, beta1, beta2, eps, gate_val,
                                 gate_thr, pack, w1_off, w2_off, pack_I, zero_grads, S, name);
  if (rc != QS_OK) return rc;
  hipLaunchKernelGGL(adam_multi_kernel, dim3(S.start[nseg]), dim3(kAdamBlock), 0, (hipStream_t)stream, S,
                     (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string(name) + ": " + hipGetErrorString(e));
}

int64_t qs_mlp_sum_adam_work_bytes(void) { return (int64_t)kSumAdamStride * (1 + kSumAdamGroups) * 4; }

int qs_mlp_sum_adam(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial, float* const* d0,
                    const int64_t* n0, float* const* d1, const int64_t* n1, float* const* d2, const int32_t* task_seg,
                    int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, float* const* step, const int64_t* nel, const float* lr,
                    const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                    const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                    const int32_t* pack_I, void* work, void* stream) {
  const char* name = "qs_mlp_sum_adam";
  MlpSumTasks T;
  int blocks;
  int rc = build_sum_tasks(n, G, P, partial, d0, n0, d1, n1, d2, T, blocks, name);
  if (rc != QS_OK) return rc;
  AdamSegs S;
  rc = build_adam_segs(nseg, params, grads, exp_avg, exp_avg_sq, step, nel, lr, beta1, beta2, eps, gate_val, gate_thr,
                       pack, w1_off, w2_off, pack_I, 0, S, name);
  if (rc != QS_OK) return rc;
  if (!task_seg || !work) return fail(QS_E_INVALID, std::string(name) + ": bad argument");
  if (blocks > kSumAdamGroups * kSumAdamGroup)
    return fail(QS_E_INVALID, std::string(name) + ": more than " + std::to_string(kSumAdamGroups * kSumAdamGroup) +
                                  " blocks of columns");
  SegOf seg{};
  for (int i = 0; i < n; ++i) {   // every destination element inside its segment's gradient buffer
    if (task_seg[i] < 0 || task_seg[i] >= nseg) return fail(QS_E_INVALID, std::string(name) + ": bad task segment");
    seg.s[i] = task_seg[i];
    const float* g0 = grads[task_seg[i]];
    const float* g1 = g0 + nel[task_seg[i]];
    auto inside = [&](const float* d, int64_t len) { return len <= 0 || (d >= g0 && d + len <= g1); };
    if (!inside(d0[i], n0[i]) || !inside(d1[i], n1[i]) || !inside(d2[i], P[i] - n0[i] - n1[i]))
      return fail(QS_E_INVALID, std::string(name) + ": a task destination lies outside its segment's gradients");
  }
  hipLaunchKernelGGL(mlp_sum_adam_kernel, dim3(blocks), dim3(kMlpSumBlock), 0, (hipStream_t)stream, T, S, seg,
                     (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string(name) + ": " + hipGetErrorString(e));
}

int qs_adam_multi(int32_t nseg, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr, const float* beta1,
                  const float* beta2, const float* eps, const float* const* gate_val, const float* gate_thr, void* work,
                  void* stream) {
  return adam_multi_launch(nseg, params, (float* const*)grads, exp_avg, exp_avg_sq, step, n, lr, beta1, beta2, eps,
                           gate_val, gate_thr, nullptr, nullptr, nullptr, nullptr, 0, work, stream, "qs_adam_multi");
}

int qs_adam_multi_pack(int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr,
                       const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                       const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                       const int32_t* pack_I, int32_t zero_grads, void* work, void* stream) {
  if (!pack || !w1_off || !w2_off || !pack_I) return fail(QS_E_INVALID, "qs_adam_multi_pack: bad argument");
  return adam_multi_launch(nseg, params, grads, exp_avg, exp_avg_sq, step, n, lr, beta1, beta2, eps, gate_val,
                           gate_thr, pack, w1_off, w2_off, pack_I, zero_grads, work, stream, "qs_adam_multi_pack");
}

int qs_adam_step(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* step, float lr,
                 float beta1, float beta2, float eps, const float* gate_val, float gate_thr, void* work, void* stream) {
  if (n <= 0 || !params || !grads || !exp_avg || !exp_avg_sq || !step || !work)
    return fail(QS_E_INVALID, "qs_adam_step: bad argument");
  const int block = 256;
  long long grid = (n + block - 1) / block;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(adam_step_kernel, dim3((unsigned)grid), dim3(block), 0, (hipStream_t)stream, (long long)n, params,
                     grads, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, gate_val, gate_thr, (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_adam_step: ") + hipGetErrorString(e));
}

int qs_value_head(int32_t mb, int32_t D, const int64_t* idx, const double* ret, const float* v, float* dv, double* acc,
                  void* work, void* stream) {
  if (mb <= 0 || D <= 0 || !idx || !ret || !v || !dv || !acc || !work) return fail(QS_E_INVALID, "qs_value_head: bad argument");
  const unsigned blocks = (unsigned)((mb + kHeadsBlock - 1) / kHeadsBlock);
  hipLaunchKernelGGL((ppo_heads_kernel<1, false>), dim3(blocks), dim3(kHeadsBlock), 0, (hipStream_t)stream, (int)mb,
                     (int)D, (const long long*)idx, nullptr, nullptr, 1.0f, nullptr, nullptr, nullptr, ret, v, 0.f, 0.f,
                     nullptr, nullptr, dv, nullptr, acc, (double*)((char*)work + 64), (unsigned*)work);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_value_head: ") + hipGetErrorString(e));
}

#ifdef QS_F_STAMP
int qs_mlp3f_stamps(unsigned long long* host, int64_t n) {   // dev probe: copy out the phase stamps
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fstamp), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
#endif

int32_t qs_mlp3f_tiles(int64_t K) { return K <= 0 ? 0 : (int32_t)((K + 16 * kFWaves - 1) / (16 * kFWaves)); }
int64_t qs_mlp3f_pack_floats(int32_t I) { return I <= 0 ? 0 : f16_w1_floats(f16_ip(I)) + 2 * kFW2Floats; }
int64_t qs_mlp3f_work_bytes(int64_t K) { return 64 + (int64_t)qs_mlp3f_tiles(K) * (2 + kMaxA) * (int64_t)sizeof(double); }

int qs_mlp3f_pack(int32_t I, const float* W1, const float* W2, float* pack, void* stream) {
  if (I <= 0 || f16_ip(I) > kFMaxIp || !W1 || !W2 || !pack) return fail(QS_E_INVALID, "qs_mlp3f_pack: bad argument (I <= 128)");
  const int64_t n = qs_mlp3f_pack_floats(I);
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(mlp3f_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int)I, W1, W2, pack);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp3f_pack: ") + hipGetErrorString(e));
}

int qs_mlp3f_actor(int64_t K, int32_t I, int32_t D, int32_t A, const float* X, const int64_t* idx, const float* pack,
                   const float* b1, const float* b2, const float* W3, const float* b3, const float* logstd,
                   float action_scale, const float* act, const float* logp_old, const double* adv, float clip,
                   float ent_coef, float* Xa, float* H1T, float* dZ2T, float* dZ1T, float* partA, float* partB,
                   float* dlogstd, float* kl_out, double* acc, void* work, float* mean_out, void* stream) {
  if (!dZ1T) return fail(QS_E_INVALID, "qs_mlp3f_actor: dZ1T is NULL (qs_mlp3f_actor_w1 folds dW1 instead)");
  return qs_mlp3f_actor_w1(K, I, D, A, X, idx, pack, b1, b2, W3, b3, logstd, action_scale, act, logp_old, adv, clip,
                           ent_coef, Xa, H1T, dZ2T, dZ1T, partA, partB, dlogstd, kl_out, acc, work, mean_out, nullptr,
                           stream);
}

int qs_mlp3f_actor_w1(int64_t K, int32_t I, int32_t D, int32_t A, const float* X, const int64_t* idx, const float* pack,
                      const float* b1, const float* b2, const float* W3, const float* b3, const float* logstd,
                      float action_scale, const float* act, const float* logp_old, const double* adv, float clip,
                      float ent_coef, float* Xa, float* H1T, float* dZ2T, float* dZ1T, float* partA, float* partB,
                      float* dlogstd, float* kl_out, double* acc, void* work, float* mean_out, float* part_w1,
                      void* stream) {
  if (K <= 0 || D <= 0 || K % D || K * kM3N * 4 >= (int64_t(1) << 31) || I <= 0 || f16_ip(I) > kFMaxIp || A < 1 ||
      A > kMaxA || !X || !idx || !pack || !b1 || !b2 || !W3 || !b3 || !logstd || !act || !logp_old || !adv || !Xa ||
      !H1T || !dZ2T || (!dZ1T && !part_w1) || !partA || !partB || !dlogstd || !kl_out || !acc || !work)
    return fail(QS_E_INVALID, "qs_mlp3f_actor: bad argument (K a multiple of D, K·1024 < 2^31, I <= 128, 1 <= A <= 4)");
  const unsigned grid = (unsigned)qs_mlp3f_tiles(K);
  unsigned* count = (unsigned*)work;
  double* lossp = (double*)((char*)work + 64);
  // the folded dW1's LDS: dZ1 half [128][144] + the X tile [128][Ip + 16]
  const int w1_lds = part_w1 ? 128 * 144 + 128 * (f16_ip(I) + 16) : 0;
  auto go = [&](auto kern, int AA) {
    const int lds = std::max(f_lds_floats(AA), w1_lds) * (int)sizeof(float);
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kFBlock), (unsigned)lds, (hipStream_t)stream, (long long)K, (int)I, (int)D,
                       X, (const long long*)idx, pack, b1, b2, W3, b3, logstd, action_scale, act, logp_old, adv, clip,
                       ent_coef, Xa, H1T, dZ2T, dZ1T, partA, partB, lossp, dlogstd, kl_out, acc, count, mean_out, part_w1);
  };
  switch (A) {
    case 1: go(mlp3f_actor_kernel<1>, 1); break;
    case 2: go(mlp3f_actor_kernel<2>, 2); break;
    case 3: go(mlp3f_actor_kernel<3>, 3); break;
    default: go(mlp3f_actor_kernel<4>, 4); break;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp3f_actor: ") + hipGetErrorString(e));
}

int32_t qs_mlp_wgrad_x_chunks(int64_t K, int32_t M) {
  return (K > 0 && K % kWxR == 0 && M > 0 && M <= 256) ? (int32_t)(K / kWxR) : 0;
}

int qs_mlp_wgrad_x(int64_t K, int32_t N, int32_t M, const float* AT, int32_t at_blocked, const float* X,
                   float* partial, void* stream) {
  if (K <= 0 || K % kWxR || N != kM3N || M <= 0 || M > 256 || !AT || !X || !partial || ((uintptr_t)AT & 15))
    return fail(QS_E_INVALID, "qs_mlp_wgrad_x: bad argument (K a multiple of 128, N = 256, M <= 256, AT 16-B aligned)");
  const dim3 grid((unsigned)(K / kWxR), (unsigned)((M + 31) / 32));
  if (at_blocked)
    hipLaunchKernelGGL(mlp_wgrad_x_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, (long long)K, (int)M, AT, X,
                       partial);
  else
    hipLaunchKernelGGL(mlp_wgrad_x_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, (long long)K, (int)M, AT, X,
                       partial);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_wgrad_x: ") + hipGetErrorString(e));
}

// chunks of qs_mlp_wgrad: the most (a power of two, <= 256) that keeps every
// chunk a multiple of 64 rows (the kernel's load batch)
int32_t qs_mlp_wgrad_chunks(int64_t K, int32_t N, int32_t M) {
  if (K <= 0 || N <= 0 || M <= 0) return 0;
  const int64_t tiles = (int64_t)((N + 31) / 32) * ((M + 31) / 32);
  int32_t C = 1;   // chunks of 64·k rows; <= 4 096 waves; partials <= 8 MiB
  while (C < 256 && K % (128 * (int64_t)C) == 0 && tiles * C * 2 <= 4096 &&
         (int64_t)2 * C * N * M * 4 <= (int64_t(8) << 20))
    C *= 2;
  return K % (64 * (int64_t)C) == 0 ? C : 0;
}

int qs_mlp_wgrad(int64_t K, int32_t N, int32_t M, const float* AT, const float* B, int32_t b_transposed, int32_t C,
                 float* partial, void* stream) {
  if (K <= 0 || N <= 0 || N % 32 || M <= 0 || C <= 0 || K % (64 * (int64_t)C) || !AT || !B || !partial ||
      ((uintptr_t)AT & 15) || (K & 3) || (b_transposed && ((uintptr_t)B & 15)))
    return fail(QS_E_INVALID, "qs_mlp_wgrad: bad argument (N % 32 == 0, K a multiple of 64·C, AT/BT 16-B aligned)");
  const int R = (int)(K / C);
  const dim3 grid((unsigned)((N / 32 + kWgWaves - 1) / kWgWaves), (unsigned)((M + 31) / 32), (unsigned)C);
  if (b_transposed)
    hipLaunchKernelGGL(mlp_wgrad_kernel<true>, grid, dim3(64 * kWgWaves), 0, (hipStream_t)stream, (long long)K, (int)N,
                       (int)M, R, AT, B, partial);
  else
    hipLaunchKernelGGL(mlp_wgrad_kernel<false>, grid, dim3(64 * kWgWaves), 0, (hipStream_t)stream, (long long)K, (int)N,
                       (int)M, R, AT, B, partial);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_wgrad: ") + hipGetErrorString(e));
}


int qs_wgrad_rm(int64_t K, int32_t N, int32_t M, const float* A, const float* B, int32_t C, float* partial,
                void* stream) {
  if (K <= 0 || N <= 0 || M <= 0 || N % 128 || M % 128 || C <= 0 || K % (8 * (int64_t)C) || !A || !B || !partial ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)partial & 15) || K / C > (int64_t)1 << 30 ||
      (int64_t)(N / 128) * (M / 128) * C > (int64_t)1 << 30)
    return fail(QS_E_INVALID, "qs_wgrad_rm: bad argument (N, M multiples of 128, K a multiple of 8·C, 16-B aligned)");
  const int grid = (N / 128) * (M / 128) * C;
  hipLaunchKernelGGL(wgrad_rm_kernel, dim3(grid), dim3(64 * kWrWaves), 0, (hipStream_t)stream, (int)N, (int)M,
                     (int)(K / C), (int)C, A, B, partial);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_wgrad_rm: ") + hipGetErrorString(e));
}

}  // extern "C"
