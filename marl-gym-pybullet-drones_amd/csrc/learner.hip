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
#include <cstdint>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }

__global__ void gae_kernel(int T, long long N, const float* __restrict__ rews, const float* __restrict__ vals,
                           const float* __restrict__ masks, const float* __restrict__ tvals,
                           const float* __restrict__ last_val, double gamma, double lam, int use_gae,
                           double* __restrict__ rets, double* __restrict__ advs) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const double lv = (double)last_val[n];
  double ret = lv, adv = 0.0, vnext = lv;
#pragma unroll 4
  for (int t = T - 1; t >= 0; --t) {
    const long long k = (long long)t * N + n;
    const double r = (double)rews[k];
    const double m = (double)masks[k];
    const double v = vals ? (double)vals[k] : 0.0;
    const double tv = tvals ? (double)tvals[k] : 0.0;
    const double ra = r + gamma * tv;                       // buffer.py:593
    ret = ra + gamma * m * ret;                             // buffer.py:602
    if (use_gae) {
      const double td = ra + gamma * m * vnext - v;         // buffer.py:608
      adv = adv * lam * gamma * m + td;                     // buffer.py:609
    } else {
      adv = ret - v;                                        // buffer.py:606
    }
    rets[k] = ret;
    advs[k] = adv;
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

__device__ __forceinline__ double block_sum(double x, double* lds) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) lds[w] = x;
  __syncthreads();
  double t = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += lds[k];
  return t;   // valid in thread 0
}

// A (actions per agent) is a template value: the per-action arrays stay in
// registers (a run-time A put them in scratch memory and cost ~70 µs a launch).
template <int A>
__global__ void __launch_bounds__(kHeadsBlock) ppo_heads_kernel(
    int mb, int D, const long long* __restrict__ idx, const float* __restrict__ mean,
    const float* __restrict__ logstd, float scale, const float* __restrict__ act, const float* __restrict__ logp_old,
    const double* __restrict__ adv, const double* __restrict__ ret, const float* __restrict__ v, float clip,
    float ent_coef, float* __restrict__ dmean, float* __restrict__ dlogstd, float* __restrict__ dv,
    float* __restrict__ kl_out, double* __restrict__ acc, double* __restrict__ partial, unsigned* __restrict__ count) {
  __shared__ double lds[kHeadsBlock / 64];
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
  if (r < R) {
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
#pragma unroll
  for (int k = 0; k < 3 + A; ++k) {
    const double t = block_sum(sums[k], lds);
    if (threadIdx.x == 0) partial[(size_t)blockIdx.x * kHeadsSums + k] = t;
  }
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(count, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: every thread sums a fixed strided subset of the
  // partials in workgroup order, then the same fixed-order block reduction
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double tot[kHeadsSums];
#pragma unroll
  for (int k = 0; k < 3 + A; ++k) {
    double t = 0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) t += partial[(size_t)b * kHeadsSums + k];
    tot[k] = block_sum(t, lds);
  }
  if (threadIdx.x != 0) return;
  *count = 0;   // ready for the next launch (graph replay)
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
__global__ void __launch_bounds__(kMlpSumBlock) mlp_sum_multi_kernel(MlpSumTasks tasks) {
  constexpr int W = kMlpSumBlock / 64;
  __shared__ float lds[W][64];
  int ti = 0;
  while (ti + 1 < tasks.n && (int)blockIdx.x >= tasks.start[ti + 1]) ++ti;
  const MlpSumTask& T = tasks.t[ti];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long j = (long long)(blockIdx.x - tasks.start[ti]) * 64 + lane;
  float t = 0.f;
  if (j < T.P) {
    int g = wv;
    for (; g + 3 * W < T.G; g += 4 * W) {
      const float a = T.partial[(size_t)g * T.P + j], b = T.partial[(size_t)(g + W) * T.P + j];
      const float c = T.partial[(size_t)(g + 2 * W) * T.P + j], d = T.partial[(size_t)(g + 3 * W) * T.P + j];
      t = (((t + a) + b) + c) + d;
    }
    for (; g < T.G; g += W) t += T.partial[(size_t)g * T.P + j];
  }
  lds[wv][lane] = t;
  __syncthreads();
  if (wv != 0 || j >= T.P) return;
  t = lds[0][lane];
  for (int k = 1; k < W; ++k) t += lds[k][lane];
  float* dst = j < T.n0 ? T.d0 + j : (j < T.n0 + T.n1 ? T.d1 + (j - T.n0) : T.d2 + (j - T.n0 - T.n1));
  *dst += t;
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
}  // namespace

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

int qs_mlp_sum_partials_multi(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial,
                              float* const* d0, const int64_t* n0, float* const* d1, const int64_t* n1,
                              float* const* d2, void* stream) {
  if (n <= 0 || n > kMlpMaxTasks || !G || !P || !partial || !d0 || !n0 || !d1 || !n1 || !d2)
    return fail(QS_E_INVALID, "qs_mlp_sum_partials_multi: bad argument (1..16 tasks)");
  MlpSumTasks T{};
  T.n = n;
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (G[i] <= 0 || P[i] <= 0 || !partial[i] || !d0[i] || n0[i] <= 0 || n0[i] > P[i] || n1[i] < 0 ||
        n0[i] + n1[i] > P[i] || (n0[i] < P[i] && !d1[i]) || (n0[i] + n1[i] < P[i] && !d2[i]))
      return fail(QS_E_INVALID, "qs_mlp_sum_partials_multi: bad task");
    T.t[i] = MlpSumTask{partial[i], d0[i], d1[i], d2[i], (long long)P[i], (long long)n0[i], (long long)n1[i], (int)G[i]};
    T.start[i] = blocks;
    blocks += (int)((P[i] + 63) / 64);
  }
  T.start[n] = blocks;
  hipLaunchKernelGGL(mlp_sum_multi_kernel, dim3(blocks), dim3(kMlpSumBlock), 0, (hipStream_t)stream, T);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : fail(QS_E_HIP, std::string("qs_mlp_sum_partials_multi: ") + hipGetErrorString(e));
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

}  // extern "C"
