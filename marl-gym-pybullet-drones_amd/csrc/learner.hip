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

#include <hip/hip_runtime.h>
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

}  // extern "C"
