// rollout.hip — the per-control-step glue of the MAPPO rollout on gfx950
// (include/qs_learner.h: qs_policy_sample, qs_rollout_record).
//
// MAPPOActorCritic.step (agent.py:389-415, the batched branch; here
// mappo/agent.py MAPPOActorCritic.step) turns the actor's mean into a sampled
// action and its log-probability: Normal(mean·s, exp(logstd)).sample(), the
// action scaled by s again, and Normal.log_prob summed over the action axis
// (distributions.py:9-33).  Under torch that is ~12 elementwise launches per
// control step, then two copies into the rollout buffer; the env side (MP:
// 818-845) adds done = terminated | truncated, the mask 1 − done and the reward
// copy.  At C4's 40 960 agent rows each launch is a few microseconds of
// latency on 0.3 MB: ~60 µs of a control step.  Here each side is one launch
// writing straight into the rollout buffer's slot.  The noise ε stays
// torch.randn's (the same generator, the same draws as the torch path).
//
// Arithmetic follows torch's float32 kernels operation by operation: loc =
// mean·s, scale = exp(logstd), sample = loc + scale·ε, act = sample·s,
// log p = Σ_a [−((act − loc)²) / (2·scale²) − log(scale) − log√(2π)], the
// division correctly rounded (the library is built with fast fp32 division;
// torch's is IEEE), the sum in action order.

#include <hip/hip_runtime.h>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_rerr;
int rfail(int code, const std::string& m) { g_rerr = m; return code; }

constexpr int kRollBlock = 256;

// a / b rounded once to float: the float64 quotient of two floats, rounded to
// float, is the correctly rounded float quotient
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }

template <int A>
__global__ void __launch_bounds__(kRollBlock) policy_sample_kernel(long long K, const float* __restrict__ mean,
                                                                   const float* __restrict__ logstd, float loc_scale,
                                                                   float act_scale, int post_scale,
                                                                   const float* __restrict__ eps,
                                                                   float* __restrict__ act, float* __restrict__ logp) {
  const long long r = (long long)blockIdx.x * kRollBlock + threadIdx.x;
  if (r >= K) return;
  float lp = 0.0f;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float sc = expf(logstd[a]);
    const float loc = mean[r * A + a] * loc_scale;
    float x = loc + sc * eps[r * A + a];
    if (post_scale) x = x * act_scale;
    act[r * A + a] = x;
    const float d = x - loc;
    const float var2 = (sc * sc) * 2.0f;
    const float term = div_rn(-(d * d), var2) - logf(sc) - 0.918938533204672742f;
    lp = a == 0 ? term : lp + term;
  }
  logp[r] = lp;
}

__global__ void __launch_bounds__(kRollBlock) rollout_record_kernel(long long E, const uint8_t* __restrict__ te,
                                                                    const uint8_t* __restrict__ tr,
                                                                    const float* __restrict__ rew_src,
                                                                    float* __restrict__ rew_dst,
                                                                    float* __restrict__ mask_dst,
                                                                    float* __restrict__ done_dst) {
  const long long e = (long long)blockIdx.x * kRollBlock + threadIdx.x;
  if (e >= E) return;
  const float done = (te[e] | tr[e]) ? 1.0f : 0.0f;
  if (mask_dst) mask_dst[e] = 1.0f - done;
  if (done_dst) done_dst[e] = done;
  if (rew_dst) rew_dst[e] = rew_src[e];
}
}  // namespace

extern "C" {

const char* qs_rollout_last_error(void) { return g_rerr.c_str(); }

int qs_policy_sample(int64_t K, int32_t A, const float* mean, const float* logstd, float loc_scale, float act_scale,
                     int32_t post_scale, const float* eps, float* act, float* logp, void* stream) {
  if (K <= 0 || A < 1 || A > 4 || !mean || !logstd || !eps || !act || !logp)
    return rfail(QS_E_INVALID, "qs_policy_sample: bad argument (1 <= A <= 4)");
  if (K > (1LL << 40)) return rfail(QS_E_INVALID, "qs_policy_sample: too many rows");
  const dim3 grid((unsigned)((K + kRollBlock - 1) / kRollBlock));
  hipStream_t st = (hipStream_t)stream;
  switch (A) {
    case 1: hipLaunchKernelGGL(policy_sample_kernel<1>, grid, dim3(kRollBlock), 0, st, (long long)K, mean, logstd,
                               loc_scale, act_scale, post_scale, eps, act, logp); break;
    case 2: hipLaunchKernelGGL(policy_sample_kernel<2>, grid, dim3(kRollBlock), 0, st, (long long)K, mean, logstd,
                               loc_scale, act_scale, post_scale, eps, act, logp); break;
    case 3: hipLaunchKernelGGL(policy_sample_kernel<3>, grid, dim3(kRollBlock), 0, st, (long long)K, mean, logstd,
                               loc_scale, act_scale, post_scale, eps, act, logp); break;
    default: hipLaunchKernelGGL(policy_sample_kernel<4>, grid, dim3(kRollBlock), 0, st, (long long)K, mean, logstd,
                                loc_scale, act_scale, post_scale, eps, act, logp); break;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : rfail(QS_E_HIP, std::string("qs_policy_sample: ") + hipGetErrorString(e));
}

int qs_rollout_record(int64_t E, const uint8_t* terminated, const uint8_t* truncated, const float* rew_src,
                      float* rew_dst, float* mask_dst, float* done_dst, void* stream) {
  if (E <= 0 || !terminated || !truncated || (rew_dst && !rew_src))
    return rfail(QS_E_INVALID, "qs_rollout_record: bad argument");
  hipLaunchKernelGGL(rollout_record_kernel, dim3((unsigned)((E + kRollBlock - 1) / kRollBlock)), dim3(kRollBlock), 0,
                     (hipStream_t)stream, (long long)E, terminated, truncated, rew_src, rew_dst, mask_dst, done_dst);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : rfail(QS_E_HIP, std::string("qs_rollout_record: ") + hipGetErrorString(e));
}

}  // extern "C"
