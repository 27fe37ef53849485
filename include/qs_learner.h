/*
 * qs_learner.h — C-ABI of the on-device MAPPO learner kernels (gfx950).
 *
 *   reference interface replaced                              entry point
 *   --------------------------------------------------------  ----------------
 *   compute_returns_and_advantages → _compute_single_agent_    qs_gae
 *     returns (mappo/buffer.py:428-614): numpy loops over
 *     E×D×T on the host, float64
 *   MAPPOAgent.update optimizer steps (mappo/agent.py:731-734,  qs_adam_gated +
 *     757-760): torch.optim.Adam.step, actor step skipped         qs_adam_commit
 *     unless approx_kl <= 1.5*target_kl (host .item() sync)
 *
 * All pointers are device pointers; every call is asynchronous on `stream`
 * (hipStream_t as void*) and contains no host synchronisation, so it can be
 * captured into a HIP graph.  Return 0 or a negative QS_E_* code
 * (quadswarm.h); message via qs_learner_last_error().
 */
#ifndef QS_LEARNER_H
#define QS_LEARNER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Returns / advantages for N independent sequences laid out [T][N].
 * rews, vals, masks, terminal_vals: float [T][N]; last_val: float [N].
 * Recurrence (buffer.py:586-612), accumulated in float64:
 *   r~_t = r_t + γ·tv_t ; ret_t = r~_t + γ·m_t·ret_{t+1} (ret_T = last_val)
 *   GAE:  δ_t = r~_t + γ·m_t·V_{t+1} − V_t (V_T = last_val)
 *         adv_t = δ_t + γ·λ·m_t·adv_{t+1} ;  else adv_t = ret_t − V_t
 * rets, advs: double [T][N].  vals/terminal_vals may be NULL (= zeros). */
int qs_gae(int32_t T, int64_t N, const float* rews, const float* vals, const float* masks,
           const float* terminal_vals, const float* last_val, double gamma, double gae_lambda,
           int32_t use_gae, double* rets, double* advs, void* stream);

/* torch.optim.Adam (amsgrad=False, weight_decay=0) over n float32 elements
 * of a flat parameter buffer, applied only when the gate holds:
 *   gate = (gate_val == NULL) || (*gate_val <= gate_thr)
 * `step` is the optimizer's step count (float32, device), read here as the
 * count BEFORE this step; qs_adam_commit must follow to increment it (same
 * gate).  lr, betas, eps as torch.optim.Adam. */
int qs_adam_gated(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                  const float* step, float lr, float beta1, float beta2, float eps, const float* gate_val,
                  float gate_thr, void* stream);
int qs_adam_commit(float* step, const float* gate_val, float gate_thr, void* stream);

const char* qs_learner_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* QS_LEARNER_H */
