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
 *     unless approx_kl <= 1.5*target_kl (host .item() sync)        qs_adam_step, qs_adam_multi
 *   compute_policy_loss / compute_value_loss forward and their   qs_ppo_heads
 *     autograd backward down to the actor mean and critic value
 *     (mappo/agent.py:602-683): ~60 small torch kernels
 *   MLP forward/backward (neural_networks.py:18-54) outside the   qs_mlp_bias_tanh,
 *     GEMMs: bias + tanh, the linear head, tanh backward and the   qs_mlp_tanh_bwd,
 *     bias / weight-gradient reductions (torch autograd kernels)   qs_mlp_sum_partials
 *   the same MLP at hidden 256, forward and backward fused on     qs_mlp3_fwd,
 *     MFMA (nn.Linear + torch.tanh autograd in the reference)      qs_mlp3_bwd
 *   the actor's forward, policy loss and backward of a minibatch  qs_mlp3f_actor,
 *     (agent.py:602-640, 728-734)                                  qs_value_head
 *   one PPO minibatch at the reference's learner shape            qs_ppo_small_step
 *     (agent.py:702-772 with mini_batch_size 32, learn_mappo.py:199)
 *   MeanStdNormalizer.__call__ / RunningMeanStd.update            qs_rms_update,
 *     (safe_control_gym normalization.py:13-120): torch float64      qs_rms_normalize
 *     column reductions per rollout step
 *   the critic forward + compute_value_loss head (AG:642-683)     qs_mlp3_fwd_rows_value
 *     in one launch (opt-in)
 *   MAPPOActorCritic.step sampling (agent.py:389-415,              qs_policy_sample,
 *     distributions.py:9-33) and the rollout's done / mask /        qs_rollout_record
 *     reward bookkeeping (MP:818-845): torch elementwise launches
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

/* The PPO loss heads of one minibatch (agent.py:602-683), forward and backward.
 * The minibatch is mb env-timesteps idx[mb] (int64) of the rollout buffer, all
 * D agents each: row r = i·D + d.
 *   mean[mb·D][A]   actor MLP output (before action_scale)
 *   logstd[A]       actor log standard deviation
 *   act[·][D][A], logp_old[·][D]  rollout actions and their log-probs (float)
 *   adv[·], ret[·]  per env-timestep advantages / returns (double)
 *   v[mb]           critic output on the gathered global obs
 * Losses: policy = -mean_r min(ratio·adv, clamp(ratio, 1±clip)·adv),
 * entropy = -mean_r Σ_a H(Normal), value = 0.5·mean_i (v - mean_d ret)².
 * Writes dmean = ∂L/∂mean, dlogstd = ∂L/∂logstd, dv = ∂L/∂v for
 * L = policy + ent_coef·entropy + value; kl_out[0] = approx_kl (float);
 * acc[4] (double) += {policy, value, entropy, approx_kl}.  A <= 4.
 * work: device scratch of qs_ppo_heads_work_bytes(mb, D) bytes, zeroed once
 * before the first call (the kernel leaves it ready for the next one); one
 * call at a time per workspace. */
int qs_ppo_heads(int32_t mb, int32_t D, int32_t A, const int64_t* idx, const float* mean, const float* logstd,
                 float action_scale, const float* act, const float* logp_old, const double* adv, const double* ret,
                 const float* v, float clip, float ent_coef, float* dmean, float* dlogstd, float* dv, float* kl_out,
                 double* acc, void* work, void* stream);
int64_t qs_ppo_heads_work_bytes(int32_t mb, int32_t D);

/* The elementwise / reduction side of the tanh MLP layers (actor and critic,
 * safe_control_gym neural_networks.py:18-54; autograd of nn.Linear + torch.tanh
 * in the reference) around the GEMMs.  Row-major [K][N] fp32, N = hidden size
 * in {64, 128, 256, 512}; A = head outputs (<= 4).
 *
 * qs_mlp_bias_tanh: h = tanh(z + b) (h may alias z); if A > 0 also the linear
 *   head out[K][A] = h·w3ᵀ + b3 (w3 [A][N]).
 * qs_mlp_tanh_bwd: dz = dH ⊙ (1 − h²) with dH = dh (A = 0) or dH = dout·w3
 *   (A > 0, dout [K][A]); writes dz (may alias dh) and, per block g of
 *   qs_mlp_bwd_blocks(K), the partial sums partial[g][P], P = N·(1+A) + A:
 *   [Σ dz | Σ dout_a·h (A rows of N) | Σ dout_a] over the block's rows.
 * qs_mlp_sum_partials: d += Σ_g partial[g][j] in block order (deterministic),
 *   j in [0, n0) → d0, [n0, n0+n1) → d1, the rest → d2.  Also reduces split-K
 *   weight-gradient partials [S][M] (G = S, P = M, n0 = M). */
int qs_mlp_bias_tanh(int64_t K, int32_t N, const float* z, const float* b, float* h, int32_t A, const float* w3,
                     const float* b3, float* out, void* stream);
int32_t qs_mlp_bwd_blocks(int64_t K);
int qs_mlp_tanh_bwd(int64_t K, int32_t N, const float* dh, const float* dout, int32_t A, const float* w3, const float* h,
                    float* dz, float* partial, void* stream);
int qs_mlp_sum_partials(int32_t G, int64_t P, const float* partial, float* d0, int64_t n0, float* d1, int64_t n1,
                        float* d2, void* stream);

/* n (<= 16) qs_mlp_sum_partials reductions in one launch; argument i of each
 * array describes task i exactly as the single-task call. */
int qs_mlp_sum_partials_multi(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial,
                              float* const* d0, const int64_t* n0, float* const* d1, const int64_t* n1,
                              float* const* d2, void* stream);

/* Fused tanh MLP with two hidden layers of N = 256 and a linear head of
 * A <= 4 outputs (the learner's actor and critic at the reference's
 * hidden_dim 256, learn_mappo.py:196), on the f32-input MFMA, activations
 * transposed and register-resident (learner.hip).
 * qs_mlp3_pack: W1 [N][I], W2 [N][N] → pack[qs_mlp3_pack_floats(I)], the
 *   weights in MFMA-operand order; repack after every weight update.
 * qs_mlp3_fwd: H1ᵀ = tanh(W1·Xᵀ + b1), H2ᵀ = tanh(W2·H1ᵀ + b2),
 *   out = H2·W3ᵀ + b3; X [K][I] (I <= 1024), W3 [A][N]; writes H1T, H2T
 *   [N][K] (saved for the backward; both NULL for inference) and out [K][A].
 * qs_mlp3_bwd: given dout [K][A]: dZ2ᵀ = (W3ᵀ·doutᵀ) ⊙ (1 − H2ᵀ²) and
 *   dZ1ᵀ = (W2ᵀ·dZ2ᵀ) ⊙ (1 − H1ᵀ²) [N][K], and per row block g of
 *   qs_mlp3_tiles(K, I) (32 rows when K < 16 384 or I > 64, else 128) the partial sums partA[g][N + A·N + A] =
 *   [Σ dZ2 | Σ dout_a·H2 | Σ dout_a] and partB[g][N] = Σ dZ1 over the block's
 *   rows (reduce with qs_mlp_sum_partials; the weight gradients are
 *   dW2 = dZ2ᵀ·H1, dW1 = dZ1ᵀ·X). */
int32_t qs_mlp3_tiles(int64_t K, int32_t I);
int64_t qs_mlp3_pack_floats(int32_t I);
int qs_mlp3_pack(int32_t I, int32_t N, const float* W1, const float* W2, float* pack, void* stream);
int qs_mlp3_fwd(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const float* pack, const float* b1,
                const float* b2, const float* W3, const float* b3, float* H1T, float* H2T, float* out, void* stream);
/* qs_mlp3_fwd with the minibatch gather folded in: row r of the batch is
 * X[rows[r]] (X [·][I], rows int64 [K]), and the gathered rows are written to
 * Xg [K][I] (may be NULL) for the weight gradients. */
int qs_mlp3_fwd_rows(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const int64_t* rows, float* Xg,
                     const float* pack, const float* b1, const float* b2, const float* W3, const float* b3, float* H1T,
                     float* H2T, float* out, void* stream);
/* qs_mlp3_fwd_rows with the centralized critic's value head folded in (A = 1;
 * compute_value_loss, AG:642-683, with qs_value_head's arithmetic): dv[r] =
 * (v_r − mean_d ret[rows[r]])/K and acc[1] += ½·mean over the K rows of
 * (v − mean_d ret)²; D: agents per env-timestep (the reference's mean over
 * them); work: qs_mlp3_value_work_bytes(K) bytes, zeroed once (left zero). */
int64_t qs_mlp3_value_work_bytes(int64_t K);
int qs_mlp3_fwd_rows_value(int64_t K, int32_t I, int32_t D, const float* X, const int64_t* rows, float* Xg,
                           const float* pack, const float* b1, const float* b2, const float* W3, const float* b3,
                           float* H1T, float* H2T, float* out, const double* ret, float* dv, double* acc, void* work,
                           void* stream);
/* qs_mlp3_fwd over groups of G consecutive rows: row r of the batch is
 * X[rows[r / G]·G + r % G] (K a multiple of G).  The actor's minibatch read
 * straight from the rollout table [T·E·D][O] with rows = the sampled
 * env-timesteps and G = num_agents (buffer.py:222-306's per-agent rows of the
 * sampled (t, env) pairs); no gathered copy is written. */
int qs_mlp3_fwd_group_rows(int64_t K, int32_t I, int32_t N, int32_t A, const float* X, const int64_t* rows, int32_t G,
                           const float* pack, const float* b1, const float* b2, const float* W3, const float* b3,
                           float* H1T, float* H2T, float* out, void* stream);
int qs_mlp3_bwd(int64_t K, int32_t I, int32_t N, int32_t A, const float* dout, const float* H1T, const float* H2T,
                const float* pack, const float* W3, float* dZ2T, float* dZ1T, float* partA, float* partB,
                void* stream);

/* Weight gradient of a layer over a long batch as fixed-order chunk partials
 * (the dW = dYᵀ·X of nn.Linear's backward, neural_networks.py:18-54 under
 * agent.py:702-772's loss.backward()): partial[c][n][m] = Σ_{b in chunk c}
 * AT[n][b]·B(b, m) for c < C, chunk c = rows [c·K/C, (c+1)·K/C), with
 * B(b, m) = B[b][m] (b_transposed 0: B [K][M], e.g. the layer input) or
 * BT[m][b] (b_transposed 1: a transposed activation [M][K]).  AT [N][K].
 * N % 32 == 0, K a multiple of 64·C, AT (and BT) 16-byte aligned.
 * Sum the C partials with qs_mlp_sum_partials / qs_mlp_sum_adam.
 * qs_mlp_wgrad_chunks: the C the learner uses (0: the shape is not taken). */
int32_t qs_mlp_wgrad_chunks(int64_t K, int32_t N, int32_t M);
int qs_mlp_wgrad(int64_t K, int32_t N, int32_t M, const float* AT, const float* B, int32_t b_transposed, int32_t C,
                 float* partial, void* stream);

/* The shared actor's whole minibatch step in one launch (MLPActor AG:87-148
 * forward, compute_policy_loss AG:602-640, and the backward of
 * (policy_loss + ent_coef·entropy_loss) down to every actor parameter —
 * loss.backward() at AG:733): 16-row tiles on the f32 MFMA, activations kept
 * in registers from the first layer to the last gradient (learner.hip).
 * Rows: K = mb·D agent rows, row r = agent r % D of env-timestep idx[r / D]
 * of the rollout table X [·][D][I] (I <= 128); act / logp_old / adv indexed
 * as in qs_ppo_heads; logstd, action scale, clip, ent_coef as there.
 * qs_mlp3f_pack: W1 [256][I], W2 [256][256] → pack[qs_mlp3f_pack_floats(I)]
 *   (W1f | W2f | W2b in 16x16x4 MFMA-step order); qs_adam_multi_pack /
 *   qs_mlp_sum_adam keep it current when pack_I carries QS_PACK_F16.
 * qs_mlp3f_actor writes: Xa [K][I] the gathered inputs; H1T, dZ2T, dZ1T row-major
 *   [K][256] (H1 = tanh(X·W1ᵀ + b1) and the pre-activation gradients dZ2, dZ1:
 *   dW2 = dZ2ᵀ·H1, dW1 = dZ1ᵀ·Xa); per workgroup g < qs_mlp3f_tiles(K) (128 rows) the partial
 *   rows partA[g][256 + 256·A + A] = [Σ dZ2 | Σ dout_a·H2 | Σ dout_a] and
 *   partB[g][256] = Σ dZ1; and, from the last workgroup, in workgroup order
 *   (as qs_ppo_heads): dlogstd[A], kl_out[0] = approx_kl, acc[0] += policy,
 *   acc[2] += entropy, acc[3] += approx_kl (acc[1], the value loss, is
 *   qs_value_head's).  mean_out [K][A] (may be NULL): the actor output.
 * work: qs_mlp3f_work_bytes(K) bytes, zeroed once before the first call. */
#define QS_PACK_F16 (1 << 16)
#define QS_PACK_W2T (1 << 17)   /* pack_I flag: `pack` is a [256][256] W2ᵀ copy (qs_ppo_critic_tiles) */
int32_t qs_mlp3f_tiles(int64_t K);
int64_t qs_mlp3f_pack_floats(int32_t I);
int64_t qs_mlp3f_work_bytes(int64_t K);
int qs_mlp3f_pack(int32_t I, const float* W1, const float* W2, float* pack, void* stream);
int qs_mlp3f_actor(int64_t K, int32_t I, int32_t D, int32_t A, const float* X, const int64_t* idx, const float* pack,
                   const float* b1, const float* b2, const float* W3, const float* b3, const float* logstd,
                   float action_scale, const float* act, const float* logp_old, const double* adv, float clip,
                   float ent_coef, float* Xa, float* H1T, float* dZ2T, float* dZ1T, float* partA, float* partB,
                   float* dlogstd, float* kl_out, double* acc, void* work, float* mean_out, void* stream);
/* qs_mlp3f_actor with dW1 folded in (round 5): part_w1 [qs_mlp3f_tiles(K)][256][I]
 * receives each workgroup's Σ over its 128 rows of dZ1ᵀ·X (their fixed-order sum
 * is the W1 gradient: qs_mlp_sum_adam); dZ1T may then be NULL (not stored). */
int qs_mlp3f_actor_w1(int64_t K, int32_t I, int32_t D, int32_t A, const float* X, const int64_t* idx, const float* pack,
                      const float* b1, const float* b2, const float* W3, const float* b3, const float* logstd,
                      float action_scale, const float* act, const float* logp_old, const double* adv, float clip,
                      float ent_coef, float* Xa, float* H1T, float* dZ2T, float* dZ1T, float* partA, float* partB,
                      float* dlogstd, float* kl_out, double* acc, void* work, float* mean_out, float* part_w1,
                      void* stream);

/* The value half of qs_ppo_heads (compute_value_loss AG:642-683, centralized,
 * unclipped): dv[i] = (v[i] − mean_d ret)/mb and acc[1] += 0.5·mean_i (v −
 * mean_d ret)², the same arithmetic and order.  work: qs_ppo_heads_work_bytes. */
int qs_value_head(int32_t mb, int32_t D, const int64_t* idx, const double* ret, const float* v, float* dv,
                  double* acc, void* work, void* stream);

/* qs_adam_gated followed by qs_adam_commit, in one launch: `work` is a device
 * uint32 counter, zero before the first call (the kernel leaves it zero). */
int qs_adam_step(int64_t n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* step,
                 float lr, float beta1, float beta2, float eps, const float* gate_val, float gate_thr, void* work,
                 void* stream);

/* The first layer's weight gradient dW[N][M] = Σ_b AT[N][b]·X[b][M] (AT = dZ1ᵀ
 * [N][K], X the layer input [K][M]; nn.Linear's dW = dYᵀ·X under AG:733 /
 * AG:759) as chunk partials partial[c][N][M], c < qs_mlp_wgrad_x_chunks(K, M)
 * chunks of 128 rows (0: the shape is not taken).  N = 256, M <= 256, K a
 * multiple of 128, AT 16-byte aligned; at_blocked != 0: AT is laid out
 * [K/8][N][8].  (Measured slower than split-K GEMMs at the learner's shapes:
 * opt-in)  Sum with qs_mlp_sum_partials /
 * qs_mlp_sum_adam (G = chunks, P = N·M). */
/* Split-K weight gradient of a 256-wide layer from row-major operands:
 * partial[c][N][M] = Σ_{b in chunk c} A[b][N]·B[b][M] over C chunks of K/C
 * rows (nn.Linear's dW = dYᵀ·X, AG:733 / AG:759, with A = dY [K][N] and B = X
 * [K][M] as qs_mlp3f_actor writes them).  N, M multiples of 128, K a multiple
 * of 8·C, pointers 16-byte aligned.  Sum with qs_mlp_sum_adam (G = C,
 * P = N·M).  Replaces the C batched row-chunk GEMMs of torch.bmm. */
int qs_wgrad_rm(int64_t K, int32_t N, int32_t M, const float* A, const float* B, int32_t C, float* partial,
                void* stream);

int32_t qs_mlp_wgrad_x_chunks(int64_t K, int32_t M);
int qs_mlp_wgrad_x(int64_t K, int32_t N, int32_t M, const float* AT, int32_t at_blocked, const float* X,
                   float* partial, void* stream);

/* qs_adam_step over nseg (<= 4) flat buffers in one launch (the learner's
 * actor, gated on approx_kl, and critic, AG:731-760): segment i is exactly the
 * single-buffer call with argument i of every array (host arrays of device
 * pointers / values).  work: device uint32[4], zero before the first call. */
int qs_adam_multi(int32_t nseg, float* const* params, const float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr, const float* beta1,
                  const float* beta2, const float* eps, const float* const* gate_val, const float* gate_thr, void* work,
                  void* stream);

/* qs_adam_multi with, per segment i: pack[i] (NULL = none) the qs_mlp3_pack
 * image of a 256-wide tanh MLP whose W1 [256][pack_I[i]] and W2 [256][256]
 * start at elements w1_off[i] / w2_off[i] of params[i] — every updated W1 / W2
 * element is also written to its pack positions, so the image stays current
 * without a qs_mlp3_pack launch (it must be packed once before the first call);
 * zero_grads != 0: every gradient element is set to 0 after it is read. */
int qs_adam_multi_pack(int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, float* const* step, const int64_t* n, const float* lr,
                       const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                       const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                       const int32_t* pack_I, int32_t zero_grads, void* work, void* stream);

/* One rank's minibatch step after the backward kernels: the n partial-sum
 * tasks of qs_mlp_sum_partials_multi (same arguments) and the Adam step of
 * qs_adam_multi_pack (segments params[nseg] …, pack images as there) in one
 * launch.  task_seg[i] names the segment whose gradient buffer task i's
 * destinations lie in; every gradient element the step reads must be the
 * destination of exactly one task column (a one-row task with partial = the
 * gradient itself covers an element written elsewhere, e.g. logstd's).  The
 * gradients are not written: each reduced value goes straight into Adam.
 * Equals qs_mlp_sum_partials_multi on zeroed gradients followed by
 * qs_adam_multi_pack, bit for bit.  work: qs_mlp_sum_adam_work_bytes() of
 * device memory, zero before the first call (the launch leaves it zero; one
 * work area per stream that may run the launch concurrently).  At most 2 016
 * blocks of columns (QS_E_INVALID beyond). */
int64_t qs_mlp_sum_adam_work_bytes(void);
int qs_mlp_sum_adam(int32_t n, const int32_t* G, const int64_t* P, const float* const* partial, float* const* d0,
                    const int64_t* n0, float* const* d1, const int64_t* n1, float* const* d2, const int32_t* task_seg,
                    int32_t nseg, float* const* params, float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, float* const* step, const int64_t* nel, const float* lr,
                    const float* beta1, const float* beta2, const float* eps, const float* const* gate_val,
                    const float* gate_thr, float* const* pack, const int64_t* w1_off, const int64_t* w2_off,
                    const int32_t* pack_I, void* work, void* stream);

const char* qs_learner_last_error(void);

/* The observation normaliser of the rollout (MeanStdNormalizer,
 * safe_control_gym/math_and_models/normalization.py:13-120; torch float64
 * column reductions in the reference's GPU-less loop).  x float32 [R][C]
 * (R rows = envs, C = D·O columns), statistics float64 on the device.
 * qs_rms_update: the batch's per-column mean and variance (np.mean / np.var
 * over axis 0), merged into mean[C] / var[C] / *count in place in
 * normalization.py:42-60's operation order (RunningMeanStd.update); with
 * sums != NULL nothing is updated and this rank's [Σx (C) | Σx² (C) | R] are
 * written to sums[2C + 1] instead (the multi-rank path all-reduces them).
 * work: qs_rms_work_bytes(R, C) bytes of scratch (tile moments and the saved count).
 * qs_rms_normalize: out[R][C] = float32(clip((x − mean)/sqrt(var + eps),
 * −clip, clip)) in float64 (normalization.py:110-113). */
int64_t qs_rms_work_bytes(int64_t R, int32_t C);
int qs_rms_update(int64_t R, int32_t C, const float* x, double* mean, double* var, double* count, double* sums,
                  void* work, void* stream);
int qs_rms_normalize(int64_t R, int32_t C, const float* x, const double* mean, const double* var, double eps,
                     double clip, float* out, void* stream);
const char* qs_rms_last_error(void);

/* The rollout's per-step glue (rollout.hip).  qs_policy_sample: mean [K][A]
 * (the actor MLP's output), logstd [A], eps [K][A] (standard normal draws) →
 * act [K][A] = (mean·loc_scale + exp(logstd)·eps)·(post_scale ? act_scale : 1)
 * and logp [K] = Σ_a Normal(mean·loc_scale, exp(logstd)).log_prob(act)
 * (MAPPOActorCritic.step's batched branch, agent.py:389-415; Normal,
 * distributions.py:9-33), 1 <= A <= 4.  qs_rollout_record: done =
 * terminated | truncated (uint8 [E]); mask_dst = 1 − done, done_dst = done,
 * rew_dst = rew_src (each optional, float32 [E]) — MP:818-845's buffer
 * writes. */
int qs_policy_sample(int64_t K, int32_t A, const float* mean, const float* logstd, float loc_scale, float act_scale,
                     int32_t post_scale, const float* eps, float* act, float* logp, void* stream);
int qs_rollout_record(int64_t E, const uint8_t* terminated, const uint8_t* truncated, const float* rew_src,
                      float* rew_dst, float* mask_dst, float* done_dst, void* stream);
const char* qs_rollout_last_error(void);

/* One PPO minibatch on 16-row tiles (the reference's own learner shape,
 * learn_mappo.py:196-216: mini_batch_size 32 → 256 actor rows, and each rank's
 * share of a minibatch split over G ranks) in two or three
 * launches, replacing qs_mlp3f_actor / qs_mlp3w_* / qs_value_head / the
 * weight-gradient GEMMs / qs_mlp_sum_adam there: the actor's forward, policy
 * loss head (AG:602-640) and backward and the critic's forward, value head
 * (AG:642-683) and backward in 16-row tiles, then every weight gradient
 * summed over the whole minibatch (64×64 tiles staged through LDS, K-chunks
 * summed in chunk order by a third launch) and applied by Adam in place (the actor's step gated
 * on approx_kl <= kl_thr when gate != 0, AG:731-734; the critic's always,
 * AG:757-760).  Both nets are 256-wide tanh MLPs (nn.Linear layout, row-major
 * [out][in], at most 640 inputs) inside flat parameter / Adam buffers; w2t is a
 * [256][256] transposed copy of W2, formed by the caller once and kept current
 * by the step.  obs is the rollout's obs table [T·E·D][O] (actor rows) =
 * [T·E][D·O] (critic rows), idx[mb] int64 env-timesteps; act [T·E·D][A],
 * logp_old [T·E·D], adv / ret [T·E] (float64).  Writes kl_out[0] = approx_kl
 * and acc[0..3] += policy, value, entropy loss, approx_kl, as qs_ppo_heads.
 * work: qs_ppo_small_work_bytes(mb, D, actor in, critic in, A) bytes, zeroed
 * once (the weight gradients read the transposed activations' zero padding;
 * launch 1 also stores the minibatch's Adam bias corrections there, formed
 * from the step counts before this minibatch's step commits them). */
#define QS_PPO_SMALL_MAX_ROWS 16384   /* mb·D at most */
typedef struct qs_mlp256 {
  float* params;       /* flat parameter buffer of the net (FlatBuffers)     */
  float* exp_avg;      /* Adam moments, same layout                           */
  float* exp_avg_sq;
  float* step;         /* Adam step count (float32, device)                  */
  float* w2t;          /* [256][256] = W2ᵀ                                    */
  int64_t w1, b1, w2, b2, w3, b3, logstd;   /* element offsets in params (logstd -1: none) */
  int32_t in, out;     /* input width (<= 640), outputs (actor <= 4, critic 1) */
  float lr, beta1, beta2, eps;
  float* w1p;          /* NULL, or [256][in padded to 16] = W1 with zero columns past in: the
                          step keeps it current and reads layer 1 as whole float4 quads */
} qs_mlp256;
int64_t qs_ppo_small_work_bytes(int32_t mb, int32_t D, int32_t Ia, int32_t Ic, int32_t A);
int qs_ppo_small_step(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const float* act,
                      const float* logp_old, const double* adv, const double* ret, float action_scale, float clip,
                      float ent_coef, int32_t gate, float kl_thr, const qs_mlp256* actor, const qs_mlp256* critic,
                      float* kl_out, double* acc, void* work, void* stream);
/* The multi-rank form of qs_ppo_small_step (AG:702-772 with the gradient
 * all-reduce of SURVEY §8(e)): qs_ppo_small_grads runs the same launches with
 * this rank's minibatch gradients written (not applied) into grad_a / grad_c
 * (the nets' flat gradient buffers, the params' layout: every parameter
 * element written, logstd included) and kl_out[0] = this rank's approx_kl.
 * The caller all-reduces (sum) [grad_c | grad_a | kl_out]; qs_ppo_small_adam
 * then applies Adam from the sums ÷ grad_div (the world size; the actor gated
 * on the summed approx_kl ÷ grad_div <= kl_thr when gate != 0) and keeps the
 * W2ᵀ / padded W1 copies current.  One rank (grad_div 1) gives
 * qs_ppo_small_step's bits.  work: the same workspace, as the preceding
 * qs_ppo_small_grads left it (its Adam bias corrections). */
int qs_ppo_small_grads(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const float* act,
                       const float* logp_old, const double* adv, const double* ret, float action_scale, float clip,
                       float ent_coef, const qs_mlp256* actor, const qs_mlp256* critic, float* grad_a, float* grad_c,
                       float* kl_out, double* acc, void* work, void* stream);
int qs_ppo_small_adam(int32_t mb, int32_t D, const qs_mlp256* actor, const qs_mlp256* critic, const float* grad_a,
                      const float* grad_c, float grad_div, int32_t gate, float kl_thr, const float* kl, void* work,
                      void* stream);
const char* qs_ppo_small_last_error(void);
/* The workspace's parts (off[QS_PPO_SMALL_LAYOUT_N]): off[0..15] byte offsets
 * of xaT, h1aT, dz2aT, dz1aT, xcT, h1cT, dz2cT, dz1cT (transposed [width][rows
 * padded to 64, + 16]), partAa, partBa, partAc, partBc (per-tile partial rows
 * [tile][256 + 256·A + A] = Σ dZ2 | Σ dout·H2 | Σ dout, and [tile][256] = Σ dZ1),
 * dlogstd, the loss partials, the counters; off[16..19] = actor tiles, critic
 * tiles, padded actor rows, padded critic rows; off[20] = bytes; off[21..22] =
 * the row strides of the actor's / critic's transposed buffers; off[23..26] =
 * byte offsets of the weight gradients' K-chunk partials [S][256][M padded to
 * 32] (actor W1, W2, critic W1, W2); off[27..28] = the actor's / critic's
 * K-chunks S.  Ia = 0: the critic-only layout of qs_ppo_critic_tiles.  Writes
 * min(n_off, QS_PPO_SMALL_LAYOUT_N) entries (never past the caller's array). */
#define QS_PPO_SMALL_LAYOUT_N 29
int qs_ppo_small_layout(int32_t mb, int32_t D, int32_t Ia, int32_t Ic, int32_t A, int64_t* off, int32_t n_off);
/* The critic half of qs_ppo_small_step's first launch at any minibatch size:
 * the critic's forward, value head (AG:642-683, acc[1] += value loss) and
 * backward in 16-row tiles over every CU, writing the transposed activations
 * and the per-tile partial rows of the Ia = 0 layout (no Adam step: the
 * caller forms the weight gradients with qs_wgrad_t and reduces everything
 * with qs_mlp_sum_adam).  critic->w2t must hold W2ᵀ (qs_mlp_sum_adam keeps a
 * QS_PACK_W2T segment's copy current). */
int qs_ppo_critic_tiles(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const double* ret,
                        const qs_mlp256* critic, double* acc, void* work, void* stream);
/* Split-K weight gradient from transposed operands: partial[s][n][m] =
 * Σ_{rows r of chunk s} AT[n][r]·XT[m][r] (AT [N][ld], XT [M][ld], rows r < KP in
 * S chunks of KP/S; N a multiple of 16, KP of 16·S, ld >= KP a multiple of 4).
 * nn.Linear's dW = dYᵀ·X. */
int qs_wgrad_t(int64_t KP, int64_t ld, int32_t N, int32_t M, const float* AT, const float* XT, int32_t S,
               float* partial, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QS_LEARNER_H */
