// ppo_small.hip — one PPO minibatch on 16-row tiles, in two or three launches
// (include/qs_learner.h: qs_ppo_small_step; the multi-rank form
// qs_ppo_small_grads → all-reduce → qs_ppo_small_adam).
//
// The reference's own learner shape (learn_mappo.py:196-216 at README.md:38-39's
// 176 envs: mini_batch_size 32 env-timesteps = 256 actor rows of 27 and 32
// critic rows of 216, hidden 256, 14 080 minibatches per update) is pure
// latency, and so is every rank's share of a minibatch once SURVEY §8(e)
// partitions the global one over G ranks (C3 at G = 8: 4 096 actor rows, 512
// critic rows): the large-batch path (qs_mlp3f_actor + split-K GEMMs +
// qs_mlp_sum_adam, built for 32 768 rows) streams every weight through a few
// CUs and chains ~10 dependent launches per minibatch.  Here:
//
//  1. ppo_small_fb_kernel: one workgroup per 16-row tile (actor tiles first,
//     then critic tiles), the hidden width split over its 16 waves (wave w owns
//     hidden block w; four waves a SIMD hide each other's MFMA chains): layer 1
//     (from a copy of W1 padded to whole quads when the caller keeps one; inputs
//     up to 640 wide: Spiral's 595-wide critic), layer 2, the head (a fixed-order
//     sum of the waves' partial dots through LDS), the PPO policy / value head
//     (AG:602-683), dZ2, dH1 = dZ2·W2 and dZ1, with the activations exchanged
//     between the waves through LDS.  v_mfma_f32_16x16x4_f32: lane (g, j)
//     supplies A[j][κ] and B[κ][j] with κ = 16t + 4g + e for the four steps e of
//     quad t, so each operand is one float4 (weights row-major from L2, the
//     activations from LDS rows padded to 4 mod 32 floats: a 16-lane float4
//     read is conflict-free).  Writes the transposed activations [h][K] (the
//     weight gradients' float4 operands), per-tile bias / head partial rows,
//     and from the last tile of each net the loss sums (ppo_heads_kernel's tail).
//  2. ppo_small_wgrad_kernel: one 4-wave workgroup per 32×32 block of a weight
//     matrix and K-chunk (the chunk's quads split over the waves, each wave a
//     2×2 grid of MFMA tiles: four independent accumulator chains, four float4
//     operands per 16 MFMAs), the waves' sums added in wave order through LDS.
//     One chunk per block (S = 1, small minibatches): the gradient goes straight
//     into its sink — Adam in place (actor gated by approx_kl, AG:731-734; W2
//     also written transposed for the next minibatch's dH1, W1 into its padded
//     copy) or the gradient buffer (the multi-rank form); otherwise the chunk
//     partials.  Four more workgroups reduce the vector parameters (biases,
//     head, logstd) from the tile partials.
//  3. ppo_small_apply_kernel (S > 1 only): the chunk partials summed in chunk
//     order into the same sinks; one thread commits the step counts (launch 1
//     formed the bias corrections from them, so nothing waits for the others).
// Multi-rank: qs_ppo_small_grads runs 1–3 with the gradient
// buffers as the sink (this rank's minibatch mean); the caller all-reduces
// [critic grads | actor grads | approx_kl]; qs_ppo_small_adam is launch 3's
// Adam from those buffers (÷ the world size, the KL gate on the global mean).
// One rank forced through that path gives the fused step's bits.
//
// MFMA-bound per CU: a 16-row tile is one workgroup on one CU; the critic's
// (216 inputs) ~6 MFLOP takes ≥ ~10 µs at one CU's share of the fp32 MFMA peak
// (phase stamps: DESIGN.md §4d).

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "qs_learner.h"
#include "quadswarm.h"

namespace {
thread_local std::string g_serr;
int sfail(int code, const std::string& m) { g_serr = m; return code; }

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kSW = 16;                // waves per workgroup of the forward/backward kernel
constexpr int kSBlock = 64 * kSW;
constexpr int kSBPW = 256 / 16 / kSW;  // hidden blocks of 16 per wave (1: four waves a SIMD hide each other's chains)
constexpr int kSH = 256;               // hidden width
constexpr int kSHS = kSH + 4;          // LDS row stride of the hidden exchange (4 mod 32 floats)
constexpr int kSMaxI = 640;            // widest input (Spiral's centralized critic: 5 × 119 = 595)
constexpr int kSNarrowI = 256;         // the forward/backward instance for inputs up to this width (smaller LDS X tile)
constexpr int kSMaxA = 4;
constexpr int kSAW = 4;                // waves (16×16 tiles) per workgroup of qs_wgrad_t
constexpr int kSGW = 4;                // waves per weight-gradient workgroup (one 64×64 tile and K-chunk)
constexpr int kSCUs = 256;              // MI355X compute units (one forward/backward tile each)
constexpr int kSBlkCnt = 0;            // (no per-block arrival counters)
constexpr int kSMaxS = 32;             // most K-chunks per net
constexpr int kSPad = 16;              // floats past the padded rows in a transposed activation row
constexpr int kSScOff = 8;             // the bias corrections' slot in the dlogstd block (SWork::dlogstd)
// Dynamic LDS reserved (unused) so the dispatcher spreads the workgroups: a
// forward/backward tile uses ~53 KB (the narrow instance) and would otherwise be
// packed up to three to a CU while other CUs idle (the grids are one workgroup
// per CU or fewer); qs_wgrad_t's workgroups two to a CU, the weight-gradient
// kernel's three.
constexpr int kSReserveFB = 32 * 1024, kSReserveW = 72 * 1024;

#ifdef QS_TILE_STAMPS
// dev builds only: s_memrealtime (100 MHz) at the tile's phase boundaries,
// workgroup thread 0, [blockIdx][8] (scripts/tile_stamps.py)
constexpr int kStampWG = 4096;
__device__ unsigned long long g_tile_stamps[kStampWG * 8];
#define S_STAMP(k)                                                                                              \
  do {                                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kStampWG) g_tile_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
__device__ unsigned long long g_wg_stamps[kStampWG * 4];
#define W_STAMP(k)                                                                                          \
  do {                                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < kStampWG) g_wg_stamps[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define S_STAMP(k) \
  do {             \
  } while (0)
#define W_STAMP(k) \
  do {             \
  } while (0)
#endif

__host__ __device__ constexpr int s_ip(int I) { return (I + 15) & ~15; }       // input padded to whole quads
__host__ __device__ constexpr int s_xs(int I) { return ((I + 31) & ~31) + 4; } // LDS row stride of the X tile

struct SNet {   // one 256-wide tanh MLP inside its flat Adam buffers (qs_mlp256)
  float* p;
  float* m;
  float* v;
  float* step;
  float* w2t;
  long long w1, b1, w2, b2, w3, b3, logstd;
  int I, A;
  float lr, beta1, beta2, eps;
  float* w1p;   // NULL or W1 padded to s_ip(I) columns (zeros past I), kept current by the Adam launch
};

struct SWork {   // workspace views (qs_ppo_small_work_bytes)
  float *xaT, *h1aT, *dz2aT, *dz1aT, *xcT, *h1cT, *dz2cT, *dz1cT;
  float *partAa, *partBa, *partAc, *partBc;
  float* dlogstd;   // [0, kSMaxA) d logstd, [kSMaxA] the entropy, [kSScOff, +4) Adam's bias corrections
                    // (actor bc1, sqrt bc2, critic bc1, sqrt bc2) for this minibatch's step
  double *lossa, *lossc;
  unsigned* cnt;   // [0] actor tiles, [64] critic tiles (qs_ppo_critic_tiles' last-tile sums)
  float* wpart[4];   // K-chunk partials [S][256][Mp] of actor W1, actor W2, critic W1, critic W2 (Mp: M padded to 32)
};

// Where the reduced gradients go (launches 2 and 3)
enum { SINK_PART = 0, SINK_ADAM = 1, SINK_GRAD = 2 };
struct SGrad {
  int S[2];          // K-chunks per net (actor, critic)
  int spc[2];        // 64-row steps per K-chunk
  int sink;          // the final sink: SINK_ADAM (one rank) or SINK_GRAD (this rank's gradient, for the all-reduce)
  float* g[2];       // SINK_GRAD / qs_ppo_small_adam: the nets' gradient buffers (flat, the params' layout)
  float gdiv;        // qs_ppo_small_adam: the all-reduced sums ÷ gdiv (the world size), approx_kl too
};

struct SArgs {
  int mb, D, nA, nC, KaP, KcP;
  int rb, rbc;             // 16-row blocks per forward/backward tile: the actor's, the critic's
  int KaS, KcS;            // row strides of the transposed activations (KaP / KcP + kSPad)
  const float* X;          // the rollout's obs table [T·E·D][O] (critic rows: [T·E][D·O])
  const long long* idx;    // the minibatch's env-timesteps [mb]
  const float* act;        // [T·E·D][A]
  const float* logp_old;   // [T·E·D]
  const double* adv;       // [T·E]
  const double* ret;       // [T·E]
  float scale, clip, ent_coef, kl_thr;
  int gate;
  int fb_tail;             // 1: the forward/backward launch's last tile of each net sums the loss rows
                           // (qs_ppo_critic_tiles); 0: launch 2 does (no release fence per tile)
  float* kl_out;
  double* acc;
  SNet a, c;
  SWork w;
  SGrad G;
};

__device__ __forceinline__ float s_tanh(float x) {   // learner.hip's m3_tanh
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}
__device__ __forceinline__ f32x4 s_mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int CTRL>
__device__ __forceinline__ float s_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Σ over the 16 lanes of a DPP row (every lane gets a sum; lane 0's order is fixed)
__device__ __forceinline__ float s_row_sum(float t) {
  t += s_dpp<0x128>(t);   // row_ror:8
  t += s_dpp<0x124>(t);   // row_ror:4
  t += s_dpp<0x4E>(t);    // quad_perm [2,3,0,1]
  return t + s_dpp<0xB1>(t);   // quad_perm [1,0,3,2]
}

__device__ __forceinline__ double s_powi(double b, unsigned t) {
  double r = 1.0;
  while (t) {
    if (t & 1u) r *= b;
    b *= b;
    t >>= 1;
  }
  return r;
}

// Branch-free operand loads: the index is clamped into the row and the value
// selected, so every load is issued unconditionally (conditional loads made the
// compiler wait for all outstanding loads before each use: one L2 round trip
// per quad, 6x the MFMA time)
__device__ __forceinline__ float4 s_ld4s(const float* row, int k0, int I) {   // scalar (any I)
  float4 r;
  r.x = row[min(k0, I - 1)];
  r.y = row[min(k0 + 1, I - 1)];
  r.z = row[min(k0 + 2, I - 1)];
  r.w = row[min(k0 + 3, I - 1)];
  if (k0 >= I) r.x = 0.f;
  if (k0 + 1 >= I) r.y = 0.f;
  if (k0 + 2 >= I) r.z = 0.f;
  if (k0 + 3 >= I) r.w = 0.f;
  return r;
}

// A wave's weight-row stream for one contraction: c += Σ over NQ quads of
// A[j][κ]·B[κ][j] (κ = 16t + 4g + e) for the wave's hidden block, the A row
// from L2 (VEC: whole float4s of a 256-wide row; otherwise scalars, elements
// past I zero, branch-free), the B row (an activation row) from LDS.  The first
// kSRing quads are loaded by s_prefill — issued phases ahead of the contraction,
// so their latency hides behind earlier work — and s_run keeps kSRing quads in
// flight (compile-time NQ: the loop unrolls fully and the load counter waits
// are exact; the scheduling barrier keeps the loads ahead of the MFMAs).  The
// even and odd quads go to two accumulators (independent MFMA chains).
constexpr int kSRing = 8;
template <bool VEC>
__device__ __forceinline__ float4 s_ldq(const float* row, int t, int I, int g) {
  if constexpr (VEC) return *reinterpret_cast<const float4*>(row + 16 * t + 4 * g);
  else return s_ld4s(row, 16 * t + 4 * g, I);
}
template <int NQ, bool VEC>
__device__ __forceinline__ void s_prefill(float4 (&ra)[kSRing], const float* wrow, int I, int g) {
#pragma unroll
  for (int t = 0; t < (NQ < kSRing ? NQ : kSRing); ++t) ra[t] = s_ldq<VEC>(wrow, t, I, g);
}
// RB row blocks of 16 share each weight quad: z[rb] += its contraction with
// the activation row brow + rb·bs (LDS).  RB = 1: the even and odd quads on two
// accumulator chains; RB > 1: the row blocks are the independent chains.
template <int NQ, bool VEC, int RB>
__device__ __forceinline__ void s_run(float4 (&ra)[kSRing], const float* wrow, int I, const float* brow, int bs, int g,
                                      f32x4 (&z)[RB]) {
  f32x4 c1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NQ; ++t) {
    const float4 a = ra[t % kSRing];
    if (t + kSRing < NQ) ra[t % kSRing] = s_ldq<VEC>(wrow, t + kSRing, I, g);
    float4 bv[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) bv[rb] = *reinterpret_cast<const float4*>(brow + rb * bs + 16 * t + 4 * g);
    __builtin_amdgcn_sched_barrier(0);   // the scheduler would sink the loads next to their use
    if constexpr (RB == 1) {
      f32x4& acc = (t & 1) ? c1 : z[0];
      acc = s_mfma(a.x, bv[0].x, acc);
      acc = s_mfma(a.y, bv[0].y, acc);
      acc = s_mfma(a.z, bv[0].z, acc);
      acc = s_mfma(a.w, bv[0].w, acc);
    } else {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) z[rb] = s_mfma(a.x, bv[rb].x, z[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) z[rb] = s_mfma(a.y, bv[rb].y, z[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) z[rb] = s_mfma(a.z, bv[rb].z, z[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) z[rb] = s_mfma(a.w, bv[rb].w, z[rb]);
    }
  }
  if constexpr (RB == 1) z[0] += c1;
}
// layer 1 over nq = ⌈I/16⌉ quads (1..16): the compile-time count by dispatch
#define S_NQ_SWITCH(nq, CALL)                                                                       \
  switch (nq) {                                                                                     \
    case 1: CALL(1); break; case 2: CALL(2); break; case 3: CALL(3); break; case 4: CALL(4); break; \
    case 5: CALL(5); break; case 6: CALL(6); break; case 7: CALL(7); break; case 8: CALL(8); break; \
    case 9: CALL(9); break; case 10: CALL(10); break; case 11: CALL(11); break;                   \
    case 12: CALL(12); break; case 13: CALL(13); break; case 14: CALL(14); break;                 \
    case 15: CALL(15); break; default: CALL(16); break;                                             \
  }

// Layer 1 over nq = ⌈I/16⌉ quads: the ring was prefilled with the first quads
// phases ahead (s_prefill<min(nq, 16)>); up to 16 quads by one compile-time run,
// wider inputs (WIDE: up to kSMaxI) in 16-quad blocks that refill the ring at
// their start, then the remainder
template <bool VEC, bool WIDE, int RB>
__device__ __forceinline__ void s_layer1(float4 (&ring)[kSRing], const float* wrow, int I, const float* brow, int bs,
                                         int g, int nq, f32x4 (&z)[RB]) {
#define S_RUNL(n) s_run<n, VEC, RB>(ring, wrow, I, brow, bs, g, z)
  if (!WIDE || nq <= 16) {
    S_NQ_SWITCH(nq, S_RUNL)
    return;
  }
#undef S_RUNL
  if constexpr (WIDE) {
    s_run<16, VEC, RB>(ring, wrow, I, brow, bs, g, z);
    int t = 16;
    for (; t + 16 <= nq; t += 16) {
      s_prefill<16, VEC>(ring, wrow + 16 * t, I - 16 * t, g);
      s_run<16, VEC, RB>(ring, wrow + 16 * t, I - 16 * t, brow + 16 * t, bs, g, z);
    }
    if (t < nq) {
      const float* wr = wrow + 16 * t;
      const float* br = brow + 16 * t;
      const int Ir = I - 16 * t;
#define S_REM(n)                                    \
  {                                                 \
    s_prefill<n, VEC>(ring, wr, Ir, g);             \
    s_run<n, VEC, RB>(ring, wr, Ir, br, bs, g, z);  \
  }
      S_NQ_SWITCH(nq - t, S_REM)
#undef S_REM
    }
  }
}

// c += Σ over NQ quads of A[j][rows]·B[rows][j], both operands transposed rows
// in global memory, kSRing quads of loads ahead; compile-time NQ
template <int NQ>
__device__ __forceinline__ void s_wgrad_acc_n(const float* arow, const float* brow, int g, f32x4& c) {
  constexpr int R = NQ < kSRing ? NQ : kSRing;
  float4 ra[R], rb[R];
#pragma unroll
  for (int t = 0; t < R; ++t) {
    ra[t] = *reinterpret_cast<const float4*>(arow + 16 * t + 4 * g);
    rb[t] = *reinterpret_cast<const float4*>(brow + 16 * t + 4 * g);
  }
#pragma unroll
  for (int t = 0; t < NQ; ++t) {
    const float4 av = ra[t % R], bv = rb[t % R];
    if (t + R < NQ) {
      ra[t % R] = *reinterpret_cast<const float4*>(arow + 16 * (t + R) + 4 * g);
      rb[t % R] = *reinterpret_cast<const float4*>(brow + 16 * (t + R) + 4 * g);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the loads R quads ahead
    c = s_mfma(av.x, bv.x, c);
    c = s_mfma(av.y, bv.y, c);
    c = s_mfma(av.z, bv.z, c);
    c = s_mfma(av.w, bv.w, c);
  }
}
// any nq: whole blocks of 16 quads, then the remainder by dispatch
__device__ __forceinline__ void s_wgrad_acc(const float* arow, const float* brow, int nq, int g, f32x4& c) {
  int t = 0;
  for (; t + 16 <= nq; t += 16) s_wgrad_acc_n<16>(arow + 16 * t, brow + 16 * t, g, c);
  switch (nq - t) {
#define S_CASE(n) case n: s_wgrad_acc_n<n>(arow + 16 * t, brow + 16 * t, g, c); break;
    S_CASE(1) S_CASE(2) S_CASE(3) S_CASE(4) S_CASE(5) S_CASE(6) S_CASE(7) S_CASE(8)
    S_CASE(9) S_CASE(10) S_CASE(11) S_CASE(12) S_CASE(13) S_CASE(14) S_CASE(15)
#undef S_CASE
    default: break;
  }
}

// ---------------------------------------------------------------- launch 1
// One tile of 16·RB rows of one net: POL = the actor (policy head over A
// outputs), otherwise the critic (value head).  Lane (g, j) of wave w holds
// hidden units 16w + 4g .. + 3 of rows r0 + 16·rb + j, rb < RB: each weight quad
// streamed from L2 feeds RB MFMA groups (RB = 2 once a launch has more tiles
// than CUs).  xs (the X tile) and dz2s share LDS: xs is dead after layer 1.
template <int A, bool POL, bool V1, int MAXI, int RB>
__device__ __forceinline__ void s_tile(const SArgs& P, const SNet& N, int tile, float* xs, float* h1s, float* dz2s,
                                       float* prm, float (*hp)[16 * RB], double (*ls_w)[2 + kSMaxA]) {
  static_assert(kSBPW == 1, "one hidden block per wave");
  constexpr int NL = POL ? 2 + A : 1;   // loss sums: policy, approx_kl, d logstd[A] | value
  constexpr int TR = 16 * RB;           // rows of the tile
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, j = l & 15, g = l >> 4;
  const int I = N.I, XS = s_xs(I), Ip = s_ip(I), nq1 = Ip / 16;
  const int K = POL ? P.mb * P.D : P.mb;
  const int KP = POL ? P.KaS : P.KcS;   // the transposed rows' stride
  const int r0 = tile * TR;
  const SWork& W = P.w;
  float* xT = POL ? W.xaT : W.xcT;
  float* h1T = POL ? W.h1aT : W.h1cT;
  float* dz2T = POL ? W.dz2aT : W.dz2cT;
  float* dz1T = POL ? W.dz1aT : W.dz1cT;
  const int b0 = w, h0 = 16 * b0 + 4 * g;   // the wave's hidden block; lane (g, j): units h0 .. h0 + 3
  // layer 1's rows: the padded copy as whole float4 quads when there is one,
  // otherwise the parameter rows with clamped scalar loads
  // (V1: the launch checked that the net has the copy)
  const float* w1row = V1 ? N.w1p + (size_t)(16 * b0 + j) * Ip : N.p + N.w1 + (size_t)(16 * b0 + j) * I;
  const float* w2row = N.p + N.w2 + (size_t)(16 * b0 + j) * kSH;
  const float* w2trow = N.w2t + (size_t)(16 * b0 + j) * kSH;
  // ---- every independent load first, so the tile pays one or two memory
  // round trips before its first MFMA instead of one per phase: the first
  // quads of both forward contractions' weight rows, the head's per-row inputs,
  // the X tile (gathered through idx), and the biases / head into LDS
  S_STAMP(0);
  float4 ring1[kSRing], ring2[kSRing];
#define S_PRE1(n) s_prefill<n, false>(ring1, w1row, I, g)
#define S_PRE1V(n) s_prefill<n, true>(ring1, w1row, Ip, g)
  if constexpr (V1) {
    S_NQ_SWITCH(nq1, S_PRE1V)
  } else {
    S_NQ_SWITCH(nq1, S_PRE1)
  }
#undef S_PRE1
#undef S_PRE1V
  // (the wide and the two-block instances fill layer 2's ring after layer 1:
  // both rings live across it would not fit in the 128 registers of a 16-wave workgroup)
  constexpr bool kEarly2 = MAXI <= kSNarrowI && RB == 1;
  if constexpr (kEarly2) s_prefill<16, true>(ring2, w2row, kSH, g);
  bool rv[RB];
  float hact[RB][A], hlpo[RB];
  double had[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int R = r0 + 16 * rb + j;
    rv[rb] = R < K;
    hlpo[rb] = 0.f;
    had[rb] = 0.0;
    if constexpr (POL) {
      const long long ei = rv[rb] ? R / P.D : 0;
      const long long e_idx = rv[rb] ? P.idx[ei] : 0;
      const long long gi = e_idx * P.D + (R - ei * P.D);
#pragma unroll
      for (int a = 0; a < A; ++a) hact[rb][a] = rv[rb] ? P.act[gi * A + a] : 0.f;
      if (rv[rb]) {
        hlpo[rb] = P.logp_old[gi];
        had[rb] = P.adv[e_idx];
      }
    } else {
#pragma unroll
      for (int a = 0; a < A; ++a) hact[rb][a] = 0.f;
      if (rv[rb]) had[rb] = P.ret[P.idx[R]];   // the value head's return
    }
  }
  {
    constexpr int kXU = (16 * MAXI + kSBlock - 1) / kSBlock;
    float v[RB][kXU];
    const int rr = tid & 15;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int Rx = r0 + 16 * rb + rr;
      const long long src = Rx < K ? (POL ? (P.idx[Rx / P.D] * P.D + Rx % P.D) : P.idx[Rx]) * I : -1;
#pragma unroll
      for (int u = 0; u < kXU; ++u) {
        const int k = (tid >> 4) + u * (kSBlock / 16);
        v[rb][u] = src >= 0 && k < I ? P.X[src + k] : 0.f;
      }
    }
    // biases and head: prm = [b1 | b2 | W3 (A rows) | b3 | logstd]
    for (int e = tid; e < 2 * kSH + A * kSH + 2 * A; e += kSBlock) {
      float pv;
      if (e < kSH) pv = N.p[N.b1 + e];
      else if (e < 2 * kSH) pv = N.p[N.b2 + e - kSH];
      else if (e < 2 * kSH + A * kSH) pv = N.p[N.w3 + e - 2 * kSH];
      else if (e < 2 * kSH + A * kSH + A) pv = N.p[N.b3 + e - 2 * kSH - A * kSH];
      else pv = POL ? N.p[N.logstd + e - 2 * kSH - A * kSH - A] : 0.f;
      prm[e] = pv;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int Rx = r0 + 16 * rb + rr;
#pragma unroll
      for (int u = 0; u < kXU; ++u) {
        const int k = (tid >> 4) + u * (kSBlock / 16);
        if (k < Ip) xs[(16 * rb + rr) * XS + k] = v[rb][u];
        if (k < I) xT[(size_t)k * KP + Rx] = v[rb][u];
      }
    }
  }
  __syncthreads();
  S_STAMP(1);
  const float* sb1 = prm;
  const float* sb2 = prm + kSH;
  const float* sw3 = prm + 2 * kSH;
  const float* sb3 = prm + 2 * kSH + A * kSH;
  const float* slogstd = sb3 + A;
  if (POL && tile == 0 && tid == 0 && !P.fb_tail) {
    // the policy's entropy from this minibatch's logstd, for launch 2's statistics
    // (launch 2 updates logstd in place; dlogstd[kSMaxA] keeps the value it reports)
    const float lc = (float)log(sqrt(2.0 * M_PI));
    float ent = 0.0f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float lsd = logf(expf(slogstd[a]));
      ent = a == 0 ? (0.5f + lc) + lsd : ent + ((0.5f + lc) + lsd);
    }
    W.dlogstd[kSMaxA] = ent;
  }
  // ---- layer 1: Z1ᵀ[h0 + r][row] in register r of lane (g, j)
  f32x4 z[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) z[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  s_layer1<V1, (MAXI > kSNarrowI), RB>(ring1, w1row, V1 ? Ip : I, xs + j * XS, 16 * XS, g, nq1, z);
#ifdef QS_TILE_STAMPS2
  S_STAMP(6);   // (dev: layer 1's MFMAs issued)
#endif
  if constexpr (!kEarly2) s_prefill<16, true>(ring2, w2row, kSH, g);
  float h1[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) h1[rb][r] = s_tanh(z[rb][r] + sb1[h0 + r]);
    *reinterpret_cast<float4*>(h1s + (16 * rb + j) * kSHS + h0) = float4{h1[rb][0], h1[rb][1], h1[rb][2], h1[rb][3]};
  }
#ifdef QS_TILE_STAMPS2
  S_STAMP(7);   // (dev: H1 formed and stored)
#endif
  __syncthreads();
  S_STAMP(2);
  // ---- layer 2: Z2ᵀ = W2·H1ᵀ (its ring filled at the start); the backward's ring filled behind it
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) z[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  s_run<16, true, RB>(ring2, w2row, kSH, h1s + j * kSHS, 16 * kSHS, g, z);
  s_prefill<16, true>(ring1, w2trow, kSH, g);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) h1T[(size_t)(h0 + r) * KP + r0 + 16 * rb + j] = h1[rb][r];   // (after the loads above)
  float h2[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    float hs[A];
#pragma unroll
    for (int a = 0; a < A; ++a) hs[a] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      h2[rb][r] = s_tanh(z[rb][r] + sb2[h0 + r]);
#pragma unroll
      for (int a = 0; a < A; ++a) hs[a] += h2[rb][r] * sw3[a * kSH + h0 + r];
    }
    // the head: the wave's partial dot of the row (lane groups g added), then the waves in order
#pragma unroll
    for (int a = 0; a < A; ++a) {
      float t = hs[a] + __shfl_xor(hs[a], 16, 64);
      t = t + __shfl_xor(t, 32, 64);
      if (g == 0) hp[w * A + a][16 * rb + j] = t;
    }
  }
  __syncthreads();
  S_STAMP(3);
  // ---- per row block: the loss head of the row (every wave forms it; wave 0,
  // lane group 0 records its loss terms), dZ2 = (dout·W3) ⊙ (1 − H2²) and the
  // tile's b2 / W3 / b3 partial rows (row sums over j, the row blocks in order)
  float* pa = (POL ? W.partAa : W.partAc) + (size_t)tile * (kSH + A * kSH + A);
  float* pb = (POL ? W.partBa : W.partBc) + (size_t)tile * kSH;
  float d4[RB][4], sbp[4], swp[A][4], sdo[A];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    float mu[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      float t = hp[a][16 * rb + j];
#pragma unroll
      for (int v = 1; v < kSW; ++v) t += hp[v * A + a][16 * rb + j];
      mu[a] = t + sb3[a];
    }
    float dout[A];
    double ls[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) ls[k] = 0.0;
    if constexpr (POL) {
      // compute_policy_loss (AG:602-640) and its gradient: ppo_heads_kernel's arithmetic
      float sd[A], lsd[A], var2[A];
#pragma unroll
      for (int a = 0; a < A; ++a) {
        sd[a] = expf(slogstd[a]);
        lsd[a] = logf(sd[a]);
        var2[a] = 2.0f * (sd[a] * sd[a]);
      }
      const float lc = (float)log(sqrt(2.0 * M_PI));
      const float lo = 1.0f - P.clip, hi = 1.0f + P.clip;
      const double G = -1.0 / (double)K;
      float t1[A], logp = 0.0f;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const float m = mu[a] * P.scale;
        t1[a] = hact[rb][a] - m;
        const float t4 = (float)((double)(-(t1[a] * t1[a])) / (double)var2[a]);
        const float lp = (t4 - lsd[a]) - lc;
        logp = a == 0 ? lp : logp + lp;
      }
      const float lpo = hlpo[rb];
      const float ratio = expf(logp - lpo);
      const double ad = had[rb];
      const float rc = fminf(fmaxf(ratio, lo), hi);
      const double s1 = (double)ratio * ad, s2 = (double)rc * ad;
      const double g1 = s1 < s2 ? G : (s1 == s2 ? G / 2 : 0.0);
      const double g2 = s2 < s1 ? G : (s1 == s2 ? G / 2 : 0.0);
      float gr = (float)(g1 * ad);
      if (ratio >= lo && ratio <= hi) gr = gr + (float)(g2 * ad);
      const float gl = gr * ratio;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const float gt3 = (float)((double)gl / (double)var2[a]);
        const float gt1 = -gt3 * 2.0f * t1[a];
        dout[a] = rv[rb] ? -gt1 * P.scale : 0.f;
        if (rv[rb]) ls[2 + a] = (double)gl * ((double)(t1[a] * t1[a]) / ((double)sd[a] * sd[a]) - 1.0);
      }
      if (rv[rb]) {
        ls[0] = -(s1 < s2 ? s1 : s2);
        ls[1] = (double)(lpo - logp);
      }
    } else {
      // compute_value_loss (AG:642-683, centralized, unclipped): qs_value_head's arithmetic
      if (rv[rb]) {
        const double rt = had[rb];
        double rs = 0;
        for (int d = 0; d < P.D; ++d) rs += rt;
        const double diff = (double)mu[0] - rs / (double)P.D;
        ls[0] = diff * diff;
        dout[0] = (float)(diff / (double)P.mb);
      } else {
        dout[0] = 0.f;
      }
    }
    if (w == 0 && g == 0)
#pragma unroll
      for (int k = 0; k < NL; ++k) ls_w[16 * rb + j][k] = ls[k];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = h0 + r;
      float gg = 0.f;
#pragma unroll
      for (int a = 0; a < A; ++a) gg += dout[a] * sw3[a * kSH + h];
      const float hv = h2[rb][r];
      d4[rb][r] = gg * (1.f - hv * hv);
      const float sb = s_row_sum(d4[rb][r]);
      sbp[r] = rb == 0 ? sb : sbp[r] + sb;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const float sw = s_row_sum(dout[a] * hv);
        swp[a][r] = rb == 0 ? sw : swp[a][r] + sw;
      }
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float t = s_row_sum(dout[a]);
      sdo[a] = rb == 0 ? t : sdo[a] + t;
    }
  }
  if (j == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[h0 + r] = sbp[r];
#pragma unroll
      for (int a = 0; a < A; ++a) pa[kSH + a * kSH + h0 + r] = swp[a][r];
    }
  if (w == 0 && l == 0)
#pragma unroll
    for (int a = 0; a < A; ++a) pa[kSH + A * kSH + a] = sdo[a];
  // (dz2s aliases xs: every wave's layer-1 reads of it precede two barriers)
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
    *reinterpret_cast<float4*>(dz2s + (16 * rb + j) * kSHS + h0) = float4{d4[rb][0], d4[rb][1], d4[rb][2], d4[rb][3]};
  S_STAMP(4);
  __syncthreads();
  // ---- dH1ᵀ = W2ᵀ·dZ2ᵀ (rows of the transposed copy; ring filled during the head), dZ1 = dH1 ⊙ (1 − H1²)
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) z[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  s_run<16, true, RB>(ring1, w2trow, kSH, dz2s + j * kSHS, 16 * kSHS, g, z);
  float sbq[4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int R = r0 + 16 * rb + j;
#pragma unroll
    for (int r = 0; r < 4; ++r) dz2T[(size_t)(h0 + r) * KP + R] = d4[rb][r];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float u = h1[rb][r];
      const float d = z[rb][r] * (1.f - u * u);
      dz1T[(size_t)(h0 + r) * KP + R] = d;
      const float sb = s_row_sum(d);
      sbq[r] = rb == 0 ? sb : sbq[r] + sb;
    }
  }
  if (j == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) pb[h0 + r] = sbq[r];
  __syncthreads();   // (ls_w)
  S_STAMP(5);
  // ---- the tile's loss sums (rows in order), then (fb_tail) the net's last tile
  __shared__ bool last;
  if (tid == 0) {
    double* lp = POL ? W.lossa + (size_t)tile * NL : W.lossc + tile;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      double sacc = 0.0;
      for (int q = 0; q < TR; ++q) sacc += ls_w[q][k];
      lp[k] = sacc;
    }
    if (P.fb_tail) {
      // (an agent-scope release per tile: hundreds of tiles' L2 write-backs
      // serialise — 9 µs a tile at 288 tiles — so launch 2 sums the rows instead)
      __threadfence();
      const int ntiles = POL ? P.nA : P.nC;
      last = atomicAdd(W.cnt + (POL ? 0 : 64), 1u) == (unsigned)ntiles - 1;
    }
  }
  if (!P.fb_tail) return;
  __syncthreads();
  S_STAMP(6);
  if (!last || w != 0) return;
  // the net's last tile: wave 0 sums the tiles' loss rows (lane q: tiles q, q + 64, ...
  // in order), then a fixed xor butterfly over the lanes (every lane ends with the
  // same bits: each level adds the same two operands)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int ntiles = POL ? P.nA : P.nC;
  double tot[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) tot[k] = 0.0;
  for (int t = l; t < ntiles; t += 64)
#pragma unroll
    for (int k = 0; k < NL; ++k) tot[k] += (POL ? W.lossa[(size_t)t * NL + k] : W.lossc[t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < NL; ++k) tot[k] += __shfl_xor(tot[k], o, 64);
  if (l != 0) return;
  S_STAMP(7);
  W.cnt[POL ? 0 : 64] = 0u;
  if constexpr (!POL) {
    P.acc[1] += 0.5 * (tot[0] / (double)P.mb);
  } else {
    const float lc = (float)log(sqrt(2.0 * M_PI));
    float ent = 0.0f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const float lsd = logf(expf(slogstd[a]));
      ent = a == 0 ? (0.5f + lc) + lsd : ent + ((0.5f + lc) + lsd);
    }
#pragma unroll
    for (int a = 0; a < A; ++a) W.dlogstd[a] = (float)tot[2 + a] - P.ent_coef;
    const float akl = (float)(tot[1] / (double)K);
    *P.kl_out = akl;
    P.acc[0] += tot[0] / (double)K;
    P.acc[2] += (double)(-ent);
    P.acc[3] += (double)akl;
  }
}

// RB: the actor's row blocks per tile; RBC: the critic's (its tiles are the
// launch's slowest — 216 inputs staged and contracted — so they stay at 16 rows
// while the actor's grow, when the CUs hold both)
// MAXA: the actor's input bound (a narrow actor beside a wide critic: its
// 48-row X tile sized for its own width)
// Adam's bias corrections of a net for its next step (float32 of the float64
// powers, as learner.hip): bc1 = 1 − β1^t, sqrt(bc2) = sqrt(1 − β2^t), t = step + 1
__device__ __forceinline__ void s_bias_corr(const SNet& N, float* out) {
  const unsigned t = (unsigned)(*N.step) + 1u;
  out[0] = (float)(1.0 - s_powi((double)N.beta1, t));
  out[1] = (float)sqrt(1.0 - s_powi((double)N.beta2, t));
}

template <int A, bool V1, int MAXI, int RB, int RBC = RB, int MAXA = MAXI>
__global__ void __launch_bounds__(kSBlock) ppo_small_fb_kernel(SArgs P) {
  // The minibatch's bias corrections, from the step counts before any launch of
  // it changes them: the Adam launches read these, so the one thread that
  // commits a step count there needs no arrival count of the other workgroups
  // (a 700-workgroup fan-in on one counter cost ~9 µs)
  if (!P.fb_tail && blockIdx.x == 0 && threadIdx.x == 0) {
    s_bias_corr(P.a, P.w.dlogstd + kSScOff);
    s_bias_corr(P.c, P.w.dlogstd + kSScOff + 2);
  }
  constexpr int RM = RB > RBC ? RB : RBC;
  constexpr int XA = 16 * RB * s_xs(MAXA), XC = 16 * RBC * s_xs(MAXI);
  constexpr int XSZ = XA > XC ? XA : XC, DSZ = 16 * RM * kSHS;
  __shared__ float xsd[XSZ > DSZ ? XSZ : DSZ];   // the X tile, then dZ2 (dead / not yet live in turn)
  __shared__ float h1s[16 * RM * kSHS];
  __shared__ float hp[kSW * kSMaxA][16 * RM];
  __shared__ double ls_w[16 * RM][2 + kSMaxA];
  __shared__ float prm[2 * kSH + kSMaxA * kSH + 2 * kSMaxA];
  if ((int)blockIdx.x < P.nA)
    s_tile<A, true, V1, MAXA, RB>(P, P.a, blockIdx.x, xsd, h1s, xsd, prm, reinterpret_cast<float (*)[16 * RB]>(hp),
                                  ls_w);
  else
    s_tile<1, false, V1, MAXI, RBC>(P, P.c, blockIdx.x - P.nA, xsd, h1s, xsd, prm,
                                    reinterpret_cast<float (*)[16 * RBC]>(hp), ls_w);
}

// ---------------------------------------------------------------- launches 2 and 3
// p / m / v of element i loaded by the caller ahead of the gradient (their
// latency hides behind the gradient's loads)
// torch.optim.Adam's element update (amsgrad=False, weight_decay=0: learner.hip's
// adam_elem) as values: p1, m1, v1 from gradient g and p, m, v
__device__ __forceinline__ void s_adam_v(const SNet& N, float g, float bc1, float bc2s, float p, float m, float v,
                                         float& p1, float& m1, float& v1) {
  m1 = m + (1.0f - N.beta1) * (g - m);
  v1 = v * N.beta2 + (1.0f - N.beta2) * g * g;
  const float denom = sqrtf(v1) / bc2s + N.eps;
  p1 = p - (N.lr / bc1) * (m1 / denom);
}
__device__ __forceinline__ void s_adam(const SNet& N, long long i, float g, float bc1, float bc2s, float* w2t,
                                       int n, int k, float* w1p, float p, float m, float v) {
  float p1, m1, v1;
  s_adam_v(N, g, bc1, bc2s, p, m, v, p1, m1, v1);
  N.m[i] = m1;
  N.v[i] = v1;
  N.p[i] = p1;
#ifdef QS_X_NO_W2T
  w2t = nullptr;   // dev probe: the transposed copy's scattered stores skipped (results wrong)
#endif
  if (w2t) w2t[(size_t)k * kSH + n] = p1;
  if (w1p) w1p[(size_t)n * s_ip(N.I) + k] = p1;
}

// Σ over a net's tile loss rows (rows [nt][NL], NL <= 2 + kSMaxA) in a fixed
// order, by one whole wave: lane q takes tiles q, q + 64, ... in order, then an
// xor butterfly (every lane ends with the same bits: each level adds the same
// two operands) — the fb tiles' tail arithmetic, so every workgroup that needs
// the totals forms identical ones
__device__ __forceinline__ void s_loss_tot(const double* rows, int nt, int NL, int l, double (&tot)[2 + kSMaxA]) {
#pragma unroll
  for (int k = 0; k < 2 + kSMaxA; ++k) tot[k] = 0.0;
  for (int t = l; t < nt; t += 64)
#pragma unroll
    for (int k = 0; k < 2 + kSMaxA; ++k)
      if (k < NL) tot[k] += rows[(size_t)t * NL + k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < 2 + kSMaxA; ++k) tot[k] += __shfl_xor(tot[k], o, 64);
}
// The actor's KL gate from the tile loss rows (approx_kl = Σ / K, float32 as the fb tail writes it)
__device__ __forceinline__ bool s_gate_rows(const SArgs& P, int l, double (&tot)[2 + kSMaxA]) {
  s_loss_tot(P.w.lossa, P.nA, 2 + P.a.A, l, tot);
  const float akl = (float)(tot[1] / (double)(P.mb * P.D));
  return !P.gate || akl <= P.kl_thr;
}

// Adam's bias corrections of both nets, as launch 1 formed them from the step
// counts (s_bias_corr): nothing in launches 2 / 3 reads a step count, so the
// one thread that commits them needs no arrival count
__device__ __forceinline__ void s_adam_scalars(const SArgs& P, float (*sc)[2], int tid) {
  if (tid < 4) sc[tid >> 1][tid & 1] = P.w.dlogstd[kSScOff + tid];
}
// The step counts' commit (torch.optim.Adam's state['step'] += 1): the critic
// always, the actor when its KL gate is open (AG:731-760); one thread of one
// workgroup, after launch 1 read them
__device__ __forceinline__ void s_commit_steps(const SArgs& P, bool open_a) {
  if (open_a) *P.a.step = *P.a.step + 1.0f;
  *P.c.step = *P.c.step + 1.0f;
}
__device__ __forceinline__ bool s_gate_open(const SArgs& P) {
  return !P.gate || *P.kl_out / P.G.gdiv <= P.kl_thr;
}

// The vector parameters of both nets (b1, b2, W3, b3 and the actor's logstd),
// element e of [actor's | critic's]: its flat index i, and where its gradient
// is formed — the column of the tile partial rows (col, stride cstride; nt
// rows, one per tile) or, for logstd, dlogstd[u] (col = NULL).  false: past the end.
__device__ __forceinline__ bool s_vec_loc(const SArgs& P, int e, bool& actor, long long& i, const float*& col,
                                          int& cstride, int& nt, int& u) {
  const int A = P.a.A;
  const int na = 2 * kSH + A * kSH + 2 * A, nc = 2 * kSH + kSH + 1;
  if (e >= na + nc) return false;
  actor = e < na;
  const SNet& N = actor ? P.a : P.c;
  const int AA = actor ? A : 1;
  nt = actor ? P.nA : P.nC;
  const float* pA = actor ? P.w.partAa : P.w.partAc;
  const float* pB = actor ? P.w.partBa : P.w.partBc;
  const int PA = kSH + AA * kSH + AA;
  u = actor ? e : e - na;
  col = nullptr;
  cstride = 0;
  if (u < kSH) {                       // b1: Σ dZ1
    col = pB + u; cstride = kSH;
    i = N.b1 + u;
  } else if ((u -= kSH) < kSH) {       // b2: Σ dZ2
    col = pA + u; cstride = PA;
    i = N.b2 + u;
  } else if ((u -= kSH) < AA * kSH) {  // W3: Σ dout·H2
    col = pA + kSH + u; cstride = PA;
    i = N.w3 + u;
  } else if ((u -= AA * kSH) < AA) {   // b3: Σ dout
    col = pA + kSH + AA * kSH + u; cstride = PA;
    i = N.b3 + u;
  } else {                             // logstd (the actor's loss tail)
    u -= AA;
    i = N.logstd + u;
  }
  return true;
}

// ---------------------------------------------------------------- launch 2: weight gradients
// dW1 = dZ1ᵀ·X and dW2 = dZ2ᵀ·H1 of both nets from the transposed activations
// launch 1 wrote ([rows][K], K contiguous: C[n][m] = Σ_k A[n][k]·B[m][k]).  One
// 4-wave workgroup per 64×64 output tile and K-chunk (a run of 64-row steps):
// each wave owns a 32×32 quadrant (2×2 MFMA tiles, four accumulator chains),
// the tile's two 64-row operand panels are staged global → LDS by
// global_load_lds (16 B a lane) into a four-stage ring, three stages in flight
// while the fourth is read (counted vmcnt + raw s_barrier: the loads stay in
// flight across the barrier; with three stages a step took ~1.6 µs against
// ~0.85 of MFMA work: the loads' latency was not covered).  The four waves share every staged byte, so L2
// serves each operand row once per 64 outputs (the 32×32 blocks of round 5,
// a wave per K-quarter, read every operand byte 8× over: 0.20 of the MFMA peak).
// One chunk per tile (S = 1): the gradient goes straight into its sink (Adam
// in place, or the gradient buffer); otherwise the chunk partials of launch 3.
constexpr int kGT = 64;                   // output tile side (n and m)
constexpr int kGBK = 64;                  // K-rows per LDS stage (four quads)
constexpr int kGNS = 4;                   // stages in the LDS ring (three in flight while one is read)
constexpr int kGPanel = kGT * kGBK;       // floats of one operand's stage image (16 KB)
constexpr int kGLdsBytes = kGNS * 2 * kGPanel * 4 + 64;   // (+ the Adam scalars and the gate flag)

__host__ __device__ inline int s_gcb(int I) { return (I + kGT - 1) / kGT; }     // W1's column tiles
__host__ __device__ inline int s_gtiles(int I) { return 16 + 4 * s_gcb(I); }    // W2's 4×4, then W1's 4×cb
__host__ __device__ inline int s_mp(int I) { return 32 * ((I + 31) / 32); }     // a chunk partial's row width

// global_load_lds_dwordx4 by inline asm: the compiler neither counts it nor, not
// knowing which LDS bytes it writes, drains it with vmcnt(0) before every ds_read
// of the ring (the builtin's form did: the stages in flight were waited for at
// each step).  The ring's waits are the counted ones in the kernel.  m0: the
// wave-uniform LDS byte address (lane l writes m0 + 16·l).
__device__ __forceinline__ void s_glds16(const float* gsrc, unsigned m0v) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(m0v)
               : "memory");
}
// A stage image of one operand: tile rows 0..63 of a transposed activation, K-columns
// k0 .. k0+63, as [row][64] with the 16-B pieces XOR-swizzled (piece p of row r at
// position p ^ (r & 15): a 16-lane float4 read of one piece of 16 consecutive rows
// covers all 64 banks).  The LDS destination of an LDS-DMA load is lane-linear, so
// the swizzle is on the source: instruction q fills rows 4q .. 4q+3, wave w issues
// q = 4w .. 4w+3; src[i] is lane l's row / piece of instruction 4w + i (rows past
// the operand's last clamped to it, their products discarded), m0: the image's
// LDS byte address of instruction 4w.
__device__ __forceinline__ void s_gstage(const float* const (&src)[4], int k0, unsigned m0) {
#pragma unroll
  for (int i = 0; i < 4; ++i) s_glds16(src[i] + k0, m0 + 1024u * i);
}
__device__ __forceinline__ void s_gsrc(const float* base, int KS, int rmax, int w, int l, const float* (&src)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * (4 * w + i) + (l >> 4), p = l & 15;
    src[i] = base + (size_t)min(r, rmax) * KS + 4 * (p ^ (r & 15));
  }
}
// The wave's quadrant over one stage's four quads: c[2·rb + cb] += A rows 32wn + 16rb + j ×
// B rows 32wm + 16cb + j, κ = 16t + 4g + e (lane (g, j) reads piece 4t + g of its row).
// mid(): issued once the first quad's operand reads are (the next stage's loads:
// their issue then overlaps those reads' latency instead of delaying them).
template <class MID>
__device__ __forceinline__ void s_gquads(const float* la, const float* lb, int wn, int wm, int g, int j,
                                         f32x4 (&c)[4], MID mid) {
  float4 a[4][2], b[4][2];
  auto rd = [&](int t) {
#if defined(QS_WG_X) && (QS_WG_X & 2)
    // dev probe: no LDS reads (register operands)
    a[t][0] = a[t][1] = b[t][0] = b[t][1] = make_float4(la[0] + t, 1.f, 2.f, 3.f);
    return;
#endif
    const int ph = 4 * ((4 * t + g) ^ j);
    a[t][0] = *reinterpret_cast<const float4*>(la + (32 * wn + j) * kGBK + ph);
    a[t][1] = *reinterpret_cast<const float4*>(la + (32 * wn + 16 + j) * kGBK + ph);
    b[t][0] = *reinterpret_cast<const float4*>(lb + (32 * wm + j) * kGBK + ph);
    b[t][1] = *reinterpret_cast<const float4*>(lb + (32 * wm + 16 + j) * kGBK + ph);
  };
  rd(0);
  mid();
#pragma unroll
  for (int t = 1; t < 4; ++t) rd(t);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#define S_GQ(E)                                  \
  c[0] = s_mfma(a[t][0].E, b[t][0].E, c[0]);     \
  c[1] = s_mfma(a[t][0].E, b[t][1].E, c[1]);     \
  c[2] = s_mfma(a[t][1].E, b[t][0].E, c[2]);     \
  c[3] = s_mfma(a[t][1].E, b[t][1].E, c[3]);
    S_GQ(x) S_GQ(y) S_GQ(z) S_GQ(w)
#undef S_GQ
  }
}

// Workgroup T of n consecutive ones (the dispatcher deals them to the 8 XCDs
// round-robin, T mod 8) → logical index: each XCD's workgroups take one
// contiguous range of logical indices (the tiles of one K-chunk share its
// operand rows in that XCD's L2); the last n mod 8 unchanged
__device__ __forceinline__ int s_xcd_swz(int T, int n) {
  const int per = n >> 3;
  if (per == 0 || T >= 8 * per) return T;
  return (T & 7) * per + (T >> 3);
}

// The vector parameters' workgroup vb of launch 2 (b1, b2, W3, b3 of both nets,
// the actor's logstd), 16 lanes per element: lane k sums the tile partial rows
// t ≡ k mod 16 in order, a fixed DPP butterfly adds the lanes, into P.G.sink.
// Workgroup 0's wave 0 also records the minibatch's loss statistics and (fin:
// no launch 3 follows, Adam) commits the step counts.
__device__ __forceinline__ void s_vec_wg(const SArgs& P, int vb, bool adam, bool fin, const float (*sc)[2]) {
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int e = (vb * (int)blockDim.x + tid) >> 4, k = tid & 15;
  bool actor = false;
  long long i = 0;
  const float* col = nullptr;
  int cstride = 0, nt = 0, u = 0;
  const bool have = s_vec_loc(P, e, actor, i, col, cstride, nt, u);   // (uniform over the element's 16 lanes)
  // the element's partial rows and Adam operands first: their latency runs under
  // the loss totals' loads and butterflies (the gate), not after them
  float acc = 0.f, p0 = 0.f, m0 = 0.f, v0 = 0.f;
  if (have) {
    const SNet& N = actor ? P.a : P.c;
    if (adam && k == 0) {
      p0 = N.p[i];
      m0 = N.m[i];
      v0 = N.v[i];
    }
    if (col) {
      int tt = k;
      for (; tt + 16 * 7 < nt; tt += 16 * 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = col[(size_t)(tt + 16 * q) * cstride];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q];
      }
      for (; tt < nt; tt += 16) acc += col[(size_t)tt * cstride];
    }
  }
  // the actor's loss totals (every wave: the gate, logstd's gradient)
  double tot[2 + kSMaxA];
  const bool open_a = s_gate_rows(P, l, tot);
  if (have) {
    const SNet& N = actor ? P.a : P.c;
    const bool doit = !adam || !actor || open_a;
    // logstd: d(policy)/d logstd from the loss rows − ent_coef (AG:602-640)
    const float gsum = col ? s_row_sum(acc) : (float)tot[2 + u] - P.ent_coef;
    if (doit && k == 0) {
      if (!adam) {
        P.G.g[actor ? 0 : 1][i] = gsum;
      } else {
        const int si = actor ? 0 : 1;
        s_adam(N, i, gsum, sc[si][0], sc[si][1], nullptr, 0, 0, nullptr, p0, m0, v0);
      }
    }
  }
  if (vb == 0 && w == 0) {
    // the minibatch's loss statistics (the fb tail of ppo_heads_kernel's arithmetic):
    // approx_kl (the gate's value; the multi-rank exchange averages it), dlogstd, acc
    double totc[2 + kSMaxA];
    s_loss_tot(P.w.lossc, P.nC, 1, l, totc);
    if (l == 0) {
      const int A = P.a.A;
      const double K = (double)(P.mb * P.D);
      const float ent = P.w.dlogstd[kSMaxA];   // (launch 1's tile 0: the logstd before this launch's Adam)
      for (int a = 0; a < A; ++a) P.w.dlogstd[a] = (float)tot[2 + a] - P.ent_coef;
      const float akl = (float)(tot[1] / K);
      *P.kl_out = akl;
      P.acc[0] += tot[0] / K;
      P.acc[1] += 0.5 * (totc[0] / (double)P.mb);
      P.acc[2] += (double)(-ent);
      P.acc[3] += (double)akl;
      // no launch 3: the step counts (nothing in this launch reads them)
      if (fin && adam) s_commit_steps(P, open_a);
    }
  }
}

// Launch 2.  Workgroups [0, Σ tiles·S): one 64×64 tile of a weight matrix and
// one K-chunk each (the actor's first; within a net chunk-major, so an XCD's
// share of them (s_xcd_swz) is one chunk's operand rows); then the vector
// parameters (s_vec_wg).  fin: no launch 3 follows (every net in one chunk).
__global__ void __launch_bounds__(256) ppo_small_wgrad_kernel(SArgs P, int fin) {
  // ONE dynamic LDS array (a second __shared__ object beside the LDS-DMA ring can
  // make the compiler drain every load before each stage's reads)
  extern __shared__ __attribute__((aligned(16))) float s_lds[];
  float (*sc)[2] = reinterpret_cast<float (*)[2]>(s_lds + kGNS * 2 * kGPanel);
  int* sopen = reinterpret_cast<int*>(s_lds + kGNS * 2 * kGPanel + 4);
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, j = l & 15, g = l >> 4;
  const bool adam = P.G.sink == SINK_ADAM;
  const int ua = s_gtiles(P.a.I) * P.G.S[0], uc = s_gtiles(P.c.I) * P.G.S[1];
  const int blk = blockIdx.x;
  s_adam_scalars(P, sc, tid);
  W_STAMP(0);
  if (blk >= ua + uc) {
    __syncthreads();   // (sc)
    s_vec_wg(P, blk - ua - uc, adam, fin, sc);
    W_STAMP(3);
    return;
  }
  const bool actor = blk < ua;
  // (by value: through a reference into the kernel arguments every Adam element
  // reloaded the net's pointers and scalars behind the stores — ~5 µs of sink)
  const SNet N = actor ? P.a : P.c;
  const int si = actor ? 0 : 1, S = P.G.S[si], spc = P.G.spc[si], nt = s_gtiles(N.I);
  const int T = s_xcd_swz(actor ? blk : blk - ua, actor ? ua : uc);
  const int s = T / nt, t = T - s * nt;
  const bool l1 = t >= 16;
  int n0, m0;
  if (!l1) {
    n0 = kGT * (t >> 2);
    m0 = kGT * (t & 3);
  } else {
    const int tt = t - 16, cb = s_gcb(N.I);
    n0 = kGT * (tt / cb);
    m0 = kGT * (tt % cb);
  }
  const int M = l1 ? N.I : kSH;
  const int KS = actor ? P.KaS : P.KcS;
  const int nsteps = ((actor ? P.KaP : P.KcP) + kGBK - 1) / kGBK;
  const int st0 = s * spc, ns = min(nsteps, st0 + spc) - st0;
  const float* Ab = (actor ? (l1 ? P.w.dz1aT : P.w.dz2aT) : (l1 ? P.w.dz1cT : P.w.dz2cT)) + (size_t)n0 * KS;
  const float* Bb = (actor ? (l1 ? P.w.xaT : P.w.h1aT) : (l1 ? P.w.xcT : P.w.h1cT)) + (size_t)m0 * KS;
  const int bmax = min(kGT - 1, M - 1 - m0);
  const int wn = w >> 1, wm = w & 1;
  const bool live = kGT / 2 * wm < M - m0;   // the wave's 32 columns hold some of the matrix's
  const bool direct = S == 1;
  // The sink takes the wave's 32×32 quadrant row-contiguous (through LDS after the
  // contraction): lane l owns rows 32wn + (l >> 3) + 8u (u < 4) at columns
  // 32wm + 4(l & 7) .. + 3, so every store (and Adam's loads) is one float4 —
  // when the matrix's rows are float4-aligned (M a multiple of 4 and a 16-B
  // aligned offset; otherwise element by element).
  const long long wo = l1 ? N.w1 : N.w2;
  const bool vec4 = (M & 3) == 0 && (wo & 3) == 0;
  const int mq = m0 + 32 * wm + 4 * (l & 7);   // the lane's first column
  float4 pp[4], pm[4], pv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    pp[u] = pm[u] = pv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (direct && adam && vec4 && mq < M) {   // Adam's operands, in flight during the contraction
      const long long e0 = wo + (long long)(n0 + 32 * wn + (l >> 3) + 8 * u) * M + mq;
      pp[u] = *reinterpret_cast<const float4*>(N.p + e0);
      pm[u] = *reinterpret_cast<const float4*>(N.m + e0);
      pv[u] = *reinterpret_cast<const float4*>(N.v + e0);
    }
  }
  f32x4 c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the ring: stage i in image i mod kGNS; stages i + 1 .. i + kGNS − 1 in flight while i is read
  const float* asrc[4];
  const float* bsrc[4];
  s_gsrc(Ab, KS, kGT - 1, w, l, asrc);
  s_gsrc(Bb, KS, bmax, w, l, bsrc);
  const unsigned wu = __builtin_amdgcn_readfirstlane(w);
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)s_lds + 4096u * wu;
  auto stage = [&](int k) {   // stage k (a step of the chunk) into image k mod kGNS
#if defined(QS_WG_X) && (QS_WG_X & 1)
    return;   // dev probe: no operand loads (the contraction reads stale LDS)
#endif
    const unsigned m0 = lds0 + (unsigned)((k % kGNS) * 2 * kGPanel * 4);
    s_gstage(asrc, kGBK * (st0 + k), m0);
    s_gstage(bsrc, kGBK * (st0 + k), m0 + kGPanel * 4);
  };
  for (int k = 0; k < kGNS - 1 && k < ns; ++k) stage(k);
  static_assert(kGNS == 4, "the counted waits below assume at most two stages after the one read");
  for (int i = 0; i < ns; ++i) {
    // this wave's eight loads of stage i landed (the later stages' may stay in
    // flight: eight loads a stage), then every wave's: the barrier
    const int ahead = min(kGNS - 2, ns - 1 - i);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const float* img = s_lds + (i % kGNS) * 2 * kGPanel;
    // stage i + kGNS − 1 goes into the image every wave finished reading in step i − 1
    auto next = [&]() {
      if (i + kGNS - 1 < ns) stage(i + kGNS - 1);
    };
    // (every wave contracts, a dead quadrant too: a branch around the MFMAs made the
    // compiler copy the accumulators between AGPRs and VGPRs every step)
    s_gquads(img, img + kGPanel, wn, wm, g, j, c, next);
  }
  W_STAMP(1);
  __syncthreads();   // (sc; no LDS-DMA in flight)
  if (w == 0 && direct && adam && actor) {   // the actor's KL gate (AG:731-734)
    double tot[2 + kSMaxA];
    const bool o = s_gate_rows(P, l, tot);
    if (l == 0) *sopen = o;
  }
  __syncthreads();
  W_STAMP(2);
  const bool act = !(adam && actor) || *sopen;
  float* part = P.w.wpart[(actor ? 0 : 2) + (l1 ? 0 : 1)];
  const int Mp = l1 ? s_mp(N.I) : kSH;
  // the quadrant into LDS ([32][36]: 16-B aligned rows), then read back row-contiguous
  float* qd = s_lds + w * (32 * 36);
#pragma unroll
  for (int f = 0; f < 16; ++f) {
    const int q = f >> 2, r = f & 3;
    qd[(16 * (q >> 1) + 4 * g + r) * 36 + 16 * (q & 1) + j] = c[q][r];
  }
  // (the wave reads only its own quadrant: its LDS writes and reads are in order)
  if (!live) return;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int nl = (l >> 3) + 8 * u, en = n0 + 32 * wn + nl;
    const float4 v = *reinterpret_cast<const float4*>(qd + nl * 36 + 4 * (l & 7));
    const float vv[4] = {v.x, v.y, v.z, v.w};
    if (!direct) {
      if (vec4) {
        if (mq < M) *reinterpret_cast<float4*>(part + ((size_t)s * kSH + en) * Mp + mq) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (mq + e < M) part[((size_t)s * kSH + en) * Mp + mq + e] = vv[e];
      }
      continue;
    }
    if (!act) continue;
    const long long e0 = wo + (long long)en * M + mq;
    if (!adam) {
      if (vec4) {
        if (mq < M) *reinterpret_cast<float4*>(P.G.g[si] + e0) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (mq + e < M) P.G.g[si][e0 + e] = vv[e];
      }
    } else if (vec4) {
      if (mq >= M) continue;
      const float p4[4] = {pp[u].x, pp[u].y, pp[u].z, pp[u].w}, m4[4] = {pm[u].x, pm[u].y, pm[u].z, pm[u].w},
                  v4[4] = {pv[u].x, pv[u].y, pv[u].z, pv[u].w};
      float np[4], nm[4], nv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) s_adam_v(N, vv[e], sc[si][0], sc[si][1], p4[e], m4[e], v4[e], np[e], nm[e], nv[e]);
      *reinterpret_cast<float4*>(N.p + e0) = make_float4(np[0], np[1], np[2], np[3]);
      *reinterpret_cast<float4*>(N.m + e0) = make_float4(nm[0], nm[1], nm[2], nm[3]);
      *reinterpret_cast<float4*>(N.v + e0) = make_float4(nv[0], nv[1], nv[2], nv[3]);
      if (!l1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) N.w2t[(size_t)(mq + e) * kSH + en] = np[e];
      } else if (N.w1p) {
        *reinterpret_cast<float4*>(N.w1p + (size_t)en * s_ip(N.I) + mq) = make_float4(np[0], np[1], np[2], np[3]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (mq + e < M)
          s_adam(N, e0 + e, vv[e], sc[si][0], sc[si][1], l1 ? nullptr : N.w2t, en, mq + e, l1 ? N.w1p : nullptr,
                 N.p[e0 + e], N.m[e0 + e], N.v[e0 + e]);
    }
  }
  W_STAMP(3);
}

// Launch 3, one thread per parameter element: FROM_G = false — the weight
// matrices of the nets with K-chunks (S > 1): the chunk partials summed in
// chunk order, into P.G.sink; FROM_G = true (qs_ppo_small_adam, after the rank
// all-reduce) — every parameter's gradient from the gradient buffers ÷ gdiv,
// into Adam.  Elements: actor W1, W2, critic W1, W2 (row-major, as the
// parameters; FROM_G = false: only those of nets with S > 1), then (FROM_G)
// the vector parameters.  With Adam one thread commits the step counts.
template <bool FROM_G>
__global__ void __launch_bounds__(256) ppo_small_apply_kernel(SArgs P) {
  __shared__ float sc[2][2];
  const int tid = threadIdx.x;
  const int sink = FROM_G ? SINK_ADAM : P.G.sink;
  // the element, its gradient and Adam operands first (in flight across the scalars' barrier)
  int e = blockIdx.x * blockDim.x + tid;
  const bool inc[2] = {FROM_G || P.G.S[0] > 1, FROM_G || P.G.S[1] > 1};
  const int nw[4] = {inc[0] ? kSH * P.a.I : 0, inc[0] ? kSH * kSH : 0, inc[1] ? kSH * P.c.I : 0,
                     inc[1] ? kSH * kSH : 0};
  int part = 0;
  while (part < 4 && e >= nw[part]) e -= nw[part++];
  bool actor = part < 2, l1 = (part & 1) == 0, have = false;
  long long i = 0;
  int n = 0, m = 0;
  float gsum = 0.f, p0 = 0.f, m0 = 0.f, v0 = 0.f;
  if (part < 4) {
    const SNet& N = actor ? P.a : P.c;
    const int M = l1 ? N.I : kSH;
    n = e / M;
    m = e - n * M;
    i = (l1 ? N.w1 : N.w2) + e;
    have = true;
    if constexpr (FROM_G) {
      gsum = P.G.g[actor ? 0 : 1][i] / P.G.gdiv;
    } else {
      // the S chunk partials, eight loads in flight (clamped: unconditional), added in chunk order
      const int S = P.G.S[actor ? 0 : 1];
      const int Mp = l1 ? s_mp(N.I) : kSH;
      const float* pp = P.w.wpart[part] + (size_t)n * Mp + m;
      const size_t cs = (size_t)kSH * Mp;
      for (int q0 = 0; q0 < S; q0 += 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = pp[(size_t)min(q0 + q, S - 1) * cs];
#pragma unroll
        for (int q = 0; q < 8; ++q) gsum = (q0 + q == 0) ? v[q] : (q0 + q < S ? gsum + v[q] : gsum);
      }
    }
  } else if (FROM_G) {
    const float* col;
    int cstride, nt, u;
    if (s_vec_loc(P, e, actor, i, col, cstride, nt, u)) {
      have = true;
      l1 = false;
      gsum = P.G.g[actor ? 0 : 1][i] / P.G.gdiv;
    }
  }
  const SNet& N = actor ? P.a : P.c;
  if (have && sink == SINK_ADAM) {
    p0 = N.p[i];
    m0 = N.m[i];
    v0 = N.v[i];
  }
  s_adam_scalars(P, sc, tid);
  const bool open_a = sink != SINK_ADAM || s_gate_open(P);
  __syncthreads();
  if (have && (sink != SINK_ADAM || !actor || open_a)) {
    const int si = actor ? 0 : 1;
    const bool w2 = part < 4 && !l1;
    if (sink == SINK_GRAD) P.G.g[si][i] = gsum;
    else s_adam(N, i, gsum, sc[si][0], sc[si][1], w2 ? N.w2t : nullptr, n, m, part < 4 && l1 ? N.w1p : nullptr, p0, m0,
                v0);
  }
  // the step counts, by one thread (nothing in this launch reads them)
  if (sink == SINK_ADAM && blockIdx.x == 0 && tid == 0) s_commit_steps(P, open_a);
}

// Split-K weight gradient from transposed activations: partial[s][n][m] =
// Σ_{rows of chunk s} AT[n][row]·XT[m][row] (AT = dZᵀ [N][KP], XT = Xᵀ [M][KP],
// rows past K zero), one wave per 16×16 output tile and chunk, the A / B
// operands one float4 each per MFMA quad (rows 16q + 4g .. +3).  The chunk
// partials are summed in chunk order by qs_mlp_sum_adam.
__global__ void __launch_bounds__(64 * kSAW) wgrad_t_kernel(int N, int M, int KP, int ld, int S, const float* __restrict__ AT,
                                                            const float* __restrict__ XT, float* __restrict__ partial) {
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, j = l & 15, g = l >> 4;
  const int nm = (M + 15) / 16, tiles = (N / 16) * nm;
  const int T = blockIdx.x * kSAW + w;   // (chunk, tile): the chunks of a tile in consecutive waves
  if (T >= tiles * S) return;
  const int s = T % S, u = T / S, nb = u / nm, mb = u - nb * nm;
  const int rows = KP / S, r0 = s * rows;
  const int m = 16 * mb + j;
  const float* arow = AT + (size_t)(16 * nb + j) * ld + r0;
  const float* brow = XT + (size_t)min(m, M - 1) * ld + r0;   // (columns past M are not stored)
  f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
  s_wgrad_acc(arow, brow, rows / 16, g, c);
  if (m < M)
#pragma unroll
    for (int r = 0; r < 4; ++r) partial[((size_t)s * N + 16 * nb + 4 * g + r) * M + m] = c[r];
}

struct SLayout {
  int rb, rbc;    // 16-row blocks per forward/backward tile: the actor's, the critic's
  int nA, nC, KaP, KcP, KaS, KcS;
  int Sa, Sc;     // K-chunks of the weight gradients per net
  int spca, spcc; // their 64-row steps per chunk
  long long off[20];
  long long bytes;
};
// The weight gradients' K-chunks of both nets (launch 2): steps of 64 rows,
// spc per chunk.  A 64×64 tile and chunk is one workgroup on one CU for about
// spc × 2 048 MFMA cycles (~0.85 µs a step) plus ~1.5 steps of fill (the first
// stages' latency), so the launch takes about (rounds of the CUs) × (the
// longest chunk + 1.5); each chunk adds ~0.3 MB of partials that launch 3
// reads back (~0.2 step), and one chunk per net needs no launch 3 (~6 steps
// with its boundary).  The cheapest (Sa, Sc) by that estimate.
inline void s_chunks(int Ia, int Ic, long long KaP, long long KcP, SLayout& L) {
  const int na = Ia > 0 ? (int)((KaP + kGBK - 1) / kGBK) : 0, nc = (int)((KcP + kGBK - 1) / kGBK);
#ifdef QS_DEV_BUILD
  // dev probe: QS_WG_SPC="a,c" fixes the steps per chunk of the actor / critic
  if (const char* e = getenv("QS_WG_SPC")) {
    int pa = 0, pc = 0;
    if (sscanf(e, "%d,%d", &pa, &pc) == 2 && pa > 0 && pc > 0) {
      L.spca = pa;
      L.spcc = pc;
      L.Sa = na > 0 ? (na + pa - 1) / pa : 0;
      L.Sc = (nc + pc - 1) / pc;
      if (L.Sa <= kSMaxS && L.Sc <= kSMaxS) return;
    }
  }
#endif
  const int ta = Ia > 0 ? s_gtiles(Ia) : 0, tc = s_gtiles(Ic);
  double best = 1e30;
  L.Sa = Ia > 0 ? 1 : 0;
  L.Sc = 1;
  for (int pa = 1; pa <= (na > 0 ? na : 1); ++pa) {        // steps per actor chunk
    const int Sa = na > 0 ? (na + pa - 1) / pa : 0;
    if (Sa > kSMaxS) continue;
    for (int pc = 1; pc <= nc; ++pc) {
      const int Sc = (nc + pc - 1) / pc;
      if (Sc > kSMaxS) continue;
      const int units = ta * Sa + tc * Sc, rounds = (units + kSCUs - 1) / kSCUs;
      const int longest = std::max(na > 0 ? pa : 0, pc);
      const double cost = rounds * (longest + 1.5) + 0.2 * (Sa + Sc) + ((Sa > 1 || Sc > 1) ? 6.0 : 0.0);
      if (cost < best - 1e-9) {
        best = cost;
        L.Sa = Sa;
        L.Sc = Sc;
        L.spca = pa;
        L.spcc = pc;
      }
    }
  }
}
// Ia = 0: the critic's tiles only (qs_ppo_critic_tiles), no actor buffers
SLayout s_layout(int mb, int D, int Ia, int Ic, int A) {
  SLayout L;
  const long long Ka = Ia > 0 ? (long long)mb * D : 0, Kc = mb;
  // 32-row tiles once 16-row ones would not fit in one round of the CUs (the
  // two-block tile does twice the MFMA work for about 1.2x the latency)
  // (one-output actors only: wider heads' per-row state spills out of the 128 registers)
  // 48-row tiles (narrow nets, the padded W1 copies) once 32-row ones would not
  // fit either: C3 at G = 4 (8 192 actor rows) ran its 288 two-block tiles in
  // two rounds (72 µs)
  // (a wide critic only beside them at 16 rows: C5/8's 432-input critic)
  const long long t16 = (Ka + 15) / 16 + (Kc + 15) / 16, t32 = (Ka + 31) / 32 + (Kc + 31) / 32;
  L.rb = 1;
  if (Ia > 0 && A == 1 && t16 > kSCUs) {
    L.rb = 2;
    if (t32 > kSCUs && Ia <= kSNarrowI && (Ic <= kSNarrowI || (Ka + 47) / 48 + (Kc + 15) / 16 <= kSCUs)) L.rb = 3;
  } else if (Ia > 0 && A > 1 && t16 > kSCUs && Ia <= kSNarrowI && (Ka + 31) / 32 + (Kc + 15) / 16 <= kSCUs) {
    // wider heads at 32 rows: the tile spills 70 registers, and still beats two
    // rounds of 16-row tiles (C4/4: 128 → 112 µs per minibatch)
    L.rb = 2;
  }
  L.nA = (int)((Ka + 16 * L.rb - 1) / (16 * L.rb));
  // the critic's tiles at 16 rows while both nets' tiles still fit one round:
  // they are the launch's slowest (C3/8: 37.8 µs at 32 rows against the
  // actor's 30.6, phase stamps)
  L.rbc = (L.rb > 1 && L.nA + (Kc + 15) / 16 <= kSCUs) ? 1 : L.rb;
  L.nC = (int)((Kc + 16 * L.rbc - 1) / (16 * L.rbc));
  L.KaP = 16 * L.rb * L.nA;
  L.KcP = 16 * L.rbc * L.nC;
  // row strides off a power of two: rows 16 KB apart all mapped to one memory
  // channel (the critic's weight gradients ran 10x slower at 4 096 rows)
#ifdef QS_DEV_BUILD
  static const int pad = [] {   // dev probe: QS_SMALL_PAD overrides the pad (floats, a multiple of 4)
    const char* e = getenv("QS_SMALL_PAD");
    const int v = e ? atoi(e) : kSPad;
    return v >= 0 && v % 4 == 0 ? v : kSPad;
  }();
#else
  constexpr int pad = kSPad;
#endif
  // (launch 2 reads whole 64-row steps: the columns up to the next multiple of
  // 64 stay zero — nothing writes them, the caller zeroes the workspace)
  L.KaS = L.KaP ? (L.KaP + kGBK - 1) / kGBK * kGBK + pad : 0;
  L.KcS = (L.KcP + kGBK - 1) / kGBK * kGBK + pad;
  s_chunks(Ia, Ic, L.KaP, L.KcP, L);
  const long long pw = 4LL * kSH;   // bytes of a [256] partial column run
  const long long sz[20] = {
      4LL * Ia * L.KaS, 4LL * kSH * L.KaS, 4LL * kSH * L.KaS, 4LL * kSH * L.KaS,   // xaT h1aT dz2aT dz1aT
      4LL * Ic * L.KcS, 4LL * kSH * L.KcS, 4LL * kSH * L.KcS, 4LL * kSH * L.KcS,   // xcT h1cT dz2cT dz1cT
      4LL * L.nA * (kSH + A * kSH + A), 4LL * L.nA * kSH,                           // partAa partBa
      4LL * L.nC * (2 * kSH + 1), 4LL * L.nC * kSH,                                 // partAc partBc
      4LL * (kSScOff + 4), 8LL * L.nA * (2 + A), 8LL * L.nC, 4LL * (256 + kSBlkCnt),   // dlogstd (+ entropy, bias corr.) lossa lossc cnt
      pw * L.Sa * 32 * ((Ia + 31) / 32), pw * L.Sa * kSH,                           // K-chunk partials: actor W1 W2
      pw * L.Sc * 32 * ((Ic + 31) / 32), pw * L.Sc * kSH};                          //                  critic W1 W2
  long long o = 0;
  for (int i = 0; i < 20; ++i) {
    L.off[i] = o;
    o += (sz[i] + 255) & ~255LL;
  }
  L.bytes = o;
  return L;
}
}  // namespace

extern "C" {

const char* qs_ppo_small_last_error(void) { return g_serr.c_str(); }

int64_t qs_ppo_small_work_bytes(int32_t mb, int32_t D, int32_t Ia, int32_t Ic, int32_t A) {
  if (mb <= 0 || D <= 0 || Ia < 0 || Ic <= 0 || A < 1 || A > kSMaxA) return 0;
  return s_layout(mb, D, Ia, Ic, A).bytes;
}

int qs_ppo_small_layout(int32_t mb, int32_t D, int32_t Ia, int32_t Ic, int32_t A, int64_t* off, int32_t n_off) {
  if (mb <= 0 || D <= 0 || Ia < 0 || Ic <= 0 || A < 1 || A > kSMaxA || !off || n_off < 1)
    return sfail(QS_E_INVALID, "qs_ppo_small_layout: bad argument");
  const SLayout L = s_layout(mb, D, Ia, Ic, A);
  int64_t v[QS_PPO_SMALL_LAYOUT_N];
  for (int i = 0; i < 16; ++i) v[i] = L.off[i];
  v[16] = L.nA;
  v[17] = L.nC;
  v[18] = L.KaP;
  v[19] = L.KcP;
  v[20] = L.bytes;
  v[21] = L.KaS;
  v[22] = L.KcS;
  for (int i = 0; i < 4; ++i) v[23 + i] = L.off[16 + i];
  v[27] = L.Sa;
  v[28] = L.Sc;
  for (int i = 0; i < QS_PPO_SMALL_LAYOUT_N && i < n_off; ++i) off[i] = v[i];   // (never past the caller's array)
  return QS_OK;
}

int qs_wgrad_t(int64_t KP, int64_t ld, int32_t N, int32_t M, const float* AT, const float* XT, int32_t S,
               float* partial, void* stream) {
  if (KP <= 0 || N <= 0 || N % 16 || M <= 0 || M > 4096 || S <= 0 || KP % (16LL * S) || ld < KP || ld % 4 || !AT ||
      !XT || !partial || ld * (int64_t)(N > M ? N : M) >= (int64_t(1) << 31))
    return sfail(QS_E_INVALID, "qs_wgrad_t: bad argument (N a multiple of 16, KP a multiple of 16·S, ld >= KP "
                               "a multiple of 4)");
  static const bool attr = ((void)hipFuncSetAttribute((const void*)wgrad_t_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kSReserveW),
                            true);
  (void)attr;
  const long long waves = (long long)(N / 16) * ((M + 15) / 16) * S;
  hipLaunchKernelGGL(wgrad_t_kernel, dim3((unsigned)((waves + kSAW - 1) / kSAW)), dim3(64 * kSAW), kSReserveW,
                     (hipStream_t)stream, (int)N, (int)M, (int)KP, (int)ld, (int)S, AT, XT, partial);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : sfail(QS_E_HIP, std::string("qs_wgrad_t: ") + hipGetErrorString(e));
}

}  // extern "C"

static void s_bind(SArgs& P, const qs_mlp256* actor, const qs_mlp256* critic, const SLayout& L, void* work);

static int s_args(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const float* act, const float* logp_old,
                  const double* adv, const double* ret, float action_scale, float clip, float ent_coef, int32_t gate,
                  float kl_thr, const qs_mlp256* actor, const qs_mlp256* critic, float* kl_out, double* acc, void* work,
                  bool need_actor, SArgs& P, SLayout& L, const char* name) {
  if (mb <= 0 || D <= 0 || !obs || !idx || !ret || !actor || !critic || !acc || !work ||
      (need_actor && (!act || !logp_old || !adv || !kl_out)))
    return sfail(QS_E_INVALID, std::string(name) + ": bad argument");
  const int A = actor->out;
  if (A < 1 || A > kSMaxA || critic->out != 1 || actor->in < 1 || actor->in > kSMaxI || critic->in < 1 ||
      critic->in > kSMaxI || (need_actor && (actor->logstd < 0 || !actor->w2t)) || !critic->w2t)
    return sfail(QS_E_INVALID, std::string(name) + ": nets must be 256-wide with <= 640 inputs, A <= 4 actor outputs "
                                                   "(with logstd) and one critic output, W2ᵀ copies given");
  if ((actor->in > kSNarrowI || critic->in > kSNarrowI) && (!critic->w1p || (need_actor && !actor->w1p)))
    return sfail(QS_E_INVALID, std::string(name) + ": nets with more than 256 inputs need the padded W1 copies (w1p)");
  if ((actor->w2 & 3) || (critic->w2 & 3) || ((actor->in & 3) == 0 && (actor->w1 & 3)) ||
      ((critic->in & 3) == 0 && (critic->w1 & 3)))
    return sfail(QS_E_INVALID, std::string(name) + ": W1 / W2 must start 16-byte aligned in the flat buffers");
  if ((long long)mb * D * kSH >= (1LL << 31))
    return sfail(QS_E_INVALID, std::string(name) + ": minibatch too large for 32-bit activation offsets");
  L = s_layout(mb, D, actor->in, critic->in, A);
  // (the three-block tiles and the wider heads' two-block ones read layer 1 from
  // the padded copies only; the critic-only launch lays out its own tiles)
  if (need_actor && (L.rb == 3 || (L.rb == 2 && A > 1)) && (!critic->w1p || !actor->w1p))
    return sfail(QS_E_INVALID, std::string(name) + ": minibatches past 256 two-block tiles need the padded W1 copies (w1p)");
  P.mb = mb;
  P.D = D;
  P.rb = L.rb;
  P.rbc = L.rbc;
  P.nA = L.nA;
  P.nC = L.nC;
  P.KaP = L.KaP;
  P.KcP = L.KcP;
  P.KaS = L.KaS;
  P.KcS = L.KcS;
  P.X = obs;
  P.idx = (const long long*)idx;
  P.act = act;
  P.logp_old = logp_old;
  P.adv = adv;
  P.ret = ret;
  P.scale = action_scale;
  P.clip = clip;
  P.ent_coef = ent_coef;
  P.kl_thr = kl_thr;
  P.gate = gate;
  P.kl_out = kl_out;
  P.acc = acc;
  P.fb_tail = 0;
  s_bind(P, actor, critic, L, work);
  return QS_OK;
}

// The nets, the workspace views of layout L and the chunk counts; the sink:
// Adam, gradients ÷ 1
static void s_bind(SArgs& P, const qs_mlp256* actor, const qs_mlp256* critic, const SLayout& L, void* work) {
  auto net = [](const qs_mlp256* q) {
    SNet n;
    n.p = q->params;
    n.m = q->exp_avg;
    n.v = q->exp_avg_sq;
    n.step = q->step;
    n.w2t = q->w2t;
    n.w1 = q->w1;
    n.b1 = q->b1;
    n.w2 = q->w2;
    n.b2 = q->b2;
    n.w3 = q->w3;
    n.b3 = q->b3;
    n.logstd = q->logstd;
    n.I = q->in;
    n.A = q->out;
    n.lr = q->lr;
    n.beta1 = q->beta1;
    n.beta2 = q->beta2;
    n.eps = q->eps;
    n.w1p = q->w1p;
    return n;
  };
  P.a = net(actor);
  P.c = net(critic);
  char* wb = (char*)work;
  float** fv[13] = {&P.w.xaT, &P.w.h1aT, &P.w.dz2aT, &P.w.dz1aT, &P.w.xcT, &P.w.h1cT, &P.w.dz2cT,
                    &P.w.dz1cT, &P.w.partAa, &P.w.partBa, &P.w.partAc, &P.w.partBc, &P.w.dlogstd};
  for (int i = 0; i < 13; ++i) *fv[i] = (float*)(wb + L.off[i]);
  P.w.lossa = (double*)(wb + L.off[13]);
  P.w.lossc = (double*)(wb + L.off[14]);
  P.w.cnt = (unsigned*)(wb + L.off[15]);
  for (int i = 0; i < 4; ++i) P.w.wpart[i] = (float*)(wb + L.off[16 + i]);
  P.G.S[0] = L.Sa;
  P.G.S[1] = L.Sc;
  P.G.spc[0] = L.spca;
  P.G.spc[1] = L.spcc;
  P.G.sink = SINK_ADAM;
  P.G.g[0] = P.G.g[1] = nullptr;
  P.G.gdiv = 1.0f;
}

static void s_launch_fb(const SArgs& P, int grid, hipStream_t st) {
  // layer 1 from the padded W1 copies when every net in the launch has one;
  // the wide instance (a 640-input LDS X tile) only when a net needs it
  const bool v1 = P.c.w1p && (P.nA == 0 || P.a.w1p);
  const bool wide = P.c.I > kSNarrowI || (P.nA > 0 && P.a.I > kSNarrowI);
  // (the two-block and the wide two-block tiles use more than 80 KB of LDS: one a CU without a reserve)
  auto go = [&](auto kern, int reserve) { hipLaunchKernelGGL(kern, dim3(grid), dim3(kSBlock), reserve, st, P); };
  // (the wide instances read layer 1 from the padded copies only: s_args
  // refuses a net wider than kSNarrowI without one)
#define S_FB(AA)                                                                                                     \
  (P.rb == 3 ? (wide ? go(ppo_small_fb_kernel<AA, true, kSMaxI, 3, 1, kSNarrowI>, 0)   /* (narrow actor, w1p) */      \
                : P.rbc == 1 ? go(ppo_small_fb_kernel<AA, true, kSNarrowI, 3, 1>, 0)                                     \
                             : go(ppo_small_fb_kernel<AA, true, kSNarrowI, 3, 3>, 0)) :                                  \
  P.rb == 2 ? (wide ? (P.rbc == 1 ? go(ppo_small_fb_kernel<AA, true, kSMaxI, 2, 1>, 0)                                \
                                  : go(ppo_small_fb_kernel<AA, true, kSMaxI, 2, 2>, 0))                                \
                     : (v1 ? (P.rbc == 1 ? go(ppo_small_fb_kernel<AA, true, kSNarrowI, 2, 1>, 0)                       \
                                         : go(ppo_small_fb_kernel<AA, true, kSNarrowI, 2, 2>, 0))                      \
                           : (P.rbc == 1 ? go(ppo_small_fb_kernel<AA, false, kSNarrowI, 2, 1>, 0)                      \
                                         : go(ppo_small_fb_kernel<AA, false, kSNarrowI, 2, 2>, 0))))                   \
             : (wide ? go(ppo_small_fb_kernel<AA, true, kSMaxI, 1>, kSReserveFB)                                      \
                     : (v1 ? go(ppo_small_fb_kernel<AA, true, kSNarrowI, 1>, kSReserveFB)                             \
                           : go(ppo_small_fb_kernel<AA, false, kSNarrowI, 1>, kSReserveFB))))
#define S_FB1(AA)                                                                                    \
  (P.rb == 2 ? go(ppo_small_fb_kernel<AA, true, kSMaxI, 2, 1, kSNarrowI>, 0) :                       \
  wide ? go(ppo_small_fb_kernel<AA, true, kSMaxI, 1>, kSReserveFB)                                 \
        : (v1 ? go(ppo_small_fb_kernel<AA, true, kSNarrowI, 1>, kSReserveFB)                        \
              : go(ppo_small_fb_kernel<AA, false, kSNarrowI, 1>, kSReserveFB)))
  switch (P.a.A) {   // (two-block tiles: one-output actors, s_layout)
    case 1: S_FB(1); break;
    case 2: S_FB1(2); break;
    case 3: S_FB1(3); break;
    default: S_FB1(4); break;
  }
#undef S_FB
#undef S_FB1
}

// Launches 2 (and 3 when a net's weight gradients are split in K-chunks) into P.G.sink
static void s_launch_grad(const SArgs& P, hipStream_t st) {
  static const bool attr = ((void)hipFuncSetAttribute((const void*)ppo_small_wgrad_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, kGLdsBytes),
                            true);
  (void)attr;
  const bool one = P.G.S[0] <= 1 && P.G.S[1] == 1;
  const int nvec = (2 * kSH + P.a.A * kSH + 2 * P.a.A) + (3 * kSH + 1);
  const int vwg = (16 * nvec + 64 * kSGW - 1) / (64 * kSGW);   // 16 lanes per vector element
  const int grid = s_gtiles(P.a.I) * P.G.S[0] + s_gtiles(P.c.I) * P.G.S[1] + vwg;
  hipLaunchKernelGGL(ppo_small_wgrad_kernel, dim3(grid), dim3(64 * kSGW), kGLdsBytes, st, P, (int)one);
  if (one) return;
  long long nel = 0;
  for (int k = 0; k < 2; ++k)
    if (P.G.S[k] > 1) nel += (long long)kSH * ((k ? P.c.I : P.a.I) + kSH);
  hipLaunchKernelGGL(ppo_small_apply_kernel<false>, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, P);
}

extern "C" {

int qs_ppo_small_step(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const float* act,
                      const float* logp_old, const double* adv, const double* ret, float action_scale, float clip,
                      float ent_coef, int32_t gate, float kl_thr, const qs_mlp256* actor, const qs_mlp256* critic,
                      float* kl_out, double* acc, void* work, void* stream) {
  SArgs P;
  SLayout L;
  int rc = s_args(mb, D, obs, idx, act, logp_old, adv, ret, action_scale, clip, ent_coef, gate, kl_thr, actor, critic,
                  kl_out, acc, work, true, P, L, "qs_ppo_small_step");
  if (rc != QS_OK) return rc;
  if ((long long)mb * D > QS_PPO_SMALL_MAX_ROWS)
    return sfail(QS_E_INVALID, "qs_ppo_small_step: minibatch above QS_PPO_SMALL_MAX_ROWS actor rows");
  hipStream_t st = (hipStream_t)stream;
  s_launch_fb(P, L.nA + L.nC, st);
  s_launch_grad(P, st);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : sfail(QS_E_HIP, std::string("qs_ppo_small_step: ") + hipGetErrorString(e));
}

int qs_ppo_small_grads(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const float* act,
                       const float* logp_old, const double* adv, const double* ret, float action_scale, float clip,
                       float ent_coef, const qs_mlp256* actor, const qs_mlp256* critic, float* grad_a, float* grad_c,
                       float* kl_out, double* acc, void* work, void* stream) {
  SArgs P;
  SLayout L;
  int rc = s_args(mb, D, obs, idx, act, logp_old, adv, ret, action_scale, clip, ent_coef, 0, 0.f, actor, critic,
                  kl_out, acc, work, true, P, L, "qs_ppo_small_grads");
  if (rc != QS_OK) return rc;
  if (!grad_a || !grad_c) return sfail(QS_E_INVALID, "qs_ppo_small_grads: bad argument");
  if ((long long)mb * D > QS_PPO_SMALL_MAX_ROWS)
    return sfail(QS_E_INVALID, "qs_ppo_small_grads: minibatch above QS_PPO_SMALL_MAX_ROWS actor rows");
  P.G.sink = SINK_GRAD;
  P.G.g[0] = grad_a;
  P.G.g[1] = grad_c;
  hipStream_t st = (hipStream_t)stream;
  s_launch_fb(P, L.nA + L.nC, st);
  s_launch_grad(P, st);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : sfail(QS_E_HIP, std::string("qs_ppo_small_grads: ") + hipGetErrorString(e));
}

int qs_ppo_small_adam(int32_t mb, int32_t D, const qs_mlp256* actor, const qs_mlp256* critic, const float* grad_a,
                      const float* grad_c, float grad_div, int32_t gate, float kl_thr, const float* kl, void* work,
                      void* stream) {
  if (mb <= 0 || D <= 0 || !actor || !critic || !grad_a || !grad_c || !(grad_div > 0.f) || !kl || !work ||
      actor->out < 1 || actor->out > kSMaxA || actor->in < 1 || actor->in > kSMaxI || critic->in < 1 ||
      critic->in > kSMaxI || critic->out != 1 || actor->logstd < 0)
    return sfail(QS_E_INVALID, "qs_ppo_small_adam: bad argument");
  SArgs P = {};
  const SLayout L = s_layout(mb, D, actor->in, critic->in, actor->out);
  s_bind(P, actor, critic, L, work);
  P.mb = mb;
  P.D = D;
  P.nA = L.nA;
  P.nC = L.nC;
  P.gate = gate;
  P.kl_thr = kl_thr;
  P.kl_out = (float*)kl;   // read only: the all-reduced approx_kl sum (÷ grad_div)
  P.G.g[0] = (float*)grad_a;
  P.G.g[1] = (float*)grad_c;
  P.G.gdiv = grad_div;
  const int A = actor->out;
  const long long nel = (long long)kSH * (actor->in + critic->in) + 2LL * kSH * kSH + (2 * kSH + A * kSH + 2 * A) +
                        (3 * kSH + 1);
  hipLaunchKernelGGL(ppo_small_apply_kernel<true>, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, P);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : sfail(QS_E_HIP, std::string("qs_ppo_small_adam: ") + hipGetErrorString(e));
}

int qs_ppo_critic_tiles(int32_t mb, int32_t D, const float* obs, const int64_t* idx, const double* ret,
                        const qs_mlp256* critic, double* acc, void* work, void* stream) {
  if (!critic) return sfail(QS_E_INVALID, "qs_ppo_critic_tiles: bad argument");
  // the workspace layout of qs_ppo_small_layout(mb, D, 0, critic->in, 1): no actor tiles or buffers
  qs_mlp256 dummy = *critic;
  SArgs P;
  SLayout L;
  int rc = s_args(mb, D, obs, idx, nullptr, nullptr, nullptr, ret, 1.f, 0.f, 0.f, 0, 0.f, &dummy, critic, nullptr, acc,
                  work, false, P, L, "qs_ppo_critic_tiles");
  if (rc != QS_OK) return rc;
  L = s_layout(mb, D, 0, critic->in, 1);
  char* wb = (char*)work;
  float** fv[13] = {&P.w.xaT, &P.w.h1aT, &P.w.dz2aT, &P.w.dz1aT, &P.w.xcT, &P.w.h1cT, &P.w.dz2cT,
                    &P.w.dz1cT, &P.w.partAa, &P.w.partBa, &P.w.partAc, &P.w.partBc, &P.w.dlogstd};
  for (int i = 0; i < 13; ++i) *fv[i] = (float*)(wb + L.off[i]);
  P.w.lossa = (double*)(wb + L.off[13]);
  P.w.lossc = (double*)(wb + L.off[14]);
  P.w.cnt = (unsigned*)(wb + L.off[15]);
  P.nA = 0;   // critic tiles only
  P.fb_tail = 1;   // (the last tile adds the value loss to acc[1])
  P.rb = L.rb;     // (1: the critic-only layout)
  P.rbc = L.rbc;
  P.nC = L.nC;
  P.KaP = P.KaS = 0;
  P.KcP = L.KcP;
  P.KcS = L.KcS;
  s_launch_fb(P, L.nC, (hipStream_t)stream);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QS_OK : sfail(QS_E_HIP, std::string("qs_ppo_critic_tiles: ") + hipGetErrorString(e));
}

#ifdef QS_TILE_STAMPS
int qs_dev_wgrad_stamps(unsigned long long* host, int64_t n) {
  if (n > (int64_t)kStampWG * 4) n = (int64_t)kStampWG * 4;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? QS_OK
             : QS_E_HIP;
}
int qs_dev_tile_stamps(unsigned long long* host, int64_t n) {
  if (n > (int64_t)kStampWG * 8) n = (int64_t)kStampWG * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tile_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? QS_OK
             : QS_E_HIP;
}
#endif

}  // extern "C"
