// Dev-only probes of step_kernel, never part of the shipped library: included by
// step_kernel.h only when QS_DEV_BUILD is defined (scripts/build_dev_step.sh,
// `make STAMPS=1`).  Each probe removes one phase so that a timing difference
// names that phase's cost; the measurements they gave are in profiles/README.md
// and DESIGN.md §4.
//   QS_X_NOCOMPUTE    no PID and no substeps: the launch's memory floor
//   QS_X_NORESETDRAW  no try-0 reset draw / pair test (the reset path's share)
//   QS_X_RSTATS       per-workgroup counters of reset_search_kernel (printf)
//   QS_STAMPS_BUILD   per-wave phase timestamps (QS_STAMPS=1 at run time,
//                     scripts/stamps.py)
#pragma once

namespace qs_dev {
#ifdef QS_X_NOCOMPUTE
constexpr bool kNoCompute = true;
#else
constexpr bool kNoCompute = false;
#endif
#ifdef QS_X_NORESETDRAW
constexpr bool kNoResetDraw = true;
#else
constexpr bool kNoResetDraw = false;
#endif
}  // namespace qs_dev

#ifdef QS_STAMPS_BUILD
#define QS_STAMP(k)                                                                                    \
  do {                                                                                                 \
    if (P.stamps && threadIdx.x == 0) P.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// keeps the loads a stamp follows from being scheduled past it
#define QS_STAMP_SINK(x)                 \
  do {                                   \
    if (P.stamps) {                      \
      volatile auto sink_ = (x);         \
      (void)sink_;                       \
    }                                    \
  } while (0)
#else
#define QS_STAMP(k) do { } while (0)
#define QS_STAMP_SINK(x) do { } while (0)
#endif

// reset_search_kernel's per-workgroup counters (QS_X_RSTATS): time in the
// launch, picks, joins (futile: the env had closed), chunks tested, finds
#ifdef QS_X_RSTATS
#define QS_RS_BEGIN()                                               \
  const uint64_t rs_t0_ = __builtin_amdgcn_s_memrealtime();         \
  int rs_picks_ = 1, rs_joins_ = 0, rs_futile_ = 0, rs_chunks_ = 0, rs_found_ = 0
#define QS_RS_JOIN(futile) do { ++rs_joins_; rs_futile_ += (futile) ? 1 : 0; } while (0)
#define QS_RS_CHUNK(found) do { ++rs_chunks_; rs_found_ += (found) ? 1 : 0; } while (0)
#define QS_RS_PICK() do { ++rs_picks_; } while (0)
#define QS_RS_END(n)                                                                                        \
  do {                                                                                                      \
    const uint64_t rs_t1_ = __builtin_amdgcn_s_memrealtime();                                               \
    if (threadIdx.x == 0 && (blockIdx.x % 32 == 0 || rs_t1_ - rs_t0_ > 5000))                                \
      printf("RS n=%d wg=%d us=%.2f picks=%d joins=%d futile=%d chunks=%d found=%d\n", (n), (int)blockIdx.x, \
             (double)(rs_t1_ - rs_t0_) * 0.01, rs_picks_, rs_joins_, rs_futile_, rs_chunks_, rs_found_);     \
  } while (0)
#else
#define QS_RS_BEGIN() do { } while (0)
#define QS_RS_JOIN(futile) do { } while (0)
#define QS_RS_CHUNK(found) do { } while (0)
#define QS_RS_PICK() do { } while (0)
#define QS_RS_END(n) do { } while (0)
#endif
