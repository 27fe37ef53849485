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
