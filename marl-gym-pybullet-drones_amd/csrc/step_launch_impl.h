// step_launch_impl.h — kernel launch dispatch, included by the per-task-family
// translation units (step_mh.hip, step_spiral.hip, step_generic.hip) so the
// kernel instantiations compile in parallel.
#pragma once
#include "step_launch.h"

namespace qs {

template <class T, int TASK, int ACT> static void launch_one(int grid, size_t lds, hipStream_t st, const Params<T>& P,
                                                             int ctrl_freq, int pyb_freq, int phys) {
  constexpr int kCF = TASK == QS_TASK_SPIRAL ? 48 : 30;   // SpiralAviary.py:28; MH:20 and the MARL tasks
  const bool cf = ctrl_freq == kCF && pyb_freq == 240;
  // the default control frequency without extra forces is the hot configuration:
  // fully compile-time (constant substeps/history, no force branch)
  const bool aux = P.aux != 0;
  if (phys == QS_PHYS_DYN) {
    if (cf && !aux) hipLaunchKernelGGL((step_kernel<T, TASK, ACT, kCF, QS_PHYS_DYN, false>), dim3(grid), dim3(kBlock), lds, st, P);
    else if (cf) hipLaunchKernelGGL((step_kernel<T, TASK, ACT, kCF, QS_PHYS_DYN, true>), dim3(grid), dim3(kBlock), lds, st, P);
    else hipLaunchKernelGGL((step_kernel<T, TASK, ACT, 0, QS_PHYS_DYN, true>), dim3(grid), dim3(kBlock), lds, st, P);
  } else {
    if (cf && !aux) hipLaunchKernelGGL((step_kernel<T, TASK, ACT, kCF, QS_PHYS_PYB, false>), dim3(grid), dim3(kBlock), lds, st, P);
    else if (cf) hipLaunchKernelGGL((step_kernel<T, TASK, ACT, kCF, QS_PHYS_PYB, true>), dim3(grid), dim3(kBlock), lds, st, P);
    else hipLaunchKernelGGL((step_kernel<T, TASK, ACT, 0, QS_PHYS_PYB, true>), dim3(grid), dim3(kBlock), lds, st, P);
  }
}

template <class T, int TASK> bool launch_task(int act, int grid, size_t lds, hipStream_t st, const Params<T>& P,
                                              int cf, int pf, int ph) {
  switch (act) {
    case QS_ACT_RPM: launch_one<T, TASK, QS_ACT_RPM>(grid, lds, st, P, cf, pf, ph); break;
    case QS_ACT_PID: launch_one<T, TASK, QS_ACT_PID>(grid, lds, st, P, cf, pf, ph); break;
    case QS_ACT_VEL: launch_one<T, TASK, QS_ACT_VEL>(grid, lds, st, P, cf, pf, ph); break;
    case QS_ACT_ONE_D_RPM: launch_one<T, TASK, QS_ACT_ONE_D_RPM>(grid, lds, st, P, cf, pf, ph); break;
    case QS_ACT_ONE_D_PID: launch_one<T, TASK, QS_ACT_ONE_D_PID>(grid, lds, st, P, cf, pf, ph); break;
    default: return false;
  }
  return true;
}


}  // namespace qs

#define QS_INSTANTIATE_LAUNCH(TASK)                                                                   \
  template bool qs::launch_task<float, TASK>(int, int, size_t, hipStream_t, const qs::Params<float>&, int, int, int); \
  template bool qs::launch_task<double, TASK>(int, int, size_t, hipStream_t, const qs::Params<double>&, int, int, int);
