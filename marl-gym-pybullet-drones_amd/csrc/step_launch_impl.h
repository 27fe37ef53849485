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
  // the default control frequency is compile-time (constant substeps/history);
  // no extra forces / downwash only / general force set (step_kernel AUXM)
  const int auxm = P.aux == 0 ? 0 : (P.aux == QS_AUX_DW ? 1 : 2);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, st, P); };
  if (P.flags & QS_FLAG_CF2P) {   // DroneModel.CF2P: the general substep (AUXM 3), run-time frequency
    if (phys == QS_PHYS_DYN) go(step_kernel<T, TASK, ACT, 0, QS_PHYS_DYN, 3>);
    else go(step_kernel<T, TASK, ACT, 0, QS_PHYS_PYB, 3>);
    return;
  }
  if (phys == QS_PHYS_DYN) {
    if (!cf) go(step_kernel<T, TASK, ACT, 0, QS_PHYS_DYN, 2>);
    else if (auxm == 0) go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_DYN, 0>);
    else if (auxm == 1) go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_DYN, 1>);
    else go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_DYN, 2>);
  } else {
    if (!cf) go(step_kernel<T, TASK, ACT, 0, QS_PHYS_PYB, 2>);
    else if (auxm == 0) go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_PYB, 0>);
    else if (auxm == 1) go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_PYB, 1>);
    else go(step_kernel<T, TASK, ACT, kCF, QS_PHYS_PYB, 2>);
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
