// step_launch.h — launch entry of the step kernel for one task family.
#pragma once
#include "step_kernel.h"

namespace qs {
// Launches step_kernel<T, TASK, act, ...> (control frequency and physics chosen
// from cf/pf/ph).  Defined and explicitly instantiated in one translation unit
// per task family.  Returns false for an unknown action type.
template <class T, int TASK>
bool launch_task(int act, int grid, size_t lds, hipStream_t st, const Params<T>& P, int cf, int pf, int ph);
}  // namespace qs
