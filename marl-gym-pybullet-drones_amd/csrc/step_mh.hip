// step_mh.hip — step-kernel instantiations for QS_TASK_MULTIHOVER (see step_launch_impl.h).
#include "step_launch_impl.h"

QS_INSTANTIATE_LAUNCH(QS_TASK_MULTIHOVER)
