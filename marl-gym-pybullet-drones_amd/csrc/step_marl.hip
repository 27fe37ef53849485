// step_marl.hip — step-kernel instantiations for the Flock / Meetup / LeaderFollower
// family (one kernel set, task chosen at run time; see step_launch_impl.h).
#include "step_launch_impl.h"

QS_INSTANTIATE_LAUNCH(qs::kTaskMarl)
