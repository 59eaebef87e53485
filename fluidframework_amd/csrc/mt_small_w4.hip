/* k_replay variant of the config 2/3 profile (HotSmall), one per translation unit */
#include "mt_kernels.h"

int32_t replay_small_w4(mt_engine* e) { return launch_replay<HotSmall>(e, k_replay<HotSmall, false, 4>); }
