/* k_replay variant of the config 2/3 profile (HotSmall) with delta events (caps.dcap > 0) */
#include "mt_kernels.h"

int32_t replay_small_dl(mt_engine* e) { return launch_replay<HotSmall>(e, k_replay<HotSmall, false, 1, 1, 0, true>); }
