/* k_replay variant of the config-5 profile (HotMat), one per translation unit */
#include "mt_kernels.h"

int32_t replay_mat_none(mt_engine* e) { return launch_replay<HotMat>(e, k_replay<HotMat, false, 7, 0>); }
