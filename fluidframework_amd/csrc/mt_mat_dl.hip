/* k_replay variant of the config-5 profile (HotMat) with delta events (caps.dcap > 0) */
#include "mt_kernels.h"

int32_t replay_mat_dl(mt_engine* e) { return launch_replay<HotMat>(e, k_replay<HotMat, false, 1, 2, 0, true>); }
