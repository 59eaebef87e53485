/* k_replay of the config-5 profile (HotMat) for batches that hold snapshot-load records: the mt_mat_lite.hip
 * build with the load path */
#include "mt_kernels.h"

int32_t replay_mat_load(mt_engine* e) { return launch_replay<HotMat>(e, k_replay<HotMat, false, 7, 2>); }
