/* k_replay variant of the config-5 profile (HotMat), one per translation unit */
#include "mt_kernels.h"

/* without snapshot-load records (Replica LOAD = false), as the config-2/3 kernel; mt_mat_load.hip has them */
int32_t replay_mat_lite(mt_engine* e) {
    return launch_replay<HotMat>(e, k_replay<HotMat, false, 7, 2, 0, false, false>);
}
