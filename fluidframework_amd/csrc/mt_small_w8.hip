/* k_replay variant of the config 2/3 profile (HotSmall), one per translation unit. MT_SMALL_W (default 8)
 * is the occupancy target; other values are built only into experiment libraries (tools/gpu_r3d.sh). */
#include "mt_kernels.h"
#ifndef MT_SMALL_W
#define MT_SMALL_W 8
#endif

/* without snapshot-load records (Replica LOAD = false): the engine's default config-2/3 kernel */
int32_t replay_small_w8(mt_engine* e) {
    return launch_replay<HotSmall>(e, k_replay<HotSmall, false, MT_SMALL_W, 1, 0, false, false>);
}
