/* k_replay of the config 2/3 profile (HotSmall) for batches that hold snapshot-load records (mt_oplog.h
 * MT_OP_RELOAD / COLLAB / APPEND): the same 8-waves-per-SIMD build as mt_small_w8.hip with the load path */
#include "mt_kernels.h"

int32_t replay_small_load(mt_engine* e) { return launch_replay<HotSmall>(e, k_replay<HotSmall, false, 8>); }
