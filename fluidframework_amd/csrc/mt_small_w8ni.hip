/* k_replay variant of the config 2/3 profile (HotSmall) with compiler-chosen inlining: the large
 * helpers (zamboni, split_row, the op bodies) stay functions, halving the kernel's code */
#define MT_NO_FORCE_INLINE
#include "mt_kernels.h"

int32_t replay_small_w8ni(mt_engine* e) { return launch_replay<HotSmall>(e, k_replay<HotSmall, false, 8, 1, 1>); }
