/* Config 4 profile (HotHuge): tiled position index, one workgroup per large document */
#include "mt_kernels.h"

static int32_t replay_huge(mt_engine* e) {
    if (e->fx) return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge, true>); /* delta events */
    return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge>);
}

const ProfOps* ops_huge() {
    static const ProfOps t = Launch<HotHuge>::table(replay_huge);
    return &t;
}
