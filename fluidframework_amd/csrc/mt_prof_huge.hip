/* Config 4 profile (HotHuge): tiled position index, one workgroup per large document */
#include "mt_kernels.h"

static int32_t replay_huge(mt_engine* e) {
    constexpr int block = WG * (1 + MT_PF_HELPERS); /* the replaying wave + its prefetch helpers */
    if (e->fx) return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge, true>, block); /* delta events */
    return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge>, block);
}

const ProfOps* ops_huge() {
    static const ProfOps t = Launch<HotHuge>::table(replay_huge);
    return &t;
}
