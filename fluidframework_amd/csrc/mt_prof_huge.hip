/* Config 4 profile (HotHuge): tiled position index, one workgroup per large document */
#include "mt_kernels.h"

static int32_t replay_huge(mt_engine* e) {
    constexpr int block = WG * (1 + MT_TILED_HELPERS); /* the replaying wave + its helper waves */
    if (e->fx) return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge, true>, block); /* delta events */
    /* the wide variant: asked for, or a replay that promotion cannot redo from the staged log (an incremental
     * batch on top of earlier ones, or promotion off), where the narrow kernel's E_CAPACITY would be final */
    if (e->wide || !e->fresh || !e->promote)
        return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge, false, false>, block);
    /* the heap in LDS; documents it cannot hold are promoted to the wide variant (mt_replay.hip promote) */
    return launch_replay<HotHuge>(e, k_replay_tiled<HotHuge, false, true>, block);
}

const ProfOps* ops_huge() {
    static const ProfOps t = Launch<HotHuge>::table(replay_huge);
    return &t;
}
