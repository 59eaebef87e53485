/* HotMid profile (2,048 nodes, HBM-resident, one wave per document) */
#include "mt_kernels.h"

static int32_t replay_mid(mt_engine* e) {
    if (e->fx) return launch_replay<HotMid>(e, k_replay<HotMid, false, 1, 1, 0, true>); /* delta events */
    return launch_replay<HotMid>(e, k_replay<HotMid, false>);
}

const ProfOps* ops_mid() {
    static const ProfOps t = Launch<HotMid>::table(replay_mid);
    return &t;
}
