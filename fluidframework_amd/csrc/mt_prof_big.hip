/* HotBig profile (16,384 nodes, HBM-resident, one wave per document) */
#include "mt_kernels.h"

static int32_t replay_big(mt_engine* e) {
    if (e->fx) return launch_replay<HotBig>(e, k_replay<HotBig, false, 1, 1, 0, true>); /* delta events */
    return launch_replay<HotBig>(e, k_replay<HotBig, false>);
}

const ProfOps* ops_big() {
    static const ProfOps t = Launch<HotBig>::table(replay_big);
    return &t;
}
