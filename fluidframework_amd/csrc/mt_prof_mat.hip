/* Config 5 profile (HotMat, PermutationVector replicas): shared launchers + the k_replay variant. */
#include "mt_kernels.h"

int32_t replay_mat_lite(mt_engine* e);
int32_t replay_mat_dl(mt_engine* e);
int32_t replay_mat_load(mt_engine* e);

/* Only SkelLite (4.5 KB) in LDS, 7 waves per SIMD: 116 Mops/s at 16k replicas in the round-1 sweep,
 * against 103 with the whole Skel (10.7 KB, residency capped at 14 documents per CU through LDS) and
 * 104 with nothing staged (those builds are no longer compiled). */
static int32_t replay_mat(mt_engine* e) {
    if (e->fx) return replay_mat_dl(e); /* the delta-event build */
    if (e->loads) return replay_mat_load(e); /* snapshot-load records */
    return replay_mat_lite(e);
}

const ProfOps* ops_mat() {
    static const ProfOps t = Launch<HotMat>::table(replay_mat);
    return &t;
}
