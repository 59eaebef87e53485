/* Config 5 profile (HotMat, PermutationVector replicas): shared launchers + the k_replay variant. */
#include "mt_kernels.h"

int32_t replay_mat_lite(mt_engine* e);
int32_t replay_mat_skel(mt_engine* e);
int32_t replay_mat_none(mt_engine* e);
int32_t replay_mat_dl(mt_engine* e);

/* Default (MT_REPLAY_MAT_SKEL=2): only SkelLite (4.5 KB) in LDS, 7 waves per SIMD (116 Mops/s at 16k
 * replicas). =1 stages the whole Skel (10.7 KB), which caps residency at 14 documents per CU through
 * LDS (103 Mops/s); =0 stages nothing (104 Mops/s). */
static int32_t replay_mat(mt_engine* e) {
    if (e->fx) return replay_mat_dl(e); /* the delta-event build */
    if (e->mat_skel == 1) return replay_mat_skel(e);
    if (e->mat_skel == 2) return replay_mat_lite(e);
    return replay_mat_none(e);
}

const ProfOps* ops_mat() {
    static const ProfOps t = Launch<HotMat>::table(replay_mat);
    return &t;
}
