/* Config 2/3 profile (HotSmall): shared launchers + the choice of k_replay variant. Each variant
 * is compiled in a translation unit of its own (mt_small_*.hip). */
#include "mt_kernels.h"

int32_t replay_small_w7(mt_engine* e);
int32_t replay_small_w8(mt_engine* e);
int32_t replay_small_w6(mt_engine* e);
int32_t replay_small_w5(mt_engine* e);
int32_t replay_small_w4(mt_engine* e);
int32_t replay_small_w2(mt_engine* e);
int32_t replay_small_lds(mt_engine* e);
int32_t replay_small_w7ni(mt_engine* e);
int32_t replay_small_w6ni(mt_engine* e);
int32_t replay_small_w8ni(mt_engine* e);
int32_t replay_small_dl(mt_engine* e);

/* Default: the hot image stays in HBM (skeleton and heap in LDS) and the kernel is built for 7 waves
 * per SIMD, so 7,168 documents are in flight (28 per CU): at one wavefront per document the replay
 * is bound by the latency of its dependent accesses, and occupancy hides more of it than full LDS
 * residency (4 documents per CU) saves (tools/gpu_occupancy.sh). A batch of <= 16,384 documents
 * (a strong-scaled shard) takes 8 waves: 1 or 2 full rounds instead of a last partial one.
 * MT_REPLAY_LDS=1 selects the fully LDS-staged form, MT_REPLAY_WAVES=2|4|5|6|7|8 the occupancy,
 * MT_REPLAY_NOINLINE=1 the build with compiler-chosen inlining. */
static int32_t replay_small(mt_engine* e) {
    if (e->fx) return replay_small_dl(e); /* the delta-event build */
    if (e->lds) return replay_small_lds(e);
    if (e->noinline) return e->waves == 8 ? replay_small_w8ni(e) : e->waves == 6 ? replay_small_w6ni(e) : replay_small_w7ni(e);
    if (e->waves == 8) return replay_small_w8(e);
    if (e->waves == 6) return replay_small_w6(e);
    if (e->waves == 5) return replay_small_w5(e);
    if (e->waves == 4) return replay_small_w4(e);
    if (e->waves == 2) return replay_small_w2(e);
    return replay_small_w7(e);
}

const ProfOps* ops_small() {
    static const ProfOps t = Launch<HotSmall>::table(replay_small);
    return &t;
}
