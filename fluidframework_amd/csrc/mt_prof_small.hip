/* Config 2/3 profile (HotSmall): shared launchers + the choice of k_replay variant. Each variant
 * is compiled in a translation unit of its own (mt_small_*.hip). */
#include "mt_kernels.h"

int32_t replay_small_w8(mt_engine* e);
int32_t replay_small_w4(mt_engine* e);
int32_t replay_small_dl(mt_engine* e);
int32_t replay_small_load(mt_engine* e);
int32_t replay_small_lds(mt_engine* e);

/* Default: the hot image stays in HBM (skeleton and heap in LDS) and the kernel is built for 8 waves
 * per SIMD, so 8,192 documents are in flight (32 per CU): at one wavefront per document the replay
 * is bound by the latency of its dependent accesses and by issue, and occupancy hides more of it than
 * full LDS residency (4 documents per CU) saves (round-2 sweep of 2-8 waves: profiles/r02_occupancy.txt;
 * the sweep's other builds are no longer compiled; the fully LDS-staged form measured 0.6x on config 2,
 * profiles/r03_c2_4096docs_bench_*.json, and is no longer built). A batch of at most 4 documents per SIMD
 * runs the 4-wave build (mt_small_w4.hip: no VGPR spills), and one of at most three documents per CU the LDS-image
 * build (mt_small_lds.hip), which has no occupancy to lose there. */
static int32_t replay_small(mt_engine* e) {
    if (e->fx) return replay_small_dl(e); /* the delta-event build */
    if (e->loads) return replay_small_load(e); /* snapshot-load records */
    if (e->waves == 1) return replay_small_lds(e); /* the hot image in LDS (mt_small_lds.hip) */
    return e->waves <= 4 ? replay_small_w4(e) : replay_small_w8(e); /* mt_engine_create picks the occupancy */
}

const ProfOps* ops_small() {
    static const ProfOps t = Launch<HotSmall>::table(replay_small);
    return &t;
}
