/* k_replay of the config 2/3 profile (HotSmall) with the whole hot image in LDS (41.6 KB: three documents per CU).
 * A batch of at most three documents per CU (config 1's farms, interactive engines, small test batches) has no
 * occupancy to lose, so each document's dependent accesses to its leaf lines, skeleton and heap become LDS round
 * trips instead of L2 / HBM ones; cold rows, the text arena and the logs stay in HBM. Built for one wave per SIMD:
 * registers for the whole event, no spills. The engine picks it when the batch fits (mt_engine_create). */
#define MT_A32 15
#include "mt_kernels.h"

int32_t replay_small_lds(mt_engine* e) {
    return launch_replay<HotSmall>(e, k_replay<HotSmall, true, 1, 1, 0, false, false>);
}
