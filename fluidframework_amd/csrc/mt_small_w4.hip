/* k_replay of the config 2/3 profile (HotSmall) built for 4 waves per SIMD: 128 VGPRs per lane, so none spill to
 * scratch (the 8-wave build: 34 VGPRs, 108 B per lane) and fewer SGPRs spill (319 vs 559). The engine runs it when
 * every document of the batch is resident at 4 waves per SIMD anyway (config 2's 4,096 documents on 256 CUs:
 * 260.6M -> 293.6M ops/s, profiles/r05u_ab/), where the 8-wave build's extra occupancy has nothing to hold. */
/* With registers to spare at 4 waves, every image array is addressed by 32-bit offsets from the block base (mt_core.h
 * MT_A32: 2 % fewer VALU instructions, 42 fewer SGPR spills, none to scratch; config 2 293.3 -> 300.2M ops/s,
 * profiles/r06e_ab/). The 8-wave build keeps 64-bit addresses: there the offsets spilled VGPRs (34 -> 59) and config 3
 * lost 10 %. */
#define MT_A32 15
#include "mt_kernels.h"

int32_t replay_small_w4(mt_engine* e) {
    return launch_replay<HotSmall>(e, k_replay<HotSmall, false, 4, 1, 0, false, false>);
}
