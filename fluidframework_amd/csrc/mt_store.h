/*
 * mt_store.h — per-document global-memory layout for a batch of documents.
 *
 * Each document owns one contiguous block: [hot image (HT) | cold rows | text arena (2 halves)
 * | membership log (gid, row id) | pending-group ring]. On the GPU the hot image is staged into
 * LDS for the duration of a replay (small profile) or used in place (larger profiles).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mt_core.h"

namespace mt {

template <class HT>
struct Store {
    typedef HT Hot;
    uint8_t* base;
    int64_t stride; /* bytes per document */
    int64_t offCold, offFrid, offArena, offMgid, offMrid, offGq;
    Caps caps;

    MT_HD Doc<HT> doc(int64_t d) const {
        uint8_t* b = base + d * stride;
        Doc<HT> v;
        v.t = (HT*)b;
        v.cold = (ColdRow*)(b + offCold);
        v.frid = (typename HT::IX*)(b + offFrid);
        v.arena = (uint16_t*)(b + offArena);
        v.mgid = (int32_t*)(b + offMgid);
        v.mrid = (int32_t*)(b + offMrid);
        v.gq = (int32_t*)(b + offGq);
        v.caps = caps;
        return v;
    }
};

inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

/* zeroed host block for a store (the hot image's leaf lines are 128-byte aligned); free() it */
inline uint8_t* host_store_alloc(int64_t bytes) {
    void* p = aligned_alloc(256, (size_t)align256(bytes));
    if (p) memset(p, 0, (size_t)align256(bytes));
    return (uint8_t*)p;
}

/* Fill offsets/stride for capacities `caps`; returns bytes for `ndocs` documents. */
template <class HT>
inline int64_t store_layout(Store<HT>& st, const Caps& caps, int64_t ndocs) {
    int64_t o = align256((int64_t)sizeof(HT));
    st.offCold = o;
    o = align256(o + (int64_t)sizeof(ColdRow) * HT::S);
    st.offFrid = o;
    o = align256(o + (int64_t)sizeof(typename HT::IX) * HT::S);
    st.offArena = o;
    o = align256(o + 2 * 2 * (int64_t)caps.acap);
    st.offMgid = o;
    o = align256(o + 4 * (int64_t)caps.mcap);
    st.offMrid = o;
    o = align256(o + 4 * (int64_t)caps.mcap);
    st.offGq = o;
    o = align256(o + 4 * (int64_t)caps.gcap);
    st.stride = o;
    st.caps = caps;
    st.base = nullptr;
    return o * ndocs;
}

inline bool caps_valid(const Caps& k) { return k.acap >= 16 && k.mcap >= 4 && k.gcap >= 1; }

/* profiles: 0 = HotSmall, 3 = HotMat, 1 = HotMid, 2 = HotBig, 4 = HotHuge (tiled, config 4) */
inline int profile_for(int32_t ncap) {
    if (ncap <= HotSmall::N) return 0;
    if (ncap <= HotMat::N) return 3;
    if (ncap <= HotMid::N) return 1;
    if (ncap <= HotBig::N) return 2;
    if (ncap <= HotHuge::N) return 4;
    return -1;
}

} /* namespace mt */
