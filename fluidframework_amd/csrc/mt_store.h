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
    int64_t stride; /* bytes per document (Doc<HT>::stride) */
    Caps caps;

    MT_HD Doc<HT> doc(int64_t d) const {
        Doc<HT> v;
        v.b = base + d * stride;
        v.t = (HT*)v.b;
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

/* Fill the stride for capacities `caps` (the block layout is Doc<HT>'s); returns bytes for `ndocs`
 * documents. */
template <class HT>
inline int64_t store_layout(Store<HT>& st, const Caps& caps, int64_t ndocs) {
    st.stride = Doc<HT>::stride(caps);
    st.caps = caps;
    st.base = nullptr;
    return st.stride * ndocs;
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
