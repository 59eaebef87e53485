/*
 * mt_core_host.cpp — serial host build of the replay core (mt_core.h with WaveHost).
 *
 * NOT the product compute path: the product replays on the GPU (mt_replay.hip). This build
 * exists for two host-side consumers that need the engine's exact semantics on the CPU:
 *   - the synthetic workload generator (mt_gen.cpp), whose replica model must place every op
 *     exactly where the engine will (so generated positions are always valid);
 *   - the CPU spec tests, which compare it with the oracle without a GPU.
 */
#include <stdlib.h>
#include <string.h>

#include "mt_core.h"
#include "mt_core_host.h"
#include "mt_store.h"
#include "mt_wave.h"

using namespace mt;

struct mth_store {
    int profile;
    int64_t ndocs;
    Store<HotSmall> s0;
    Store<HotMid> s1;
    Store<HotBig> s2;
    Store<HotMat> s3;
    Store<HotHuge> s4;
    uint8_t* mem;
    uint8_t* vkind; /* value kinds (mth_set_value_kinds; mt_engine_set_value_kinds) */
    int32_t nvk;
};

/* call F with a Replica<WaveHost, HT, true> (delta events on) for doc d of the store's profile */
template <class F>
static auto with_replica(mth_store* s, int64_t d, F&& f) {
    /* every call ends with commit(): the replica's register header goes back to the image */
    if (s->profile == 0) {
        Replica<WaveHost, HotSmall, true> r(s->s0.doc(d), WaveHost());
        auto res = f(r);
        r.commit();
        return res;
    } else if (s->profile == 3) {
        Replica<WaveHost, HotMat, true> r(s->s3.doc(d), WaveHost());
        auto res = f(r);
        r.commit();
        return res;
    } else if (s->profile == 1) {
        Replica<WaveHost, HotMid, true> r(s->s1.doc(d), WaveHost());
        auto res = f(r);
        r.commit();
        return res;
    } else if (s->profile == 4) {
        Replica<WaveHost, HotHuge, true> r(s->s4.doc(d), WaveHost());
        auto res = f(r);
        r.commit();
        return res;
    }
    Replica<WaveHost, HotBig, true> r(s->s2.doc(d), WaveHost());
    auto res = f(r);
    r.commit();
    return res;
}

extern "C" {

mth_store* mth_create(int64_t ndocs, const int32_t* caps6) { return mth_create_dl(ndocs, caps6, 0); }

mth_store* mth_create_dl(int64_t ndocs, const int32_t* caps6, int32_t dcap) {
    return mth_create_fx(ndocs, caps6, dcap, 0);
}

mth_store* mth_create_fx(int64_t ndocs, const int32_t* caps6, int32_t dcap, int32_t rcap) {
    return mth_create_fx2(ndocs, caps6, dcap, rcap, 0);
}

mth_store* mth_create_fx2(int64_t ndocs, const int32_t* caps6, int32_t dcap, int32_t rcap, int32_t pcap) {
    /* caps6 = (ncap, hcap[ignored: 2*ncap], acap, mcap, gcap, ccap[ignored: 64]); dcap: delta event
     * log words per doc (mt_caps.dcap); rcap: local references per doc (mt_caps.rcap); pcap:
     * PermutationVector handles per doc (mt_caps.pcap) */
    Caps k = {caps6[2], caps6[3], caps6[4], dcap < 0 ? 0 : dcap, rcap < 0 ? 0 : rcap, pcap < 0 ? 0 : pcap};
    int prof = profile_for(caps6[0]);
    if (!caps_valid(k) || ndocs < 1 || prof < 0) return nullptr;
    mth_store* s = (mth_store*)calloc(1, sizeof(mth_store));
    s->profile = prof;
    s->ndocs = ndocs;
    int64_t bytes = prof == 0 ? store_layout(s->s0, k, ndocs)
                  : prof == 1 ? store_layout(s->s1, k, ndocs)
                  : prof == 3 ? store_layout(s->s3, k, ndocs)
                  : prof == 4 ? store_layout(s->s4, k, ndocs)
                              : store_layout(s->s2, k, ndocs);
    s->mem = host_store_alloc(bytes);
    if (!s->mem) {
        free(s);
        return nullptr;
    }
    s->s0.base = s->s1.base = s->s2.base = s->s3.base = s->s4.base = s->mem;
    for (int64_t d = 0; d < ndocs; d++) with_replica(s, d, [](auto& r) { r.init(); return 0; });
    return s;
}

void mth_destroy(mth_store* s) {
    if (!s) return;
    free(s->vkind);
    free(s->mem);
    free(s);
}

void mth_start_collab(mth_store* s, int64_t doc, int32_t long_id, int32_t min_seq, int32_t cur_seq) {
    with_replica(s, doc, [&](auto& r) { r.start_collab(long_id, min_seq, cur_seq); return 0; });
}

int32_t mth_apply(mth_store* s, int64_t doc, const mt_op_rec* op, const uint16_t* text, const mt_props_rec* props,
                  const mt_kv* kv) {
    return with_replica(s, doc, [&](auto& r) {
        Pools p = {op, 1, text, props, kv, s->vkind, s->nvk};
        r.vk = s->vkind;
        r.nvk = s->nvk;
        r.apply(*op, p);
        return r.h.err;
    });
}

int32_t mth_replay(mth_store* s, int64_t doc, const mt_op_rec* ops, int64_t n, const uint16_t* text,
                   const mt_props_rec* props, const mt_kv* kv) {
    return with_replica(s, doc, [&](auto& r) {
        Pools p = {ops, n, text, props, kv, s->vkind, s->nvk};
        r.replay(p);
        return r.h.err;
    });
}

void mth_set_value_kinds(mth_store* s, const uint8_t* kinds, int32_t n) {
    free(s->vkind);
    s->vkind = n > 0 ? (uint8_t*)malloc((size_t)n) : nullptr;
    if (n > 0) memcpy(s->vkind, kinds, (size_t)n);
    s->nvk = n > 0 ? n : 0;
}

int32_t mth_error(mth_store* s, int64_t doc) {
    return with_replica(s, doc, [](auto& r) { return r.h.err; });
}
int32_t mth_error_op(mth_store* s, int64_t doc) {
    return with_replica(s, doc, [](auto& r) { return r.z.h.errOp; });
}

int32_t mth_length(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client) {
    return with_replica(s, doc, [&](auto& r) {
        if (long_client < 0) return r.length_local();
        int32_t sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff; /* an unseen client sees only sequenced content */
        return r.length(ref_seq, sh);
    });
}
int32_t mth_length_local(mth_store* s, int64_t doc) {
    return with_replica(s, doc, [](auto& r) { return r.length_local(); });
}

int64_t mth_text(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out, int64_t cap) {
    return mth_text_range(s, doc, ref_seq, long_client, nullptr, 0, INT32_MIN, INT32_MIN, out, cap);
}

int64_t mth_text_range(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client, const uint16_t* ph,
                       int32_t pl, int32_t start, int32_t end, uint16_t* out, int64_t cap) {
    return with_replica(s, doc, [&](auto& r) {
        int32_t sh;
        int32_t rs = ref_seq;
        if (long_client < 0) {
            sh = r.h.localShort;
            rs = r.h.currentSeq;
        } else {
            sh = r.short_of(long_client);
            if (sh < 0) sh = 0x7fff;
        }
        return r.get_text_range(rs, sh, start, end, ph, pl, out, cap);
    });
}

/* SharedSequence.getItems(start, end) in the local view (Replica::get_items; end = INT32_MIN: undefined) */
int64_t mth_items(mth_store* s, int64_t doc, int32_t start, int32_t end, uint16_t* out, int64_t cap) {
    return with_replica(s, doc, [&](auto& r) { return r.get_items(start, end, out, cap); });
}

/* getContainingSegment + getPosition of the found row: out6 = {found, offset, length, seq, long client,
 * position} (the layout of the oracle's mto_get_containing) */
int32_t mth_containing(mth_store* s, int64_t doc, int32_t pos, int32_t ref_seq, int32_t long_client, int32_t* out6) {
    return with_replica(s, doc, [&](auto& r) {
        int32_t sh = long_client < 0 ? r.h.localShort : r.short_of(long_client);
        int32_t rs = long_client < 0 ? r.h.currentSeq : ref_seq;
        if (sh < 0) sh = 0x7fff;
        for (int i = 0; i < 6; i++) out6[i] = 0;
        int32_t off = 0;
        int32_t slot = r.containing(pos, rs, sh, &off);
        if (slot < 0) return 0;
        out6[0] = 1;
        out6[1] = off;
        out6[2] = r.z.len(slot);
        out6[3] = r.z.seq(slot);
        out6[4] = r.long_of_cli(slot);
        out6[5] = r.position_of(slot, rs, sh);
        return 1;
    });
}

int64_t mth_dump(mth_store* s, int64_t doc, uint8_t* out, int64_t cap) {
    return with_replica(s, doc, [&](auto& r) { return r.dump(out, cap); });
}

uint64_t mth_digest(mth_store* s, int64_t doc) {
    return with_replica(s, doc, [](auto& r) { return r.digest(); });
}

/* delta events of one doc (mt_oplog.h): words emitted (returned), their FNV-1a-64, and the logged
 * words (at most min(n, dcap, cap)) */
int64_t mth_deltas(mth_store* s, int64_t doc, int32_t* out, int64_t cap, uint64_t* hash) {
    return with_replica(s, doc, [&](auto& r) -> int64_t {
        if (r.d.caps.dcap <= 0) {
            if (hash) *hash = 0;
            return 0;
        }
        const DState* st = r.d.dstate();
        int64_t m = st->n < r.d.caps.dcap ? st->n : r.d.caps.dcap;
        if (m > cap) m = cap;
        for (int64_t i = 0; out && i < m; i++) out[i] = r.d.dlog()[i];
        if (hash) *hash = st->h;
        return st->n;
    });
}

/* local references of one doc: their count (returned) and LocalReference.toPosition() of each */
int32_t mth_ref_positions(mth_store* s, int64_t doc, int32_t* out, int32_t cap) {
    return with_replica(s, doc, [&](auto& r) -> int32_t {
        if (r.d.caps.rcap <= 0) return 0;
        int32_t n = r.d.dstate()->nref;
        for (int32_t i = 0; i < n && i < cap; i++) out[i] = r.ref_position(i);
        return n;
    });
}

/* the doc's HandleTable.snapshot(): its length (returned) and up to cap entries */
int64_t mth_handle_table(mth_store* s, int64_t doc, int32_t* out, int64_t cap) {
    return with_replica(s, doc, [&](auto& r) -> int64_t {
        if (r.d.caps.pcap <= 0) return -1;
        int64_t n = r.d.dstate()->hlen;
        for (int64_t i = 0; out && i < n && i < cap; i++) out[i] = r.d.ht()[i];
        return n;
    });
}

/* HandleCache.getHandle(pos) in the local view: start + offset, INT32_MIN if unallocated; -1: no segment */
int32_t mth_get_handle(mth_store* s, int64_t doc, int32_t pos, int32_t* out) {
    return with_replica(s, doc, [&](auto& r) -> int32_t {
        int32_t off = 0;
        int32_t sl = r.containing(pos, r.h.currentSeq, r.h.localShort, &off);
        if (sl < 0) return -1;
        uint32_t st = (r.z.flags(sl) & RF_PERM) ? r.cold(sl).toff : 0u;
        *out = st ? (int32_t)st + off : INT32_MIN;
        return 0;
    });
}

/* pending segment groups (local ops in flight) of one doc */
int32_t mth_pending(mth_store* s, int64_t doc) {
    return with_replica(s, doc, [](auto& r) { return r.zh->gqN; });
}

void mth_stats(mth_store* s, int64_t doc, int32_t* out8) {
    with_replica(s, doc, [&](auto& r) {
        const RegHdr* h = &r.h; /* the fields the replica keeps in registers (MT_HDR_FIELDS) */
        DocHdr* zh = r.zh;   /* the rest (the image header) */
        out8[0] = h->nleaf;
        out8[1] = zh->hwSlots;
        out8[2] = zh->hwHeap;
        out8[3] = h->heapN;
        out8[4] = zh->memN;
        out8[5] = h->arenaTop;
        out8[6] = (int32_t)(sizeof(r.z.nparent) / sizeof(r.z.nparent[0])) - zh->nfree;
        out8[7] = h->opsDone;
        return 0;
    });
}

} /* extern "C" */

/* MergeTree.posFromRelativePos in the local view (long_client < 0) or (ref_seq, long_client); returns 0 and
 * the position (-1: no marker holds the id), or MT_E_UNSUPPORTED (4) if several markers hold it */
int32_t mth_pos_from_relpos(mth_store* s, int64_t doc, int32_t kid, int32_t vid, int32_t before, int32_t has_off,
                            int32_t off, int32_t ref_seq, int32_t long_client, int32_t* out) {
    return with_replica(s, doc, [&](auto& r) {
        int32_t sh = long_client < 0 ? r.h.localShort : r.short_of(long_client);
        int32_t rs = long_client < 0 ? r.h.currentSeq : ref_seq;
        if (sh < 0) sh = 0x7fff;
        int32_t m = r.marker_by_id(kid, vid);
        if (m == -2) return (int32_t)4;
        int32_t pos = -1;
        if (m >= 0) {
            pos = r.position_of(m, rs, sh);
            if (!before) pos += r.z.len(m) + (has_off ? off : 0);
            else if (has_off) pos -= off;
        }
        *out = pos;
        return (int32_t)0;
    });
}
