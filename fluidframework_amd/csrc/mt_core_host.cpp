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
    Cols c;
    Caps k;
    int64_t ndocs;
    uint8_t* mem;
};

extern "C" {

mth_store* mth_create(int64_t ndocs, const int32_t* caps6) {
    Caps k = {caps6[0], caps6[1], caps6[2], caps6[3], caps6[4], caps6[5]};
    if (!caps_valid(k) || ndocs < 1) return nullptr;
    mth_store* s = (mth_store*)calloc(1, sizeof(mth_store));
    s->k = k;
    s->ndocs = ndocs;
    size_t bytes = layout(s->c, k, ndocs, nullptr);
    s->mem = (uint8_t*)calloc(1, bytes);
    if (!s->mem) {
        free(s);
        return nullptr;
    }
    layout(s->c, k, ndocs, s->mem);
    for (int64_t d = 0; d < ndocs; d++) {
        Replica<WaveHost> r(doc_view(s->c, k, d), WaveHost());
        r.init();
    }
    return s;
}

void mth_destroy(mth_store* s) {
    if (!s) return;
    free(s->mem);
    free(s);
}

void mth_start_collab(mth_store* s, int64_t doc, int32_t long_id, int32_t min_seq, int32_t cur_seq) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    r.start_collab(long_id, min_seq, cur_seq);
}

int32_t mth_apply(mth_store* s, int64_t doc, const mt_op_rec* op, const uint16_t* text, const mt_props_rec* props,
                  const mt_kv* kv) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    Pools p = {op, 1, text, props, kv};
    r.apply(*op, p);
    return r.d.h->err;
}

int32_t mth_replay(mth_store* s, int64_t doc, const mt_op_rec* ops, int64_t n, const uint16_t* text,
                   const mt_props_rec* props, const mt_kv* kv) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    Pools p = {ops, n, text, props, kv};
    r.replay(p);
    return r.d.h->err;
}

int32_t mth_error(mth_store* s, int64_t doc) { return s->c.hdr[doc].err; }
int32_t mth_error_op(mth_store* s, int64_t doc) { return s->c.hdr[doc].errOp; }

int32_t mth_length(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    if (long_client < 0) return r.length_local();
    int32_t sh = r.short_of(long_client);
    if (sh < 0) sh = 0x7fff; /* an unseen client sees only sequenced content */
    return r.length(ref_seq, sh);
}
int32_t mth_length_local(mth_store* s, int64_t doc) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    return r.length_local();
}

int64_t mth_text(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out, int64_t cap) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    int32_t sh;
    if (long_client < 0) {
        sh = r.d.h->localShort;
        ref_seq = r.d.h->currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff;
    }
    return r.get_text(ref_seq, sh, out, cap);
}

int64_t mth_dump(mth_store* s, int64_t doc, uint8_t* out, int64_t cap) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    return r.dump(out, cap);
}

uint64_t mth_digest(mth_store* s, int64_t doc) {
    Replica<WaveHost> r(doc_view(s->c, s->k, doc), WaveHost());
    return r.digest();
}

void mth_stats(mth_store* s, int64_t doc, int32_t* out8) {
    DocHdr* h = &s->c.hdr[doc];
    out8[0] = h->nleaf;
    out8[1] = h->hwSlots;
    out8[2] = h->hwHeap;
    out8[3] = h->heapN;
    out8[4] = h->memN;
    out8[5] = h->arenaTop;
    out8[6] = s->k.ncap - h->nfree;
    out8[7] = h->opsDone;
}

} /* extern "C" */
