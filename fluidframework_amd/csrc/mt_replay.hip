/*
 * mt_replay.hip — the C ABI of include/mt_engine.h over the replay kernels (mt_kernels.h).
 * Store-dependent launches go through the engine's ProfOps table; each profile's kernels live in
 * their own translation units (mt_prof_*.hip, mt_small_*.hip, mt_mat_*.hip).
 */
#include "mt_kernels.h"

#include <algorithm>
#include <thread>

static int32_t ensure(mt_engine* e, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return MT_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    hipError_t st = hipMalloc(&b.p, bytes);
    if (st != hipSuccess) return hip_fail(e, st, "hipMalloc(staging)");
    b.cap = bytes;
    return MT_OK;
}

static int32_t launch_init(mt_engine* e) { return e->ops->init(e); }

extern "C" {

int32_t mt_engine_create(int32_t device, int64_t ndocs, const mt_caps* caps, mt_engine** out) {
    if (!out || !caps || ndocs < 1 || ndocs > (int64_t)0x7fffffff) return MT_E_ARG;
    *out = nullptr;
    Caps k = {caps->acap, caps->mcap, caps->gcap, caps->dcap, caps->rcap};
    int prof = profile_for(caps->ncap);
    if (!caps_valid(k) || prof < 0 || caps->ccap > 254 || caps->dcap < 0 || caps->rcap < 0)
        return MT_E_ARG; /* short ids are bytes; 0xFF = LocalClientId */
    mt_engine* e = new mt_engine();
    e->device = device;
    e->ndocs = ndocs;
    e->dcap = caps->dcap;
    e->rcap = caps->rcap;
    e->fx = caps->dcap > 0 || caps->rcap > 0;
    const char* g = getenv("MT_REPLAY_LDS");
    e->lds = g && g[0] == '1';
    e->waves = 8; /* occupancy of the HBM-resident small-profile kernel (mt_prof_small.hip) */
    e->profile = prof;
    e->ops = prof == 0 ? ops_small() : prof == 1 ? ops_mid() : prof == 3 ? ops_mat() : prof == 4 ? ops_huge() : ops_big();
    if (hipSetDevice(device) != hipSuccess) {
        delete e;
        return MT_E_HIP;
    }
    int64_t bytes = prof == 0 ? store_layout(e->s0, k, ndocs)
                  : prof == 1 ? store_layout(e->s1, k, ndocs)
                  : prof == 3 ? store_layout(e->s3, k, ndocs)
                  : prof == 4 ? store_layout(e->s4, k, ndocs)
                              : store_layout(e->s2, k, ndocs);
    if (hipMalloc(&e->mem, (size_t)bytes) != hipSuccess) {
        delete e;
        return MT_E_NOMEM;
    }
    e->s0.base = e->s1.base = e->s2.base = e->s3.base = e->s4.base = (uint8_t*)e->mem;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_E_HIP;
    }
    /* The zero fill goes on the engine's own stream, ahead of k_init. A hipMemset on the null
     * stream is not ordered with a non-blocking stream: a large store's fill could still be running
     * when k_init wrote the last documents' headers, and zeroed them after it (round 2: the last
     * documents of a 3.2 GB tiled store failed at their first events, only in long test runs). */
    if (hipMemsetAsync(e->mem, 0, (size_t)bytes, e->stream) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_E_HIP;
    }
    if (launch_init(e) != MT_OK || hipStreamSynchronize(e->stream) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_E_HIP;
    }
    *out = e;
    return MT_OK;
}

void mt_engine_destroy(mt_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    DevBuf* bufs[] = {&e->ops_buf, &e->op_off, &e->text, &e->text_off, &e->props,     &e->props_off,
                      &e->kv,     &e->kv_off, &e->tmp,  &e->local_ids, &e->prof};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    if (e->mem) (void)hipFree(e->mem);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char* mt_engine_last_error(const mt_engine* e) { return e ? e->err.c_str() : "null engine"; }
int64_t mt_engine_ndocs(const mt_engine* e) { return e ? e->ndocs : 0; }
void* mt_engine_stream(const mt_engine* e) { return e ? (void*)e->stream : nullptr; }
float mt_engine_last_run_ms(const mt_engine* e) { return e ? e->last_ms : 0.f; }

int32_t mt_engine_start_collab(mt_engine* e, const int32_t* local_long_ids, int32_t min_seq, int32_t cur_seq) {
    if (!e || !local_long_ids) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->local_ids, sizeof(int32_t) * e->ndocs);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(e->local_ids.p, local_long_ids, sizeof(int32_t) * e->ndocs, hipMemcpyHostToDevice,
                             e->stream));
    e->min_seq0 = min_seq;
    e->cur_seq0 = cur_seq;
    e->collab = true;
    rc = e->ops->start_collab(e, min_seq, cur_seq);
    if (rc) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_submit(mt_engine* e, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                         int64_t text_units, const int64_t* text_off, const mt_props_rec* props, int64_t nprops,
                         const int64_t* props_off, const mt_kv* kv, int64_t nkv, const int64_t* kv_off) {
    if (!e || !op_off || !text_off || !props_off || !kv_off) return MT_E_ARG;
    int64_t nd = e->ndocs;
    int64_t nops = op_off[nd];
    for (int64_t d = 0; d < nd; d++) {
        /* host-side shape checks before the kernel trusts any offset */
        if (op_off[d] < 0 || op_off[d] > op_off[d + 1] || text_off[d] < 0 || text_off[d] > text_units ||
            props_off[d] < 0 || props_off[d] > nprops || kv_off[d] < 0 || kv_off[d] > nkv)
            return MT_E_ARG;
    }
    /* every pool reference of every event must be in bounds before the kernel dereferences it: the
     * documents are checked in parallel on the host (up to 16 threads, one contiguous range each) */
    auto check = [&](int64_t d0, int64_t d1) -> bool {
        for (int64_t d = d0; d < d1; d++) {
            for (int64_t i = op_off[d]; i < op_off[d + 1]; i++) {
                const mt_op_rec& o = ops[i];
                int kind = o.kind & MT_OP_KIND_MASK;
                if (kind == MT_OP_INSERT && o.seg_kind == MT_SEG_TEXT &&
                    text_off[d] + (int64_t)o.text_off + o.text_len > text_units)
                    return false;
                /* snapshot-load records carry the segment length in pos2 (mt_oplog.h) */
                if ((kind == MT_OP_RELOAD || kind == MT_OP_APPEND) && o.seg_kind == MT_SEG_TEXT &&
                    (o.pos2 < 0 || text_off[d] + (int64_t)o.text_off + o.pos2 > text_units))
                    return false;
                if (o.props) {
                    if (props_off[d] + (int64_t)o.props > nprops) return false;
                    const mt_props_rec& pr = props[props_off[d] + o.props - 1];
                    if (kv_off[d] + (int64_t)pr.kv_off + pr.nkv > nkv) return false;
                }
            }
        }
        return true;
    };
    int nth = nops > (1 << 20) ? (int)std::min<int64_t>(16, std::max<unsigned>(1, std::thread::hardware_concurrency())) : 1;
    if (nth <= 1) {
        if (!check(0, nd)) return MT_E_ARG;
    } else {
        std::vector<std::thread> th;
        std::vector<char> ok((size_t)nth, 1);
        for (int t = 0; t < nth; t++)
            th.emplace_back([&, t] { ok[(size_t)t] = check(nd * t / nth, nd * (t + 1) / nth); });
        for (auto& x : th) x.join();
        for (char c : ok)
            if (!c) return MT_E_ARG;
    }
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc;
    if ((rc = ensure(e, e->ops_buf, sizeof(mt_op_rec) * nops))) return rc;
    if ((rc = ensure(e, e->op_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->text, 2 * text_units))) return rc;
    if ((rc = ensure(e, e->text_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->props, sizeof(mt_props_rec) * nprops))) return rc;
    if ((rc = ensure(e, e->props_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->kv, sizeof(mt_kv) * nkv))) return rc;
    if ((rc = ensure(e, e->kv_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if (nops) HIPCHK(e, hipMemcpyAsync(e->ops_buf.p, ops, sizeof(mt_op_rec) * nops, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->op_off.p, op_off, sizeof(int64_t) * (nd + 1), hipMemcpyHostToDevice, e->stream));
    if (text_units) HIPCHK(e, hipMemcpyAsync(e->text.p, text, 2 * text_units, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->text_off.p, text_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, e->stream));
    if (nprops)
        HIPCHK(e, hipMemcpyAsync(e->props.p, props, sizeof(mt_props_rec) * nprops, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->props_off.p, props_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, e->stream));
    if (nkv) HIPCHK(e, hipMemcpyAsync(e->kv.p, kv, sizeof(mt_kv) * nkv, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->kv_off.p, kv_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->staged = true;
    return MT_OK;
}

int32_t mt_engine_reset(mt_engine* e) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    return launch_init(e);
}

int32_t mt_engine_run(mt_engine* e) {
    if (!e || !e->staged) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
#ifdef MT_PROF
    if (ensure(e, e->prof, sizeof(uint64_t) * PH_N * e->ndocs)) return MT_E_NOMEM;
#endif
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    int32_t rc = e->ops->replay(e);
    if (rc) return rc;
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    return MT_OK;
}

int32_t mt_engine_sync(mt_engine* e) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->ev0, e->ev1) == hipSuccess) e->last_ms = ms;
    return MT_OK;
}

static int32_t read_hdr(mt_engine* e, int32_t* err, int32_t* err_op, int32_t* stats4, int64_t* work3) {
    HIPCHK(e, hipSetDevice(e->device));
    int64_t n = e->ndocs;
    int32_t rc = ensure(e, e->tmp, (size_t)n * (4 + 4 + 16 + 24));
    if (rc) return rc;
    int32_t* de = (int32_t*)e->tmp.p;
    int32_t* deo = de + n;
    int32_t* ds = deo + n;
    int64_t* dw = (int64_t*)(ds + 4 * n);
    rc = e->ops->hdr(e, de, deo, ds, dw);
    if (rc) return rc;
    if (err) HIPCHK(e, hipMemcpyAsync(err, de, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (err_op) HIPCHK(e, hipMemcpyAsync(err_op, deo, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (stats4) HIPCHK(e, hipMemcpyAsync(stats4, ds, 16 * n, hipMemcpyDeviceToHost, e->stream));
    if (work3) HIPCHK(e, hipMemcpyAsync(work3, dw, 24 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_errors(mt_engine* e, int32_t* err, int32_t* err_op) {
    if (!e) return MT_E_ARG;
    return read_hdr(e, err, err_op, nullptr, nullptr);
}
int32_t mt_engine_stats(mt_engine* e, int32_t* out4) {
    if (!e || !out4) return MT_E_ARG;
    return read_hdr(e, nullptr, nullptr, out4, nullptr);
}
int32_t mt_engine_work(mt_engine* e, int64_t* out3) {
    if (!e || !out3) return MT_E_ARG;
    return read_hdr(e, nullptr, nullptr, nullptr, out3);
}

int32_t mt_engine_digests(mt_engine* e, uint64_t* out) {
    if (!e || !out) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, sizeof(uint64_t) * e->ndocs);
    if (rc) return rc;
    rc = e->ops->digest(e, (uint64_t*)e->tmp.p);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(out, e->tmp.p, sizeof(uint64_t) * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int64_t mt_engine_dump(mt_engine* e, int64_t doc, uint8_t* out, int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    size_t need = sizeof(int64_t) + (size_t)(out ? cap : 0) + 16;
    if (ensure(e, e->tmp, need)) return -MT_E_HIP;
    int64_t* dn = (int64_t*)e->tmp.p;
    uint8_t* dbuf = out ? (uint8_t*)e->tmp.p + 16 : nullptr;
    int32_t rc = e->ops->dump(e, doc, dbuf, out ? cap : 0, dn);
    if (rc) return -rc;
    int64_t n = 0;
    if (hipMemcpyAsync(&n, dn, sizeof(int64_t), hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    if (out && n <= cap) {
        if (hipMemcpyAsync(out, dbuf, n, hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
        if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    }
    return n;
}

int32_t mt_engine_get_length(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t* out) {
    if (!e || !out || doc < 0 || doc >= e->ndocs) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, 16);
    if (rc) return rc;
    rc = e->ops->length(e, doc, ref_seq, long_client, (int32_t*)e->tmp.p);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(out, e->tmp.p, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int64_t mt_engine_get_text(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out,
                           int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    if (ensure(e, e->tmp, 16 + 2 * (size_t)(out ? cap : 0) + 16)) return -MT_E_HIP;
    int64_t* dn = (int64_t*)e->tmp.p;
    uint16_t* dbuf = out ? (uint16_t*)((uint8_t*)e->tmp.p + 16) : nullptr;
    int32_t rc = e->ops->text(e, doc, ref_seq, long_client, dbuf, out ? cap : 0, dn);
    if (rc) return -rc;
    int64_t n = 0;
    if (hipMemcpyAsync(&n, dn, sizeof(int64_t), hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    if (out) {
        int64_t m = n < cap ? n : cap;
        if (m > 0 && hipMemcpyAsync(out, dbuf, 2 * m, hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
        if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    }
    return n;
}

static int32_t seg_query(mt_engine* e, int64_t doc, int32_t mode, int32_t a, int32_t b, int32_t ref_seq,
                         int32_t long_client, int32_t* res7) {
    if (!e || doc < 0 || doc >= e->ndocs) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, 64);
    if (rc) return rc;
    rc = e->ops->seg(e, doc, mode, a, b, ref_seq, long_client, (int32_t*)e->tmp.p);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(res7, e->tmp.p, 7 * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_get_containing_segment(mt_engine* e, int64_t doc, int32_t pos, int32_t ref_seq, int32_t long_client,
                                         mt_seg_ref* out) {
    if (!out) return MT_E_ARG;
    int32_t r[7];
    int32_t rc = seg_query(e, doc, 0, pos, 0, ref_seq, long_client, r);
    if (rc) return rc;
    out->rid = r[0] ? r[1] : -1;
    out->gen = r[2];
    out->offset = r[3];
    out->length = r[4];
    out->seq = r[5];
    out->client = r[6];
    return MT_OK;
}

int32_t mt_engine_get_position(mt_engine* e, int64_t doc, int32_t rid, int32_t gen, int32_t ref_seq,
                               int32_t long_client, int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[7];
    int32_t rc = seg_query(e, doc, 1, rid, gen, ref_seq, long_client, r);
    if (rc) return rc;
    if (!r[0]) return MT_E_ARG;
    *out = r[1];
    return MT_OK;
}

/* the delta region of every document: offset inside a document's block, and the block stride */
static void delta_geometry(const mt_engine* e, int64_t* off, int64_t* stride) {
    switch (e->profile) {
    case 0: *off = Doc<HotSmall>::off_dl(e->s0.caps), *stride = e->s0.stride; break;
    case 1: *off = Doc<HotMid>::off_dl(e->s1.caps), *stride = e->s1.stride; break;
    case 3: *off = Doc<HotMat>::off_dl(e->s3.caps), *stride = e->s3.stride; break;
    case 4: *off = Doc<HotHuge>::off_dl(e->s4.caps), *stride = e->s4.stride; break;
    default: *off = Doc<HotBig>::off_dl(e->s2.caps), *stride = e->s2.stride; break;
    }
}

int32_t mt_engine_delta_state(mt_engine* e, int64_t* n_out, uint64_t* hash_out) {
    if (!e || e->dcap <= 0) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int64_t off, stride;
    delta_geometry(e, &off, &stride);
    std::vector<DState> st((size_t)e->ndocs);
    /* one strided copy: the DState at the head of each document's delta region */
    HIPCHK(e, hipMemcpy2DAsync(st.data(), sizeof(DState), (const uint8_t*)e->mem + off, (size_t)stride, sizeof(DState),
                               (size_t)e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (int64_t d = 0; d < e->ndocs; d++) {
        if (n_out) n_out[d] = st[d].n;
        if (hash_out) hash_out[d] = st[d].h;
    }
    return MT_OK;
}

int64_t mt_engine_deltas(mt_engine* e, int64_t doc, int32_t* out, int64_t cap) {
    if (!e || e->dcap <= 0 || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    int64_t off, stride;
    delta_geometry(e, &off, &stride);
    const uint8_t* base = (const uint8_t*)e->mem + doc * stride + off;
    DState st;
    if (hipMemcpyAsync(&st, base, sizeof st, hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    int64_t logged = st.n < e->dcap ? st.n : e->dcap;
    int64_t m = logged < cap ? logged : cap;
    if (out && m > 0) {
        if (hipMemcpyAsync(out, base + sizeof(DState), 4 * (size_t)m, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            return -MT_E_HIP;
        if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    }
    return logged;
}

int32_t mt_engine_ref_capacity(const mt_engine* e) { return e ? e->rcap : 0; }

int32_t mt_engine_ref_positions(mt_engine* e, int32_t* nref_out, int32_t* pos_out) {
    if (!e || e->rcap <= 0) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int64_t n = e->ndocs;
    int32_t rc = ensure(e, e->tmp, 4 * (size_t)n * (1 + (size_t)e->rcap));
    if (rc) return rc;
    int32_t* dn = (int32_t*)e->tmp.p;
    int32_t* dpos = dn + n;
    rc = e->ops->refpos(e, dn, dpos);
    if (rc) return rc;
    if (nref_out) HIPCHK(e, hipMemcpyAsync(nref_out, dn, 4 * (size_t)n, hipMemcpyDeviceToHost, e->stream));
    if (pos_out)
        HIPCHK(e, hipMemcpyAsync(pos_out, dpos, 4 * (size_t)n * e->rcap, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

#ifdef MT_PROF
/* profiling build only: per-doc phase cycles of the last run (PH_* order in mt_core.h) */
int32_t mt_engine_profile(mt_engine* e, uint64_t* out) {
    if (!e || !out || !e->prof.p) return MT_E_ARG;
    HIPCHK(e, hipMemcpyAsync(out, e->prof.p, sizeof(uint64_t) * PH_N * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}
#endif

} /* extern "C" */
