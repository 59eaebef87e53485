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

/* ---- staging the op logs ------------------------------------------------------------------------ */
struct SubmitArgs {
    const mt_op_rec* ops;
    const int64_t* op_off;
    const uint16_t* text;
    int64_t text_units;
    const int64_t* text_off;
    const mt_props_rec* props;
    int64_t nprops;
    const int64_t* props_off;
    const mt_kv* kv;
    int64_t nkv;
    const int64_t* kv_off;
};

/* host-side shape checks before the kernel trusts any offset */
static bool offsets_ok(const SubmitArgs& a, int64_t nd) {
    if (!a.op_off || !a.text_off || !a.props_off || !a.kv_off || a.text_units < 0 || a.nprops < 0 || a.nkv < 0)
        return false;
    if (a.op_off[0] < 0) return false;
    for (int64_t d = 0; d < nd; d++) {
        if (a.op_off[d] > a.op_off[d + 1] || a.text_off[d] < 0 || a.text_off[d] > a.text_units || a.props_off[d] < 0 ||
            a.props_off[d] > a.nprops || a.kv_off[d] < 0 || a.kv_off[d] > a.nkv)
            return false;
    }
    return !a.op_off[nd] || a.ops;
}

/* every pool reference of every event of documents [d0, d1) in bounds before the kernel dereferences it (in parallel
 * on the host: up to 16 threads, one contiguous range each); also each document's perspective floors
 * (mt_kernels.h persp_refused), whether it holds snapshot-load records, and (text_end) the end of the text the
 * documents reference */
static bool check_docs(const SubmitArgs& a, int64_t d0, int64_t d1, mt_engine::Persp* persp, char* loads,
                       int64_t* text_end) {
    int64_t te = 0;
    for (int64_t d = d0; d < d1; d++) {
        mt_engine::Persp& pp = persp[d];
        const int64_t to = a.text_off[d];
        for (int64_t i = a.op_off[d]; i < a.op_off[d + 1]; i++) {
            const mt_op_rec& o = a.ops[i];
            int kind = o.kind & MT_OP_KIND_MASK;
            if (!(o.kind & MT_OPF_LOCAL)) { /* perspective floors (mt_kernels.h persp_refused) */
                if (kind == MT_OP_RELOAD || kind == MT_OP_COLLAB || kind == MT_OP_APPEND) {
                    if (!(o.kind & MT_OPF_TREE)) loads[d] = 1; /* a snapshot load: the full build */
                    if (o.seq > pp.all) pp.all = o.seq;
                } else if (kind != MT_OP_NOOP && o.client != MT_CLIENT_LOCAL) {
                    pp.note(o.client, o.ref_seq);
                }
            }
            int64_t end = 0;
            if (kind == MT_OP_INSERT || kind == MT_OP_RELOAD || kind == MT_OP_APPEND) {
                /* a segment-bearing record: a known kind, and a document of TextSegments or of SubSequences, not both
                 * (mt_oplog.h MT_SEG_RUN; the kinds its earlier batches inserted are seeded by seed_segk) */
                const int sk = o.seg_kind & 0x7F;
                if (sk > MT_SEG_RUN) return false;
                const bool regen = (o.kind & (MT_OPF_LOCAL | MT_OPF_REGEN)) == (MT_OPF_LOCAL | MT_OPF_REGEN);
                const int32_t len = kind == MT_OP_INSERT ? o.text_len : o.pos2;
                if ((sk == MT_SEG_TEXT || sk == MT_SEG_RUN) && !regen && len > 0) pp.segk |= sk == MT_SEG_TEXT ? 1 : 2;
                if (pp.segk == 3) return false;
            }
            const bool units = (o.seg_kind & 0x7F) == MT_SEG_TEXT || (o.seg_kind & 0x7F) == MT_SEG_RUN;
            if (kind == MT_OP_INSERT && units) end = to + (int64_t)o.text_off + o.text_len;
            if (kind == MT_OP_NOOP && (o.kind & MT_OPF_LOCAL) && o.seg_kind == MT_NOOP_HTLOAD)
                end = to + (int64_t)o.text_off + o.text_len;
            if (o.seg_kind & MT_SEG_RELPOS) end = std::max(end, to + (int64_t)o.text_off + o.text_len + MT_RELPOS_UNITS);
            /* snapshot-load records carry the segment length in pos2 (mt_oplog.h) */
            if ((kind == MT_OP_RELOAD || kind == MT_OP_APPEND) && units) {
                if (o.pos2 < 0) return false;
                end = std::max(end, to + (int64_t)o.text_off + o.pos2);
            }
            if (end > a.text_units) return false;
            te = std::max(te, end);
            if (o.props) {
                if (a.props_off[d] + (int64_t)o.props > a.nprops) return false;
                const mt_props_rec& pr = a.props[a.props_off[d] + o.props - 1];
                if (a.kv_off[d] + (int64_t)pr.kv_off + pr.nkv > a.nkv) return false;
            }
        }
    }
    if (text_end) *text_end = te;
    return true;
}

static int host_threads() {
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::min<unsigned>(16, std::max<unsigned>(1, hc));
}

/* the segment kinds the staged documents' replicas already hold (an incremental batch; a reset clears them) */
static void seed_segk(const mt_engine* e, std::vector<mt_engine::Persp>& persp, const int64_t* docs) {
    for (size_t k = 0; k < persp.size(); k++) {
        size_t d = docs ? (size_t)docs[k] : k;
        persp[k].segk = !e->fresh && d < e->persp_applied.size() ? e->persp_applied[d].segk : 0;
    }
}

static bool check_range(const SubmitArgs& a, int64_t d0, int64_t d1, mt_engine::Persp* persp, char* loads,
                        int64_t* text_end) {
    int64_t nops = a.op_off[d1] - a.op_off[d0];
    int nth = nops > (1 << 20) ? host_threads() : 1;
    if (nth <= 1 || d1 - d0 < 2) return check_docs(a, d0, d1, persp, loads, text_end);
    nth = (int)std::min<int64_t>(nth, d1 - d0);
    std::vector<std::thread> th;
    std::vector<char> ok((size_t)nth, 1);
    std::vector<int64_t> te((size_t)nth, 0);
    for (int t = 0; t < nth; t++)
        th.emplace_back([&, t] {
            ok[(size_t)t] = check_docs(a, d0 + (d1 - d0) * t / nth, d0 + (d1 - d0) * (t + 1) / nth, persp, loads,
                                       &te[(size_t)t]);
        });
    for (auto& x : th) x.join();
    for (char c : ok)
        if (!c) return false;
    if (text_end) *text_end = *std::max_element(te.begin(), te.end());
    return true;
}

static int32_t ensure_staging(mt_engine* e, const SubmitArgs& a, int64_t nd = -1) {
    if (nd < 0) nd = e->ndocs; /* staged entries */
    int64_t nops = a.op_off[nd];
    int32_t rc;
    if ((rc = ensure(e, e->ops_buf, sizeof(mt_op_rec) * nops))) return rc;
    if ((rc = ensure(e, e->op_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->text, 2 * a.text_units))) return rc;
    if ((rc = ensure(e, e->text_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->props, sizeof(mt_props_rec) * a.nprops))) return rc;
    if ((rc = ensure(e, e->props_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->kv, sizeof(mt_kv) * a.nkv))) return rc;
    return ensure(e, e->kv_off, sizeof(int64_t) * (nd + 1));
}

/* the offsets and the property pools (small next to the records and the text) */
static int32_t copy_small(mt_engine* e, const SubmitArgs& a, hipStream_t s, int64_t nd = -1) {
    if (nd < 0) nd = e->ndocs; /* staged entries */
    HIPCHK(e, hipMemcpyAsync(e->op_off.p, a.op_off, sizeof(int64_t) * (nd + 1), hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->text_off.p, a.text_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, s));
    if (a.nprops) HIPCHK(e, hipMemcpyAsync(e->props.p, a.props, sizeof(mt_props_rec) * a.nprops, hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->props_off.p, a.props_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, s));
    if (a.nkv) HIPCHK(e, hipMemcpyAsync(e->kv.p, a.kv, sizeof(mt_kv) * a.nkv, hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->kv_off.p, a.kv_off, sizeof(int64_t) * nd, hipMemcpyHostToDevice, s));
    return MT_OK;
}

/* the host copies of a staged batch's offsets, floors and load flag */
static void keep_staged(mt_engine* e, const SubmitArgs& a, std::vector<mt_engine::Persp>& persp,
                        const std::vector<char>& loads) {
    int64_t nd = (int64_t)persp.size(); /* staged entries: every document, or the listed ones (mt_engine_submit_docs) */
    e->h_op_off.assign(a.op_off, a.op_off + nd + 1);
    e->h_text_off.assign(a.text_off, a.text_off + nd);
    e->h_props_off.assign(a.props_off, a.props_off + nd);
    e->h_kv_off.assign(a.kv_off, a.kv_off + nd);
    e->persp_staged.swap(persp);
    e->loads = std::find(loads.begin(), loads.end(), 1) != loads.end();
    e->staged = true;
}

static bool host_pinned(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    hipError_t st = hipPointerGetAttributes(&at, p);
    if (st != hipSuccess) {
        (void)hipGetLastError(); /* pageable memory is an error here, not a sticky one */
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

/* n bytes from host `src` to device `dst` on the copy stream: directly (pinned memory, or a single chunk), or through the engine's
 * pinned staging buffers (host threads fill one while the DMA engine drains the others) */
static constexpr size_t PIN_BYTES = (size_t)128 << 20;
static int32_t stage_h2d(mt_engine* e, void* dst, const void* src, size_t n, bool pinned) {
    if (!n) return MT_OK;
    if (pinned) {
        HIPCHK(e, hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, e->cstream));
        return MT_OK;
    }
    uint8_t* d = (uint8_t*)dst;
    const uint8_t* s = (const uint8_t*)src;
    while (n) {
        mt_engine::Pin& b = e->pin[e->pin_i];
        e->pin_i = (e->pin_i + 1) % mt_engine::NPIN;
        if (!b.p) {
            HIPCHK(e, hipHostMalloc(&b.p, PIN_BYTES, hipHostMallocDefault));
            HIPCHK(e, hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
        } else {
            HIPCHK(e, hipEventSynchronize(b.ev)); /* its previous copy has left it */
        }
        size_t m = std::min(n, PIN_BYTES);
        int nth = m >= ((size_t)8 << 20) ? std::min(8, host_threads()) : 1;
        if (nth <= 1) {
            memcpy(b.p, s, m);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < nth; t++)
                th.emplace_back([&, t] {
                    size_t lo = (m * t / nth) & ~(size_t)63, hi = t + 1 == nth ? m : (m * (t + 1) / nth) & ~(size_t)63;
                    memcpy((uint8_t*)b.p + lo, s + lo, hi - lo);
                });
            for (auto& x : th) x.join();
        }
        HIPCHK(e, hipMemcpyAsync(d, b.p, m, hipMemcpyHostToDevice, e->cstream));
        HIPCHK(e, hipEventRecord(b.ev, e->cstream));
        d += m, s += m, n -= m;
    }
    return MT_OK;
}

extern "C" {

int32_t mt_engine_create(int32_t device, int64_t ndocs, const mt_caps* caps, mt_engine** out) {
    if (!out || !caps || ndocs < 1 || ndocs > (int64_t)0x7fffffff) return MT_E_ARG;
    *out = nullptr;
    Caps k = {caps->acap, caps->mcap, caps->gcap, caps->dcap, caps->rcap, caps->pcap};
    int prof = profile_for(caps->ncap);
    if (!caps_valid(k) || prof < 0 || caps->ccap > 254 || caps->dcap < 0 || caps->rcap < 0 || caps->pcap < 0 ||
        caps->pcap > (1 << 24))
        return MT_E_ARG; /* short ids are bytes; 0xFF = LocalClientId */
    mt_engine* e = new mt_engine();
    e->device = device;
    e->ndocs = ndocs;
    e->dcap = caps->dcap;
    e->rcap = caps->rcap;
    e->pcap = caps->pcap;
    e->fx = caps->dcap > 0 || caps->rcap > 0 || caps->pcap > 0;
    const char* np = getenv("MT_NO_PROMOTE");
    e->promote = !(np && np[0] == '1');
    e->caps0 = *caps;
    e->pro.assign((size_t)ndocs, -1);
    e->profile = prof;
    e->ops = prof == 0 ? ops_small() : prof == 1 ? ops_mid() : prof == 3 ? ops_mat() : prof == 4 ? ops_huge() : ops_big();
    if (hipSetDevice(device) != hipSuccess) {
        delete e;
        return MT_E_HIP;
    }
    /* the small-profile kernel build (mt_prof_small.hip): the hot image in LDS when the batch's documents fit three
     * per CU (1: config 1 0.667 -> 0.691M ops/s, config 3 at 256 / 768 documents +3.0 / +1.5 %, profiles/r06l_ab/);
     * else HBM-resident, 4 waves per SIMD (no VGPR spills) when the documents, one wave each, fit 4 per SIMD (4 SIMDs
     * per CU), 8 otherwise; MT_SMALL_WAVES overrides */
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
    e->waves = ndocs <= (int64_t)ncu * 3 ? 1 : ndocs <= (int64_t)ncu * 4 * 4 ? 4 : 8;
    if (const char* sw = getenv("MT_SMALL_WAVES")) e->waves = atoi(sw) == 1 ? 1 : atoi(sw) == 4 ? 4 : 8;
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
    mt_engine_destroy(e->over);
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->borrowed) e->text.p = e->props.p = e->kv.p = nullptr; /* the parent's */
    DevBuf* bufs[] = {&e->ops_buf, &e->op_off, &e->text, &e->text_off, &e->props,     &e->props_off,
                      &e->kv,     &e->kv_off, &e->tmp,  &e->local_ids, &e->prof, &e->order, &e->sub, &e->vkind};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    if (e->mem) (void)hipFree(e->mem);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->cstream) {
        (void)hipStreamSynchronize(e->cstream);
        (void)hipStreamSynchronize(e->stream2);
        (void)hipStreamDestroy(e->cstream);
        (void)hipStreamDestroy(e->stream2);
        (void)hipEventDestroy(e->evs);
        (void)hipEventDestroy(e->evc);
        (void)hipEventDestroy(e->ev2);
    }
    for (auto& b : e->pin) {
        if (b.p) (void)hipHostFree(b.p);
        if (b.ev) (void)hipEventDestroy(b.ev);
    }
    delete e;
}

const char* mt_engine_last_error(const mt_engine* e) { return e ? e->err.c_str() : "null engine"; }
int64_t mt_engine_ndocs(const mt_engine* e) { return e ? e->ndocs : 0; }
void* mt_engine_stream(const mt_engine* e) { return e ? (void*)e->stream : nullptr; }
float mt_engine_last_run_ms(const mt_engine* e) { return e ? e->last_ms : 0.f; }

int32_t mt_engine_start_collab(mt_engine* e, const int32_t* local_long_ids, int32_t min_seq, int32_t cur_seq) {
    if (!e || !local_long_ids) return MT_E_ARG;
    std::vector<int32_t> mins((size_t)e->ndocs, min_seq), curs((size_t)e->ndocs, cur_seq);
    return mt_engine_start_collab_docs(e, local_long_ids, mins.data(), curs.data());
}

int32_t mt_engine_start_collab_docs(mt_engine* e, const int32_t* local_long_ids, const int32_t* min_seqs,
                                    const int32_t* cur_seqs) {
    if (!e || !local_long_ids || !min_seqs || !cur_seqs) return MT_E_ARG;
    int64_t nd = e->ndocs;
    HIPCHK(e, hipSetDevice(e->device));
    e->h_local.assign(local_long_ids, local_long_ids + nd);
    e->h_local.insert(e->h_local.end(), min_seqs, min_seqs + nd);
    e->h_local.insert(e->h_local.end(), cur_seqs, cur_seqs + nd);
    int32_t rc = ensure(e, e->local_ids, sizeof(int32_t) * 3 * nd);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(e->local_ids.p, e->h_local.data(), sizeof(int32_t) * 3 * nd, hipMemcpyHostToDevice,
                             e->stream));
    e->collab = true;
    rc = e->ops->start_collab(e);
    if (rc) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->over && !e->pro_docs.empty()) { /* promoted documents live in `over` */
        size_t m = e->pro_docs.size();
        std::vector<int32_t> ids(m), mn(m), cu(m);
        for (size_t i = 0; i < m; i++) {
            int64_t d = e->pro_docs[i];
            ids[i] = local_long_ids[d];
            mn[i] = min_seqs[d];
            cu[i] = cur_seqs[d];
        }
        return mt_engine_start_collab_docs(e->over, ids.data(), mn.data(), cu.data());
    }
    return MT_OK;
}

int32_t mt_engine_submit(mt_engine* e, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                         int64_t text_units, const int64_t* text_off, const mt_props_rec* props, int64_t nprops,
                         const int64_t* props_off, const mt_kv* kv, int64_t nkv, const int64_t* kv_off) {
    if (!e) return MT_E_ARG;
    const SubmitArgs a{ops, op_off, text, text_units, text_off, props, nprops, props_off, kv, nkv, kv_off};
    if (!offsets_ok(a, e->ndocs)) return MT_E_ARG;
    int64_t nd = e->ndocs;
    int64_t nops = op_off[nd];
    std::vector<mt_engine::Persp> persp((size_t)nd);
    std::vector<char> loads((size_t)nd, 0);
    seed_segk(e, persp, nullptr);
    if (!check_range(a, 0, nd, persp.data(), loads.data(), nullptr)) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc;
    if ((rc = ensure_staging(e, a))) return rc;
    e->nsub = -1;
    e->h_sub.clear();
    if (nops) HIPCHK(e, hipMemcpyAsync(e->ops_buf.p, ops, sizeof(mt_op_rec) * nops, hipMemcpyHostToDevice, e->stream));
    if (text_units) HIPCHK(e, hipMemcpyAsync(e->text.p, text, 2 * text_units, hipMemcpyHostToDevice, e->stream));
    if ((rc = copy_small(e, a, e->stream))) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    keep_staged(e, a, persp, loads);
    return MT_OK;
}

int32_t mt_engine_submit_docs(mt_engine* e, int64_t m, const int64_t* docs, const mt_op_rec* ops, const int64_t* op_off,
                              const uint16_t* text, int64_t text_units, const int64_t* text_off,
                              const mt_props_rec* props, int64_t nprops, const int64_t* props_off, const mt_kv* kv,
                              int64_t nkv, const int64_t* kv_off) {
    if (!e || m < 0 || m > e->ndocs || (m && !docs)) return MT_E_ARG;
    for (int64_t k = 0; k < m; k++)
        if (docs[k] < 0 || docs[k] >= e->ndocs || (k && docs[k] <= docs[k - 1])) return MT_E_ARG; /* increasing ids */
    const SubmitArgs a{ops, op_off, text, text_units, text_off, props, nprops, props_off, kv, nkv, kv_off};
    if (!offsets_ok(a, m)) return MT_E_ARG;
    std::vector<mt_engine::Persp> persp((size_t)m);
    std::vector<char> loads((size_t)m, 0);
    seed_segk(e, persp, docs);
    if (!check_range(a, 0, m, persp.data(), loads.data(), nullptr)) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc;
    if ((rc = ensure_staging(e, a, m))) return rc;
    if ((rc = ensure(e, e->sub, sizeof(int32_t) * (size_t)std::max<int64_t>(m, 1)))) return rc;
    e->h_sub.assign(docs, docs + m);
    std::vector<int32_t> ids(docs, docs + m);
    int64_t nops = op_off[m];
    if (nops) HIPCHK(e, hipMemcpyAsync(e->ops_buf.p, ops, sizeof(mt_op_rec) * nops, hipMemcpyHostToDevice, e->stream));
    if (text_units) HIPCHK(e, hipMemcpyAsync(e->text.p, text, 2 * text_units, hipMemcpyHostToDevice, e->stream));
    if (m) HIPCHK(e, hipMemcpyAsync(e->sub.p, ids.data(), sizeof(int32_t) * m, hipMemcpyHostToDevice, e->stream));
    if ((rc = copy_small(e, a, e->stream, m))) return rc;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->nsub = m;
    keep_staged(e, a, persp, loads);
    return MT_OK;
}

int32_t mt_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes < 0) return MT_E_ARG;
    *out = nullptr;
    if (hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return MT_E_NOMEM;
    }
    return MT_OK;
}
void mt_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int32_t mt_engine_reset(mt_engine* e) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    std::fill(e->pro.begin(), e->pro.end(), -1);
    e->pro_docs.clear();
    e->fresh = true;
    return launch_init(e);
}

static int32_t stage_subset(mt_engine* e, mt_engine* o);

static int32_t after_launch(mt_engine* e);

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
    return after_launch(e);
}

/* documents per chunk of mt_engine_submit_run: an eighth of the batch, but never fewer than the documents the GPU
 * holds at once (a chunk's launch must fill the machine by itself; config 4's 256 documents stay one launch) */
static int64_t chunk_docs(const mt_engine* e) {
    if (e->chunk > 0) return e->chunk;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || ncu < 1) ncu = 256;
    int64_t resident = e->profile == 4                      ? ncu
                       : e->profile == 0 && e->waves == 1 ? (int64_t)ncu * 3 /* the LDS-image build */
                                                          : (int64_t)ncu * 4 * (e->profile == 0 ? e->waves : 7);
    return std::max<int64_t>(resident, (e->ndocs + 7) / 8);
}

int32_t mt_engine_submit_run(mt_engine* e, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                             int64_t text_units, const int64_t* text_off, const mt_props_rec* props, int64_t nprops,
                             const int64_t* props_off, const mt_kv* kv, int64_t nkv, const int64_t* kv_off) {
    if (!e) return MT_E_ARG;
    const SubmitArgs a{ops, op_off, text, text_units, text_off, props, nprops, props_off, kv, nkv, kv_off};
    if (!offsets_ok(a, e->ndocs)) return MT_E_ARG;
    const int64_t nd = e->ndocs;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc;
    if ((rc = ensure_staging(e, a))) return rc;
#ifdef MT_PROF
    if (ensure(e, e->prof, sizeof(uint64_t) * PH_N * e->ndocs)) return MT_E_NOMEM;
#endif
    if (!e->cstream) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->cstream, hipStreamNonBlocking));
        HIPCHK(e, hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
        HIPCHK(e, hipEventCreateWithFlags(&e->evs, hipEventDisableTiming));
        HIPCHK(e, hipEventCreateWithFlags(&e->evc, hipEventDisableTiming));
        HIPCHK(e, hipEventCreateWithFlags(&e->ev2, hipEventDisableTiming));
    }
    e->staged = false;
    e->nsub = -1;
    e->h_sub.clear();
    /* everything queued on the engine stream so far (a reset, the last replay reading the buffers about to be
     * overwritten) comes first, for the copies and both compute streams */
    HIPCHK(e, hipEventRecord(e->evs, e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->cstream, e->evs, 0));
    HIPCHK(e, hipStreamWaitEvent(e->stream2, e->evs, 0));
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    if ((rc = copy_small(e, a, e->cstream))) return rc;
    const int64_t step = e->order.p ? nd : chunk_docs(e); /* a dispatch order permutes across chunks: one launch */
    /* one chunk leaves nothing to overlap: the runtime's own pageable copy then beats the staging buffers (8,192
     * documents: 66 vs 105 ms, profiles/r06z_c3_share0of8_8192docs_bench.json) */
    const bool single = step >= nd;
    const bool pin_ops = single || host_pinned(ops), pin_text = single || host_pinned(text);
    std::vector<mt_engine::Persp> persp((size_t)nd);
    std::vector<char> loads((size_t)nd, 0);
    seed_segk(e, persp, nullptr);
    int64_t text_hi = 0; /* the text staged so far: a prefix of the pool */
    int k = 0;
    rc = MT_OK;
    /* the first chunks ramp up (a quarter, then half a chunk): the replay starts once a quarter of the first chunk is
     * copied instead of all of it, and the later, full chunks overlap the copies as before */
    static const int ramp_env = getenv("MT_SUBMIT_RAMP") ? atoi(getenv("MT_SUBMIT_RAMP")) : 1;
    const bool ramp = ramp_env != 0 && !single && e->chunk <= 0;
    int64_t len = step;
    for (int64_t d0 = 0; d0 < nd; d0 += len, k++) {
        len = ramp && k < 2 ? std::max<int64_t>(1, step >> (2 - k)) : step;
        const int64_t d1 = std::min(nd, d0 + len);
        int64_t te = 0;
        if (!check_range(a, d0, d1, persp.data(), loads.data(), &te)) {
            rc = MT_E_ARG;
            break;
        }
        if (te > text_hi) {
            if ((rc = stage_h2d(e, (uint16_t*)e->text.p + text_hi, text + text_hi, 2 * (size_t)(te - text_hi), pin_text)))
                break;
            text_hi = te;
        }
        if ((rc = stage_h2d(e, (mt_op_rec*)e->ops_buf.p + op_off[d0], ops + op_off[d0],
                            sizeof(mt_op_rec) * (size_t)(op_off[d1] - op_off[d0]), pin_ops)))
            break;
        HIPCHK(e, hipEventRecord(e->evc, e->cstream));
        hipStream_t s = (k & 1) ? e->stream2 : e->stream;
        HIPCHK(e, hipStreamWaitEvent(s, e->evc, 0));
        e->loads = std::find(loads.begin() + d0, loads.begin() + d1, 1) != loads.begin() + d1;
        e->run_d0 = d0, e->run_n = d1 - d0, e->run_stream = s;
        rc = e->ops->replay(e);
        e->run_d0 = 0, e->run_n = -1, e->run_stream = nullptr;
        if (rc) break;
    }
    /* the second compute stream joins the engine stream; the caller's buffers are free once the copies are done */
    HIPCHK(e, hipEventRecord(e->ev2, e->stream2));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev2, 0));
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->cstream));
    if (rc) {
        (void)hipStreamSynchronize(e->stream); /* the chunks launched before the failure have replayed */
        return rc;
    }
    keep_staged(e, a, persp, loads);
    return after_launch(e);
}

/* the bookkeeping after a replay launch (mt_engine_run, mt_engine_submit_run) */
static int32_t after_launch(mt_engine* e) {
    int32_t rc;
    e->ran = true;
    e->ran_fresh = e->fresh;
    if (e->fresh) e->persp_applied.assign((size_t)e->ndocs, mt_engine::Persp());
    for (size_t k = 0; k < e->persp_staged.size(); k++) {
        size_t d = e->nsub >= 0 ? (size_t)e->h_sub[k] : k;
        if (d < e->persp_applied.size()) e->persp_applied[d].merge(e->persp_staged[k]);
    }
    e->fresh = false;
    e->forwarded = false;
    /* documents promoted by an earlier replay of this replica history live on in `over`: their parent
     * replicas stay latched (E_CAPACITY, every later record a no-op), so this batch's records for them
     * replay there, on top of the state they already hold (no reset) */
    if (e->over && !e->pro_docs.empty()) {
        if ((rc = stage_subset(e, e->over))) return rc;
        if ((rc = mt_engine_run(e->over))) return rc;
        e->forwarded = true;
    }
    return MT_OK;
}

static int32_t promote(mt_engine* e);

int32_t mt_engine_sync(mt_engine* e) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->ev0, e->ev1) == hipSuccess) e->last_ms = ms;
    if (e->ran) {
        e->ran = false;
        int32_t rc;
        if (e->forwarded) {
            e->forwarded = false;
            if ((rc = mt_engine_sync(e->over))) return rc;
            e->last_ms += e->over->last_ms;
        } else if (e->promote && e->ran_fresh) {
            /* only a replay that started from create / reset holds each replica's whole history in the staged
             * log; a document that overflows in a later incremental batch keeps E_CAPACITY visible */
            if ((rc = promote(e))) return rc;
            if (e->over && !e->pro_docs.empty()) e->last_ms += e->over->last_ms;
        }
    }
    return MT_OK;
}

static int32_t read_hdr(mt_engine* e, int32_t* err, int32_t* err_op, int32_t* stats4, int64_t* work3,
                        int64_t* times2 = nullptr) {
    HIPCHK(e, hipSetDevice(e->device));
    int64_t n = e->ndocs;
    int32_t rc = ensure(e, e->tmp, (size_t)n * (4 + 4 + 16 + 24 + 16));
    if (rc) return rc;
    int32_t* de = (int32_t*)e->tmp.p;
    int32_t* deo = de + n;
    int32_t* ds = deo + n;
    int64_t* dw = (int64_t*)(ds + 4 * n);
    int64_t* dt = dw + 3 * n;
    rc = e->ops->hdr(e, de, deo, ds, dw, times2 ? dt : nullptr);
    if (rc) return rc;
    if (err) HIPCHK(e, hipMemcpyAsync(err, de, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (err_op) HIPCHK(e, hipMemcpyAsync(err_op, deo, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (stats4) HIPCHK(e, hipMemcpyAsync(stats4, ds, 16 * n, hipMemcpyDeviceToHost, e->stream));
    if (work3) HIPCHK(e, hipMemcpyAsync(work3, dw, 24 * n, hipMemcpyDeviceToHost, e->stream));
    if (times2) HIPCHK(e, hipMemcpyAsync(times2, dt, 16 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

/* ---- capacity promotion ------------------------------------------------------------------------
 * A document whose replay latched E_CAPACITY (row slots, nodes, heap, key slots, text arena, membership
 * log, pending groups) replays again from its staged log, from an empty replica, in an engine of the
 * next profile: small / config-5 -> HotMid (2,048 nodes, 24 key slots) -> HotBig (16,384) -> HotHuge
 * (262,144, tiled), with four times the arena, membership and pending-group capacities. The promoted
 * documents' records are gathered on the device; their text / props / kv pools stay the parent's. */
static int32_t next_ncap(const mt_engine* e) {
    switch (e->profile) {
    case 0: case 3: return HotMid::N;
    case 1: return HotBig::N;
    case 2: return HotHuge::N;
    case 4: return e->fx || e->wide ? -1 : HotHuge::N; /* the tiled kernel's LDS heap -> its wide variant */
    default: return -1;
    }
}
extern "C++" {
template <class T>
static void scatter(T* dst, const std::vector<T>& src, const std::vector<int64_t>& docs, int k) {
    for (size_t i = 0; i < docs.size(); i++)
        for (int j = 0; j < k; j++) dst[docs[i] * k + j] = src[i * k + j];
}
}
/* stage, in `o`, the records `e` has staged for its promoted documents (e->pro_docs, in order), gathered
 * device to device; their text / props / kv pools stay the parent's */
/* the staged entry holding document d's records (-1: none staged for it) */
static int64_t staged_entry(const mt_engine* e, int64_t d) {
    if (e->nsub < 0) return d;
    auto it = std::lower_bound(e->h_sub.begin(), e->h_sub.end(), d);
    return it != e->h_sub.end() && *it == d ? (int64_t)(it - e->h_sub.begin()) : -1;
}
static int32_t stage_subset(mt_engine* e, mt_engine* o) {
    int64_t m = (int64_t)e->pro_docs.size();
    int32_t rc;
    o->h_op_off.assign((size_t)m + 1, 0);
    o->h_text_off.resize((size_t)m);
    o->h_props_off.resize((size_t)m);
    o->h_kv_off.resize((size_t)m);
    o->nsub = -1;
    std::vector<int64_t> src((size_t)m);
    for (int64_t i = 0; i < m; i++) {
        int64_t k = staged_entry(e, e->pro_docs[(size_t)i]);
        src[(size_t)i] = k;
        int64_t n = k < 0 ? 0 : e->h_op_off[(size_t)k + 1] - e->h_op_off[(size_t)k];
        o->h_op_off[(size_t)i + 1] = o->h_op_off[(size_t)i] + n;
        o->h_text_off[(size_t)i] = k < 0 ? 0 : e->h_text_off[(size_t)k];
        o->h_props_off[(size_t)i] = k < 0 ? 0 : e->h_props_off[(size_t)k];
        o->h_kv_off[(size_t)i] = k < 0 ? 0 : e->h_kv_off[(size_t)k];
    }
    if ((rc = ensure(o, o->ops_buf, sizeof(mt_op_rec) * o->h_op_off[(size_t)m]))) return rc;
    if ((rc = ensure(o, o->op_off, sizeof(int64_t) * (m + 1)))) return rc;
    if ((rc = ensure(o, o->text_off, sizeof(int64_t) * m))) return rc;
    if ((rc = ensure(o, o->props_off, sizeof(int64_t) * m))) return rc;
    if ((rc = ensure(o, o->kv_off, sizeof(int64_t) * m))) return rc;
    for (int64_t i = 0; i < m; i++) {
        int64_t k = src[(size_t)i], n = o->h_op_off[(size_t)i + 1] - o->h_op_off[(size_t)i];
        if (n)
            HIPCHK(o, hipMemcpyAsync((mt_op_rec*)o->ops_buf.p + o->h_op_off[(size_t)i],
                                     (const mt_op_rec*)e->ops_buf.p + e->h_op_off[(size_t)k], sizeof(mt_op_rec) * n,
                                     hipMemcpyDeviceToDevice, o->stream));
    }
    HIPCHK(o, hipMemcpyAsync(o->op_off.p, o->h_op_off.data(), sizeof(int64_t) * (m + 1), hipMemcpyHostToDevice, o->stream));
    HIPCHK(o, hipMemcpyAsync(o->text_off.p, o->h_text_off.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, o->stream));
    HIPCHK(o, hipMemcpyAsync(o->props_off.p, o->h_props_off.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, o->stream));
    HIPCHK(o, hipMemcpyAsync(o->kv_off.p, o->h_kv_off.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, o->stream));
    o->borrowed = true;
    o->text = e->text;
    o->props = e->props;
    o->kv = e->kv;
    o->staged = true;
    return MT_OK;
}
static int32_t promote(mt_engine* e) {
    std::fill(e->pro.begin(), e->pro.end(), -1);
    e->pro_docs.clear();
    int32_t nc = next_ncap(e);
    if (nc < 0) return MT_OK;
    int64_t nd = e->ndocs;
    std::vector<int32_t> err((size_t)nd);
    int32_t rc = read_hdr(e, err.data(), nullptr, nullptr, nullptr);
    if (rc) return rc;
    for (int64_t d = 0; d < nd; d++)
        if (err[(size_t)d] == MT_E_CAPACITY) e->pro_docs.push_back(d);
    int64_t m = (int64_t)e->pro_docs.size();
    if (m == 0) return MT_OK;
    mt_caps c = e->caps0;
    c.ncap = nc;
    c.hcap = std::max(c.hcap, 2 * nc);
    c.acap = (int32_t)std::min<int64_t>(4 * (int64_t)c.acap, 1 << 23);
    c.mcap = (int32_t)std::min<int64_t>(4 * (int64_t)c.mcap, 1 << 18);
    c.gcap = (int32_t)std::min<int64_t>(4 * (int64_t)c.gcap, 1 << 16);
    /* the client-feature capacities grow too (delta-log words, references, PermutationVector handles),
     * so a document that overflowed one of them is not replayed again into the same limit */
    c.dcap = (int32_t)std::min<int64_t>(4 * (int64_t)c.dcap, 1 << 26);
    c.rcap = (int32_t)std::min<int64_t>(4 * (int64_t)c.rcap, 1 << 16);
    c.pcap = (int32_t)std::min<int64_t>(4 * (int64_t)c.pcap, 1 << 24);
    mt_engine* o = e->over;
    if (o && (o->ndocs != m || o->caps0.ncap != c.ncap)) {
        mt_engine_destroy(o);
        o = e->over = nullptr;
    }
    if (!o) {
        rc = mt_engine_create(e->device, m, &c, &o);
        if (rc) return rc;
        e->over = o;
    }
    o->promote = e->promote;
    o->wide = e->profile == 4; /* HotHuge -> HotHuge: the same layout, the wide kernel */
    if (e->nvk && (rc = mt_engine_set_value_kinds(o, e->h_vkind.data(), e->nvk))) return rc;
    if (e->collab) {
        std::vector<int32_t> loc((size_t)(3 * m)); /* the promoted documents' ids, minSeqs, currentSeqs */
        for (int64_t i = 0; i < m; i++)
            for (int64_t k = 0; k < 3; k++)
                loc[(size_t)(k * m + i)] = e->h_local[(size_t)(k * nd + e->pro_docs[(size_t)i])];
        HIPCHK(o, hipSetDevice(o->device));
        if ((rc = ensure(o, o->local_ids, sizeof(int32_t) * 3 * m))) return rc;
        HIPCHK(o, hipMemcpyAsync(o->local_ids.p, loc.data(), sizeof(int32_t) * 3 * m, hipMemcpyHostToDevice, o->stream));
        HIPCHK(o, hipStreamSynchronize(o->stream));
        o->h_local = loc;
        o->collab = true;
    }
    if ((rc = stage_subset(e, o))) return rc;
    /* an empty replica (create / reset state), the same local ids; then the replay, promoting further */
    if ((rc = mt_engine_reset(o))) return rc;
    if ((rc = mt_engine_run(o))) return rc;
    if ((rc = mt_engine_sync(o))) return rc;
    for (int64_t i = 0; i < m; i++) e->pro[(size_t)e->pro_docs[(size_t)i]] = (int32_t)i;
    return MT_OK;
}
/* the perspective floor of (doc, long client) for the reads (mt_kernels.h persp_refused) */
static int32_t persp_floor(const mt_engine* e, int64_t doc, int32_t long_client) {
    if (long_client < 0 || (size_t)doc >= e->persp_applied.size()) return INT32_MIN;
    return e->persp_applied[(size_t)doc].floor(long_client);
}
/* the engine and index that hold document `doc` (promoted documents live in `over`) */
static mt_engine* route(mt_engine* e, int64_t* doc) {
    while (e && e->over && *doc >= 0 && *doc < e->ndocs && e->pro[(size_t)*doc] >= 0) {
        *doc = e->pro[(size_t)*doc];
        e = e->over;
    }
    return e;
}
static bool promoted(const mt_engine* e) { return e->over && !e->pro_docs.empty(); }

int32_t mt_engine_errors(mt_engine* e, int32_t* err, int32_t* err_op) {
    if (!e) return MT_E_ARG;
    int32_t rc = read_hdr(e, err, err_op, nullptr, nullptr);
    if (rc || !promoted(e)) return rc;
    size_t m = e->pro_docs.size();
    std::vector<int32_t> a(m), b(m);
    if ((rc = mt_engine_errors(e->over, a.data(), b.data()))) return rc;
    if (err) scatter(err, a, e->pro_docs, 1);
    if (err_op) scatter(err_op, b, e->pro_docs, 1);
    return MT_OK;
}
int32_t mt_engine_stats(mt_engine* e, int32_t* out4) {
    if (!e || !out4) return MT_E_ARG;
    int32_t rc = read_hdr(e, nullptr, nullptr, out4, nullptr);
    if (rc || !promoted(e)) return rc;
    std::vector<int32_t> a(4 * e->pro_docs.size());
    if ((rc = mt_engine_stats(e->over, a.data()))) return rc;
    scatter(out4, a, e->pro_docs, 4);
    return MT_OK;
}
int32_t mt_engine_doc_times(mt_engine* e, int64_t* out2) {
    if (!e || !out2) return MT_E_ARG;
    int32_t rc = read_hdr(e, nullptr, nullptr, nullptr, nullptr, out2);
    if (rc || !promoted(e)) return rc;
    std::vector<int64_t> a(2 * e->pro_docs.size());
    if ((rc = mt_engine_doc_times(e->over, a.data()))) return rc;
    scatter(out2, a, e->pro_docs, 2);
    return MT_OK;
}

int32_t mt_engine_set_order(mt_engine* e, const int32_t* order) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    if (!order) {
        if (e->order.p) (void)hipFree(e->order.p);
        e->order = DevBuf();
        return MT_OK;
    }
    std::vector<char> seen((size_t)e->ndocs, 0);
    for (int64_t i = 0; i < e->ndocs; i++) {
        if (order[i] < 0 || order[i] >= e->ndocs || seen[(size_t)order[i]]) return MT_E_ARG; /* a permutation */
        seen[(size_t)order[i]] = 1;
    }
    if (ensure(e, e->order, sizeof(int32_t) * e->ndocs)) return MT_E_NOMEM;
    HIPCHK(e, hipMemcpyAsync(e->order.p, order, sizeof(int32_t) * e->ndocs, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_set_value_kinds(mt_engine* e, const uint8_t* kinds, int32_t n) {
    if (!e || n < 0 || (n && !kinds) || n > MT_VALUE_DERIVED) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->vkind, (size_t)std::max(n, 1));
    if (rc) return rc;
    e->h_vkind.assign(kinds, kinds + n);
    if (n) HIPCHK(e, hipMemcpyAsync(e->vkind.p, kinds, (size_t)n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->nvk = n;
    if (e->over) return mt_engine_set_value_kinds(e->over, kinds, n); /* promoted documents replay there */
    return MT_OK;
}

int32_t mt_engine_set_variant(mt_engine* e, int32_t key, int32_t value) {
    if (!e) return MT_E_ARG;
    switch (key) {
    case MT_VAR_SMALL_WAVES:
        if (value != 1 && value != 4 && value != 8) return MT_E_ARG;
        e->waves = value;
        return MT_OK;
    case MT_VAR_TILED_WIDE:
        if (value != 0 && value != 1) return MT_E_ARG;
        e->wide = value == 1;
        return MT_OK;
    case MT_VAR_CHUNK_DOCS:
        if (value < 0) return MT_E_ARG;
        e->chunk = value;
        return MT_OK;
    default:
        return MT_E_ARG;
    }
}

int32_t mt_engine_work(mt_engine* e, int64_t* out3) {
    if (!e || !out3) return MT_E_ARG;
    int32_t rc = read_hdr(e, nullptr, nullptr, nullptr, out3);
    if (rc || !promoted(e)) return rc;
    std::vector<int64_t> a(3 * e->pro_docs.size());
    if ((rc = mt_engine_work(e->over, a.data()))) return rc;
    scatter(out3, a, e->pro_docs, 3);
    return MT_OK;
}
int64_t mt_engine_promoted(const mt_engine* e, int64_t* docs_out, int64_t cap) {
    if (!e) return -MT_E_ARG;
    int64_t m = promoted(e) ? (int64_t)e->pro_docs.size() : 0;
    for (int64_t i = 0; i < m && i < cap && docs_out; i++) docs_out[i] = e->pro_docs[(size_t)i];
    return m;
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
    if (promoted(e)) {
        std::vector<uint64_t> a(e->pro_docs.size());
        if ((rc = mt_engine_digests(e->over, a.data()))) return rc;
        scatter(out, a, e->pro_docs, 1);
    }
    return MT_OK;
}

int64_t mt_engine_dump(mt_engine* e, int64_t doc, uint8_t* out, int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    e = route(e, &doc);
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
    int32_t floor = persp_floor(e, doc, long_client);
    e = route(e, &doc);
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, 16);
    if (rc) return rc;
    rc = e->ops->length(e, doc, ref_seq, long_client, floor, (int32_t*)e->tmp.p);
    if (rc) return rc;
    int32_t r2[2];
    HIPCHK(e, hipMemcpyAsync(r2, e->tmp.p, sizeof(r2), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (r2[1]) return MT_E_UNSUPPORTED; /* a perspective the reference's partial lengths answer differently */
    *out = r2[0];
    return MT_OK;
}

int64_t mt_engine_get_text(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out,
                           int64_t cap) {
    return mt_engine_get_text_range(e, doc, ref_seq, long_client, nullptr, 0, MT_TEXT_DEFAULT, MT_TEXT_DEFAULT, out,
                                    cap);
}

static int64_t text_read(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, const uint16_t* placeholder,
                         int32_t placeholder_len, int32_t start, int32_t end, uint16_t* out, int64_t cap);

int64_t mt_engine_get_text_range(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client,
                                 const uint16_t* placeholder, int32_t placeholder_len, int32_t start, int32_t end,
                                 uint16_t* out, int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0 || placeholder_len < 0 || placeholder_len > 4096 ||
        (placeholder_len > 0 && !placeholder))
        return -MT_E_ARG;
    if (placeholder_len == 1 && placeholder[0] == '*') return -MT_E_UNSUPPORTED; /* Marker.toString() */
    return text_read(e, doc, ref_seq, long_client, placeholder, placeholder_len, start, end, out, cap);
}

int64_t mt_engine_get_items(mt_engine* e, int64_t doc, int32_t start, int32_t end, uint16_t* out, int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0 || start == MT_TEXT_DEFAULT) return -MT_E_ARG;
    return text_read(e, doc, 0, -1, nullptr, -1, start, end, out, cap); /* placeholder length -1: k_text's items mode */
}

static int64_t text_read(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, const uint16_t* placeholder,
                         int32_t placeholder_len, int32_t start, int32_t end, uint16_t* out, int64_t cap) {
    int32_t floor = persp_floor(e, doc, long_client);
    e = route(e, &doc);
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    size_t phb = (2 * (size_t)(placeholder_len > 0 ? placeholder_len : 0) + 15) & ~(size_t)15;
    if (ensure(e, e->tmp, 16 + phb + 2 * (size_t)(out ? cap : 0) + 16)) return -MT_E_HIP;
    int64_t* dn = (int64_t*)e->tmp.p;
    uint16_t* dph = (uint16_t*)((uint8_t*)e->tmp.p + 16);
    uint16_t* dbuf = out ? (uint16_t*)((uint8_t*)e->tmp.p + 16 + phb) : nullptr;
    if (placeholder_len > 0 &&
        hipMemcpyAsync(dph, placeholder, 2 * (size_t)placeholder_len, hipMemcpyHostToDevice, e->stream) != hipSuccess)
        return -MT_E_HIP;
    int32_t rc = e->ops->text(e, doc, ref_seq, long_client, floor, start, end, dph, placeholder_len, dbuf,
                              out ? cap : 0, dn);
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

static void seg_ref_of(const int32_t* r, mt_seg_ref* out) {
    out->rid = r[0] == 1 ? r[1] : -1;
    out->gen = r[2];
    out->offset = r[3];
    out->length = r[4];
    out->seq = r[5];
    out->client = r[6];
    out->removed_seq = r[7];
    out->removed_client = r[8];
    out->ordinal = r[9];
}
static int32_t seg_query(mt_engine* e, int64_t doc, int32_t mode, int32_t a, int32_t b, int32_t ref_seq,
                         int32_t long_client, int32_t* res7) { /* res7: MT_SEGQ_N words (mt_kernels.h k_seg) */
    if (!e || doc < 0 || doc >= e->ndocs) return MT_E_ARG;
    int32_t floor = persp_floor(e, doc, long_client);
    e = route(e, &doc);
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, 64);
    if (rc) return rc;
    rc = e->ops->seg(e, doc, mode, a, b, ref_seq, long_client, floor, (int32_t*)e->tmp.p);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(res7, e->tmp.p, MT_SEGQ_N * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (res7[0] == 3) return MT_E_UNSUPPORTED; /* a perspective the reference's partial lengths answer differently */
    return MT_OK;
}

int32_t mt_engine_get_containing_segment(mt_engine* e, int64_t doc, int32_t pos, int32_t ref_seq, int32_t long_client,
                                         mt_seg_ref* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 0, pos, 0, ref_seq, long_client, r);
    if (rc) return rc;
    seg_ref_of(r, out);
    return MT_OK;
}

int32_t mt_engine_get_position(mt_engine* e, int64_t doc, int32_t rid, int32_t gen, int32_t ref_seq,
                               int32_t long_client, int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 1, rid, gen, ref_seq, long_client, r);
    if (rc) return rc;
    if (!r[0]) return MT_E_ARG;
    *out = r[1];
    return MT_OK;
}

int32_t mt_engine_pos_from_relative_pos(mt_engine* e, int64_t doc, int32_t id_key, int32_t id_value, int32_t before,
                                        int32_t has_offset, int32_t offset, int32_t ref_seq, int32_t long_client,
                                        int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 2, id_key, id_value, ref_seq, long_client, r);
    if (rc) return rc;
    if (r[0] == 2) return MT_E_UNSUPPORTED; /* several markers hold the id */
    int32_t pos = -1;
    if (r[0] == 1) { /* mergeTree.ts:1986-1996: a marker's cachedLength is 1 */
        pos = r[1];
        if (!before) pos += 1 + (has_offset ? offset : 0);
        else if (has_offset) pos -= offset;
    }
    *out = pos;
    return MT_OK;
}

int32_t mt_engine_resolve_remote_client_position(mt_engine* e, int64_t doc, int32_t pos, int32_t ref_seq,
                                                 int32_t long_client, int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 4, pos, 0, ref_seq, long_client, r);
    if (rc) return rc;
    *out = r[0] == 1 ? r[1] : (pos == r[3] ? r[4] : -1);
    return MT_OK;
}

int32_t mt_engine_adjust_position(mt_engine* e, int64_t doc, int32_t pos, int32_t from_seq, int32_t long_client,
                                  int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 4, pos, 0, from_seq, long_client, r);
    if (rc) return rc;
    *out = r[0] == 1 && !r[2] ? r[1] : -1;
    return MT_OK;
}

int32_t mt_engine_handle_to_position(mt_engine* e, int64_t doc, int32_t handle, int32_t local_seq, int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 6, handle, local_seq, 0, -1, r);
    if (rc) return rc;
    /* assert(localSeq <= collabWindow.localSeq) (client.ts:676) and assert(isHandleValid(containingSegment.start)) */
    if (r[0] != 1) return MT_E_ARG;
    *out = r[1];
    return MT_OK;
}

int32_t mt_engine_get_marker_from_id(mt_engine* e, int64_t doc, int32_t id_key, int32_t id_value, mt_seg_ref* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 5, id_key, id_value, 0, -1, r);
    if (rc) return rc;
    if (r[0] == 2) return MT_E_UNSUPPORTED; /* several markers hold the id, or an annotate changed it */
    seg_ref_of(r, out);
    return MT_OK;
}

int64_t mt_engine_segment_ids(mt_engine* e, int64_t doc, int32_t* out, int64_t cap) {
    if (!e || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    e = route(e, &doc);
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    if (ensure(e, e->tmp, 16 + 8 * (size_t)(out ? cap : 0) + 16)) return -MT_E_HIP;
    int64_t* dn = (int64_t*)e->tmp.p;
    int32_t* dbuf = (int32_t*)((uint8_t*)e->tmp.p + 16);
    int32_t rc = e->ops->segids(e, doc, dbuf, out ? cap : 0, dn);
    if (rc) return -rc;
    int64_t n = 0;
    if (hipMemcpyAsync(&n, dn, sizeof(int64_t), hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    int64_t m = n < cap ? n : cap;
    if (out && m > 0) {
        if (hipMemcpyAsync(out, dbuf, 8 * (size_t)m, hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
        if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    }
    return n;
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
    if (promoted(e)) {
        std::vector<int64_t> a(e->pro_docs.size());
        std::vector<uint64_t> b(e->pro_docs.size());
        int32_t rc = mt_engine_delta_state(e->over, a.data(), b.data());
        if (rc) return rc;
        if (n_out) scatter(n_out, a, e->pro_docs, 1);
        if (hash_out) scatter(hash_out, b, e->pro_docs, 1);
    }
    return MT_OK;
}

int64_t mt_engine_deltas(mt_engine* e, int64_t doc, int32_t* out, int64_t cap) {
    if (!e || e->dcap <= 0 || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    e = route(e, &doc);
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

int32_t mt_engine_doc_error(mt_engine* e, int64_t doc, int32_t* err, int32_t* err_op) {
    if (!e || doc < 0 || doc >= e->ndocs) return MT_E_ARG;
    e = route(e, &doc);
    HIPCHK(e, hipSetDevice(e->device));
    int64_t stride = 0, off = 0;
    delta_geometry(e, &off, &stride); /* the block stride; the header is at the block's start */
    int32_t v[2];
    const uint8_t* h = (const uint8_t*)e->mem + doc * stride + offsetof(DocHdr, err);
    static_assert(offsetof(DocHdr, errOp) == offsetof(DocHdr, err) + 4, "err, errOp adjacent");
    HIPCHK(e, hipMemcpyAsync(v, h, sizeof v, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (err) *err = v[0];
    if (err_op) *err_op = v[1];
    return MT_OK;
}

int32_t mt_engine_ref_capacity(const mt_engine* e) { return e ? e->rcap : 0; }

static void ht_geometry(const mt_engine* e, int64_t* off, int64_t* dl) {
    switch (e->profile) {
    case 0: *off = Doc<HotSmall>::off_ht(e->s0.caps), *dl = Doc<HotSmall>::off_dl(e->s0.caps); break;
    case 1: *off = Doc<HotMid>::off_ht(e->s1.caps), *dl = Doc<HotMid>::off_dl(e->s1.caps); break;
    case 3: *off = Doc<HotMat>::off_ht(e->s3.caps), *dl = Doc<HotMat>::off_dl(e->s3.caps); break;
    case 4: *off = Doc<HotHuge>::off_ht(e->s4.caps), *dl = Doc<HotHuge>::off_dl(e->s4.caps); break;
    default: *off = Doc<HotBig>::off_ht(e->s2.caps), *dl = Doc<HotBig>::off_dl(e->s2.caps); break;
    }
}

int64_t mt_engine_handle_table(mt_engine* e, int64_t doc, int32_t* out, int64_t cap) {
    if (!e || e->pcap <= 0 || doc < 0 || doc >= e->ndocs || cap < 0) return -MT_E_ARG;
    e = route(e, &doc);
    if (hipSetDevice(e->device) != hipSuccess) return -MT_E_HIP;
    int64_t off, dl, stride, o2;
    ht_geometry(e, &off, &dl);
    delta_geometry(e, &o2, &stride);
    const uint8_t* base = (const uint8_t*)e->mem + doc * stride;
    DState st;
    if (hipMemcpyAsync(&st, base + dl, sizeof st, hipMemcpyDeviceToHost, e->stream) != hipSuccess) return -MT_E_HIP;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    int64_t n = st.hlen, m = n < cap ? n : cap;
    if (out && m > 0) {
        if (hipMemcpyAsync(out, base + off, 4 * (size_t)m, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            return -MT_E_HIP;
        if (hipStreamSynchronize(e->stream) != hipSuccess) return -MT_E_HIP;
    }
    return n;
}

int32_t mt_engine_get_handle(mt_engine* e, int64_t doc, int32_t pos, int32_t* out) {
    if (!out) return MT_E_ARG;
    int32_t r[MT_SEGQ_N];
    int32_t rc = seg_query(e, doc, 3, pos, 0, 0, -1, r);
    if (rc) return rc;
    if (!r[0]) return MT_E_ARG; /* RangeError: no segment at pos (ensureRange) */
    *out = r[1];
    return MT_OK;
}

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
    if (promoted(e)) {
        size_t m = e->pro_docs.size();
        std::vector<int32_t> a(m), b(m * (size_t)e->rcap);
        if ((rc = mt_engine_ref_positions(e->over, a.data(), b.data()))) return rc;
        if (nref_out) scatter(nref_out, a, e->pro_docs, 1);
        if (pos_out) scatter(pos_out, b, e->pro_docs, e->rcap);
    }
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
