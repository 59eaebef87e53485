/*
 * mt_replay.hip — CDNA4 (gfx950) replay kernels and the C ABI of include/mt_engine.h.
 *
 * One 64-lane wavefront replays one document: control flow is wave-uniform, and the
 * data-parallel parts of every op — the perspective prefix scan that replaces the reference's
 * root-to-leaf walk (mergeTree.ts:2378-2507, nodeLength 1692-1732), range marking
 * (nodeMap 2936-2998), stable-id lookup and text copies — run across the 64 lanes with
 * DPP/permute shuffles and 64-bit ballots (mt_wave.h). Documents are independent, so the grid
 * is one workgroup per document and the machine is filled by documents.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/mt_engine.h"
#include "mt_core.h"
#include "mt_store.h"
#include "mt_wave.h"

using namespace mt;

#define WG 64

__global__ __launch_bounds__(WG) void k_init(Cols c, Caps k, int64_t ndocs) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU> r(doc_view(c, k, d), WaveGPU());
    r.init();
}

__global__ __launch_bounds__(WG) void k_start_collab(Cols c, Caps k, int64_t ndocs, const int32_t* local_long,
                                                    int32_t min_seq, int32_t cur_seq) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU> r(doc_view(c, k, d), WaveGPU());
    r.start_collab(local_long[d], min_seq, cur_seq);
}

/* K1-K4 fused: the whole event stream of a document, one wave per document. */
__global__ __launch_bounds__(WG) void k_replay(Cols c, Caps k, int64_t ndocs, const mt_op_rec* ops,
                                              const int64_t* op_off, const uint16_t* text, const int64_t* text_off,
                                              const mt_props_rec* props, const int64_t* props_off, const mt_kv* kv,
                                              const int64_t* kv_off) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU> r(doc_view(c, k, d), WaveGPU());
    Pools p;
    p.ops = ops + op_off[d];
    p.nops = op_off[d + 1] - op_off[d];
    p.text = text + text_off[d];
    p.props = props + props_off[d];
    p.kv = kv + kv_off[d];
    r.replay(p);
}

/* K5: per-doc digest of the canonical dump */
__global__ __launch_bounds__(WG) void k_digest(Cols c, Caps k, int64_t ndocs, uint64_t* out) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU> r(doc_view(c, k, d), WaveGPU());
    uint64_t h = r.digest();
    if (threadIdx.x == 0) out[d] = h;
}

__global__ __launch_bounds__(WG) void k_dump(Cols c, Caps k, int64_t doc, uint8_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU> r(doc_view(c, k, doc), WaveGPU());
    int64_t m = r.dump(out, cap);
    if (threadIdx.x == 0) *n = m;
}

__global__ __launch_bounds__(WG) void k_length(Cols c, Caps k, int64_t doc, int32_t ref_seq, int32_t long_client,
                                              int32_t* out) {
    Replica<WaveGPU> r(doc_view(c, k, doc), WaveGPU());
    int32_t v;
    if (long_client < 0) {
        v = r.length_local();
    } else {
        int32_t sh = r.short_of(long_client);
        v = r.length(ref_seq, sh < 0 ? 0x7fff : sh);
    }
    if (threadIdx.x == 0) *out = v;
}

__global__ __launch_bounds__(WG) void k_text(Cols c, Caps k, int64_t doc, int32_t ref_seq, int32_t long_client,
                                            uint16_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU> r(doc_view(c, k, doc), WaveGPU());
    int32_t sh;
    if (long_client < 0) {
        sh = r.d.h->localShort;
        ref_seq = r.d.h->currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff;
    }
    int64_t m = r.get_text(ref_seq, sh, out, cap);
    if (threadIdx.x == 0) *n = m;
}

/* per-doc (seqOps, sumR, sumW) for the roofline accounting */
__global__ void k_work(const DocHdr* h, int64_t ndocs, int64_t* out3) {
    int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndocs) return;
    out3[3 * d + 0] = h[d].seqOps;
    out3[3 * d + 1] = h[d].sumR;
    out3[3 * d + 2] = h[d].sumW;
}

__global__ void k_errors(const DocHdr* h, int64_t ndocs, int32_t* err, int32_t* err_op, int32_t* stats4) {
    int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndocs) return;
    if (err) err[d] = h[d].err;
    if (err_op) err_op[d] = h[d].errOp;
    if (stats4) {
        stats4[4 * d + 0] = h[d].nleaf;
        stats4[4 * d + 1] = h[d].hwSlots;
        stats4[4 * d + 2] = h[d].hwHeap;
        stats4[4 * d + 3] = h[d].opsDone;
    }
}

/* ------------------------------------------------------------------------------------------
 * engine (host side)
 * ---------------------------------------------------------------------------------------- */
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct mt_engine {
    int device;
    int64_t ndocs;
    Caps k;
    Cols c;
    void* mem = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    bool staged = false;
    DevBuf ops, op_off, text, text_off, props, props_off, kv, kv_off, tmp, local_ids;
    int32_t min_seq0 = 0, cur_seq0 = 0;
    bool collab = false;
    std::string err;
};

static int32_t hip_fail(mt_engine* e, hipError_t st, const char* what) {
    if (e) e->err = std::string(what) + ": " + hipGetErrorString(st);
    return MT_E_HIP;
}
#define HIPCHK(e, x)                                     \
    do {                                                 \
        hipError_t st_ = (x);                            \
        if (st_ != hipSuccess) return hip_fail(e, st_, #x); \
    } while (0)

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

static int32_t launch_check(mt_engine* e, const char* what) {
    hipError_t st = hipGetLastError();
    if (st != hipSuccess) return hip_fail(e, st, what);
    return MT_OK;
}

extern "C" {

int32_t mt_engine_create(int32_t device, int64_t ndocs, const mt_caps* caps, mt_engine** out) {
    if (!out || !caps || ndocs < 1 || ndocs > (int64_t)0x7fffffff) return MT_E_ARG;
    *out = nullptr;
    Caps k = {caps->ncap, caps->hcap, caps->acap, caps->mcap, caps->gcap, caps->ccap};
    if (!caps_valid(k)) return MT_E_ARG;
    mt_engine* e = new mt_engine();
    e->device = device;
    e->ndocs = ndocs;
    e->k = k;
    hipError_t st = hipSetDevice(device);
    if (st != hipSuccess) {
        delete e;
        return MT_E_HIP;
    }
    size_t bytes = layout(e->c, k, ndocs, nullptr);
    st = hipMalloc(&e->mem, bytes);
    if (st != hipSuccess) {
        delete e;
        return MT_E_NOMEM;
    }
    layout(e->c, k, ndocs, (uint8_t*)e->mem);
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_E_HIP;
    }
    hipLaunchKernelGGL(k_init, dim3((unsigned)ndocs), dim3(WG), 0, e->stream, e->c, k, ndocs);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess) {
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
    DevBuf* bufs[] = {&e->ops,   &e->op_off, &e->text, &e->text_off, &e->props,
                      &e->props_off, &e->kv, &e->kv_off, &e->tmp, &e->local_ids};
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
    hipLaunchKernelGGL(k_start_collab, dim3((unsigned)e->ndocs), dim3(WG), 0, e->stream, e->c, e->k, e->ndocs,
                       (const int32_t*)e->local_ids.p, min_seq, cur_seq);
    if ((rc = launch_check(e, "k_start_collab"))) return rc;
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
    /* every pool reference of every event must be in bounds before the kernel dereferences it */
    for (int64_t d = 0; d < nd; d++) {
        for (int64_t i = op_off[d]; i < op_off[d + 1]; i++) {
            const mt_op_rec& o = ops[i];
            int kind = o.kind & MT_OP_KIND_MASK;
            if (kind == MT_OP_INSERT && o.seg_kind == MT_SEG_TEXT &&
                text_off[d] + (int64_t)o.text_off + o.text_len > text_units)
                return MT_E_ARG;
            if (o.props) {
                if (props_off[d] + (int64_t)o.props > nprops) return MT_E_ARG;
                const mt_props_rec& pr = props[props_off[d] + o.props - 1];
                if (kv_off[d] + (int64_t)pr.kv_off + pr.nkv > nkv) return MT_E_ARG;
            }
        }
    }
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc;
    if ((rc = ensure(e, e->ops, sizeof(mt_op_rec) * nops))) return rc;
    if ((rc = ensure(e, e->op_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->text, 2 * text_units))) return rc;
    if ((rc = ensure(e, e->text_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->props, sizeof(mt_props_rec) * nprops))) return rc;
    if ((rc = ensure(e, e->props_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if ((rc = ensure(e, e->kv, sizeof(mt_kv) * nkv))) return rc;
    if ((rc = ensure(e, e->kv_off, sizeof(int64_t) * (nd + 1)))) return rc;
    if (nops) HIPCHK(e, hipMemcpyAsync(e->ops.p, ops, sizeof(mt_op_rec) * nops, hipMemcpyHostToDevice, e->stream));
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
    hipLaunchKernelGGL(k_init, dim3((unsigned)e->ndocs), dim3(WG), 0, e->stream, e->c, e->k, e->ndocs);
    int32_t rc = launch_check(e, "k_init");
    if (rc) return rc;
    if (e->collab) {
        hipLaunchKernelGGL(k_start_collab, dim3((unsigned)e->ndocs), dim3(WG), 0, e->stream, e->c, e->k, e->ndocs,
                           (const int32_t*)e->local_ids.p, e->min_seq0, e->cur_seq0);
        if ((rc = launch_check(e, "k_start_collab"))) return rc;
    }
    return MT_OK;
}

int32_t mt_engine_work(mt_engine* e, int64_t* out3) {
    if (!e || !out3) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, sizeof(int64_t) * 3 * e->ndocs);
    if (rc) return rc;
    hipLaunchKernelGGL(k_work, dim3((unsigned)((e->ndocs + 255) / 256)), dim3(256), 0, e->stream, e->c.hdr, e->ndocs,
                       (int64_t*)e->tmp.p);
    if ((rc = launch_check(e, "k_work"))) return rc;
    HIPCHK(e, hipMemcpyAsync(out3, e->tmp.p, sizeof(int64_t) * 3 * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_run(mt_engine* e) {
    if (!e || !e->staged) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    hipLaunchKernelGGL(k_replay, dim3((unsigned)e->ndocs), dim3(WG), 0, e->stream, e->c, e->k, e->ndocs,
                       (const mt_op_rec*)e->ops.p, (const int64_t*)e->op_off.p, (const uint16_t*)e->text.p,
                       (const int64_t*)e->text_off.p, (const mt_props_rec*)e->props.p,
                       (const int64_t*)e->props_off.p, (const mt_kv*)e->kv.p, (const int64_t*)e->kv_off.p);
    int32_t rc = launch_check(e, "k_replay");
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

int32_t mt_engine_errors(mt_engine* e, int32_t* err, int32_t* err_op) {
    if (!e) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, sizeof(int32_t) * 2 * e->ndocs);
    if (rc) return rc;
    int32_t* de = (int32_t*)e->tmp.p;
    int32_t* deo = de + e->ndocs;
    hipLaunchKernelGGL(k_errors, dim3((unsigned)((e->ndocs + 255) / 256)), dim3(256), 0, e->stream, e->c.hdr,
                       e->ndocs, de, deo, (int32_t*)nullptr);
    if ((rc = launch_check(e, "k_errors"))) return rc;
    if (err) HIPCHK(e, hipMemcpyAsync(err, de, sizeof(int32_t) * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    if (err_op) HIPCHK(e, hipMemcpyAsync(err_op, deo, sizeof(int32_t) * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_stats(mt_engine* e, int32_t* out4) {
    if (!e || !out4) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, sizeof(int32_t) * 4 * e->ndocs);
    if (rc) return rc;
    hipLaunchKernelGGL(k_errors, dim3((unsigned)((e->ndocs + 255) / 256)), dim3(256), 0, e->stream, e->c.hdr,
                       e->ndocs, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)e->tmp.p);
    if ((rc = launch_check(e, "k_errors"))) return rc;
    HIPCHK(e, hipMemcpyAsync(out4, e->tmp.p, sizeof(int32_t) * 4 * e->ndocs, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MT_OK;
}

int32_t mt_engine_digests(mt_engine* e, uint64_t* out) {
    if (!e || !out) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    int32_t rc = ensure(e, e->tmp, sizeof(uint64_t) * e->ndocs);
    if (rc) return rc;
    hipLaunchKernelGGL(k_digest, dim3((unsigned)e->ndocs), dim3(WG), 0, e->stream, e->c, e->k, e->ndocs,
                       (uint64_t*)e->tmp.p);
    if ((rc = launch_check(e, "k_digest"))) return rc;
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
    hipLaunchKernelGGL(k_dump, dim3(1), dim3(WG), 0, e->stream, e->c, e->k, doc, dbuf, out ? cap : 0, dn);
    if (launch_check(e, "k_dump")) return -MT_E_HIP;
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
    hipLaunchKernelGGL(k_length, dim3(1), dim3(WG), 0, e->stream, e->c, e->k, doc, ref_seq, long_client,
                       (int32_t*)e->tmp.p);
    if ((rc = launch_check(e, "k_length"))) return rc;
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
    hipLaunchKernelGGL(k_text, dim3(1), dim3(WG), 0, e->stream, e->c, e->k, doc, ref_seq, long_client, dbuf,
                       out ? cap : 0, dn);
    if (launch_check(e, "k_text")) return -MT_E_HIP;
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

} /* extern "C" */
