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
#include <tuple>
#include <type_traits>
#include <vector>

#include "../../include/mt_engine.h"
#include "mt_core.h"
#include "mt_store.h"
#include "mt_wave.h"

using namespace mt;

#define WG 64

template <class HT>
__global__ __launch_bounds__(WG) void k_init(Store<HT> st, int64_t ndocs) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    r.init();
    r.commit();
}

template <class HT>
__global__ __launch_bounds__(WG) void k_start_collab(Store<HT> st, int64_t ndocs, const int32_t* local_long,
                                                    int32_t min_seq, int32_t cur_seq) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    r.start_collab(local_long[d], min_seq, cur_seq);
    r.commit();
}

/* 16-byte vector copy of a hot image by the wave (HT is a multiple of 16 bytes) */
template <class HT>
__device__ inline void copy_image(HT* dst, const HT* src) {
    static_assert(sizeof(HT) % 16 == 0, "hot image must be 16-byte granular");
    const uint4* s = (const uint4*)src;
    uint4* d = (uint4*)dst;
    constexpr int n = sizeof(HT) / 16;
    for (int i = threadIdx.x; i < n; i += WG) d[i] = s[i];
}

/* The tree skeleton's per-node arrays and the zamboni heap of one document: staged into LDS by the
 * HBM-resident kernel (the rest of the hot image stays in HBM). */
template <class HT>
struct Skel {
    int16_t lorder[HT::N], lpos[HT::N], nparent[HT::N];
    int8_t nchild[HT::N], nlevel[HT::N], nscour[HT::N];
    int32_t hseq[HT::H];
    int16_t hrid[HT::H];
    uint8_t hgen[HT::H];
};
/* The scan-critical subset of the skeleton (document order, child counts, parents): staged alone
 * where the whole Skel would cap residency through LDS (config-5 profile). */
template <class HT>
struct SkelLite {
    int16_t lorder[HT::N], lpos[HT::N], nparent[HT::N];
    int8_t nchild[HT::N];
};
template <class T>
__device__ inline void wave_copy(T* dst, const T* src, int n) {
    for (int i = threadIdx.x; i < n; i += WG) dst[i] = src[i];
}
template <class HT>
__device__ inline void skel_move(Skel<HT>& k, HT& z, bool in) {
    constexpr int N = HT::N, H = HT::H;
    if (in) {
        wave_copy(k.lorder, z.lorder, N), wave_copy(k.lpos, z.lpos, N), wave_copy(k.nparent, z.nparent, N);
        wave_copy(k.nchild, z.nchild, N), wave_copy(k.nlevel, z.nlevel, N), wave_copy(k.nscour, z.nscour, N);
        wave_copy(k.hseq, z.hseq, H), wave_copy(k.hrid, z.hrid, H), wave_copy(k.hgen, z.hgen, H);
    } else {
        wave_copy(z.lorder, k.lorder, N), wave_copy(z.lpos, k.lpos, N), wave_copy(z.nparent, k.nparent, N);
        wave_copy(z.nchild, k.nchild, N), wave_copy(z.nlevel, k.nlevel, N), wave_copy(z.nscour, k.nscour, N);
        wave_copy(z.hseq, k.hseq, H), wave_copy(z.hrid, k.hrid, H), wave_copy(z.hgen, k.hgen, H);
    }
}

template <class HT>
__device__ inline void skel_lite_move(SkelLite<HT>& k, HT& z, bool in) {
    constexpr int N = HT::N;
    if (in) {
        wave_copy(k.lorder, z.lorder, N), wave_copy(k.lpos, z.lpos, N), wave_copy(k.nparent, z.nparent, N);
        wave_copy(k.nchild, z.nchild, N);
    } else {
        wave_copy(z.lorder, k.lorder, N), wave_copy(z.lpos, k.lpos, N), wave_copy(z.nparent, k.nparent, N);
        wave_copy(z.nchild, k.nchild, N);
    }
}

/* K1-K4 fused: the whole event stream of a document, one wave per document. LDS = true stages the
 * whole small-profile hot image in LDS; otherwise the image stays in HBM and only the skeleton and
 * the heap (Skel, 3.5 KB for the small profile) are staged. */
template <class HT, bool LDS, int MINW = 1, int SKM = 1> /* SKM: 1 Skel, 2 SkelLite, 0 none */
__global__ __launch_bounds__(WG, MINW) void k_replay(Store<HT> st, int64_t ndocs, const mt_op_rec* ops,
                                              const int64_t* op_off, const uint16_t* text, const int64_t* text_off,
                                              const mt_props_rec* props, const int64_t* props_off, const mt_kv* kv,
                                              const int64_t* kv_off, uint64_t* prof) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Pools p;
    p.ops = ops + op_off[d];
    p.nops = op_off[d + 1] - op_off[d];
    p.text = text + text_off[d];
    p.props = props + props_off[d];
    p.kv = kv + kv_off[d];
    Doc<HT> v = st.doc(d);
    if constexpr (LDS) {
        __shared__ __attribute__((aligned(16))) HT hot;
        HT* g = v.t;
        copy_image(&hot, g);
        __syncthreads();
        v.t = &hot;
        Replica<WaveGPU, HT> r(v, WaveGPU());
        r.replay(p);
        r.commit();
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
        __syncthreads();
        copy_image(g, &hot);
    } else if constexpr (SKM == 2) {
        __shared__ __attribute__((aligned(16))) SkelLite<HT> sk;
        skel_lite_move(sk, *v.t, true);
        __syncthreads();
        Replica<WaveGPU, HT> r(v, WaveGPU());
        r.lo = sk.lorder, r.lp = sk.lpos, r.npar = sk.nparent, r.nch = sk.nchild;
        r.replay(p);
        r.commit();
        __syncthreads();
        skel_lite_move(sk, *v.t, false);
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    } else if constexpr (SKM == 1 && sizeof(Skel<HT>) <= 12288) {
        __shared__ __attribute__((aligned(16))) Skel<HT> sk;
        skel_move(sk, *v.t, true);
        __syncthreads();
        Replica<WaveGPU, HT> r(v, WaveGPU());
        r.lo = sk.lorder, r.lp = sk.lpos, r.npar = sk.nparent, r.nch = sk.nchild, r.nlev = sk.nlevel;
        r.nsc = sk.nscour, r.hsq = sk.hseq, r.hrd = sk.hrid, r.hgn = sk.hgen;
        r.replay(p);
        r.commit();
        __syncthreads();
        skel_move(sk, *v.t, false);
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    } else {
        Replica<WaveGPU, HT> r(v, WaveGPU());
        r.replay(p);
        r.commit();
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    }
}

/* Config 4 (large documents, the tiled profile): one workgroup per document, which has the CU's LDS to
 * itself for the position-search scratch: per-chunk window deltas (NCH counters, all zero between
 * searches) and each window row's chunk position / leaf index / perspective length. The image, the
 * rope and the summaries stay in HBM (~0.2 GB per 1M-op document). */
template <class HT>
__global__ __launch_bounds__(WG) void k_replay_tiled(Store<HT> st, int64_t ndocs, const mt_op_rec* ops,
                                                     const int64_t* op_off, const uint16_t* text,
                                                     const int64_t* text_off, const mt_props_rec* props,
                                                     const int64_t* props_off, const mt_kv* kv, const int64_t* kv_off,
                                                     uint64_t* prof) {
    static_assert(HT::TILED, "tiled profile only");
    __shared__ int32_t cdel[HT::TL::NCH];
    __shared__ int32_t wcp[HT::TL::WCAP], wvs[HT::TL::WCAP];
    __shared__ uint8_t wlx[HT::TL::WCAP];
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    for (int i = threadIdx.x; i < HT::TL::NCH; i += WG) cdel[i] = 0;
    __syncthreads();
    Pools p;
    p.ops = ops + op_off[d];
    p.nops = op_off[d + 1] - op_off[d];
    p.text = text + text_off[d];
    p.props = props + props_off[d];
    p.kv = kv + kv_off[d];
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    r.cdel = cdel;
    r.wcp = wcp;
    r.wvs = wvs;
    r.wlx = wlx;
    r.replay(p);
    r.commit();
#ifdef MT_PROF
    if (prof && threadIdx.x == 0)
        for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
}

/* K5: per-doc digest of the canonical dump */
template <class HT>
__global__ __launch_bounds__(WG) void k_digest(Store<HT> st, int64_t ndocs, uint64_t* out) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    /* The compiler reads the document here with scalar (SMEM) loads, including the
     * base + SGPR-offset + immediate form no other kernel uses. Round 1 put a compiler barrier here
     * after a digest mismatch; tools/smem_probe.hip shows that form (compiler- and asm-emitted)
     * returns what vector loads return, the round-1 failing case is clean without the barrier, and
     * tests/test_gpu_parity.py checks this digest against FNV-1a of k_dump for every document. */
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    uint64_t h = r.digest();
    if (threadIdx.x == 0) out[d] = h;
}

template <class HT>
__global__ __launch_bounds__(WG) void k_dump(Store<HT> st, int64_t doc, uint8_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int64_t m = r.dump(out, cap);
    if (threadIdx.x == 0) *n = m;
}

template <class HT>
__global__ __launch_bounds__(WG) void k_length(Store<HT> st, int64_t doc, int32_t ref_seq, int32_t long_client,
                                              int32_t* out) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int32_t v;
    if (long_client < 0) {
        v = r.length_local();
    } else {
        int32_t sh = r.short_of(long_client);
        v = r.length(ref_seq, sh < 0 ? 0x7fff : sh);
    }
    if (threadIdx.x == 0) *out = v;
}

template <class HT>
__global__ __launch_bounds__(WG) void k_text(Store<HT> st, int64_t doc, int32_t ref_seq, int32_t long_client,
                                            uint16_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int32_t sh;
    if (long_client < 0) {
        sh = r.h.localShort;
        ref_seq = r.h.currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff;
    }
    int64_t m = r.get_text(ref_seq, sh, out, cap);
    if (threadIdx.x == 0) *n = m;
}

/* getContainingSegment (mode 0: a = pos) / getPosition (mode 1: a = rid, b = gen) of one document;
 * out[0] = status (1 found / 0 none), then mt_seg_ref fields or the position */
template <class HT>
__global__ __launch_bounds__(WG) void k_seg(Store<HT> st, int64_t doc, int32_t mode, int32_t a, int32_t b,
                                           int32_t ref_seq, int32_t long_client, int32_t* out) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int32_t sh;
    if (long_client < 0) {
        sh = r.h.localShort;
        ref_seq = r.h.currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff; /* a client the replica has not seen: sequenced content only */
    }
    int32_t res[7] = {0, -1, 0, 0, 0, 0, 0};
    if (mode == 0) {
        int32_t off = 0;
        int32_t s = r.containing(a, ref_seq, sh, &off);
        if (s >= 0) {
            int32_t rid = r.z.rid[s];
            res[0] = 1;
            res[1] = rid;
            res[2] = r.z.rgen[rid];
            res[3] = off;
            res[4] = r.z.len(s);
            res[5] = r.z.seq(s);
            res[6] = r.long_of(r.z.cli(s));
        }
    } else {
        int32_t s = (a >= 0 && a < HT::S) ? r.slot_of(a, b) : -1;
        if (s >= 0) {
            res[0] = 1;
            res[1] = r.position_of(s, ref_seq, sh);
        }
    }
    if (threadIdx.x == 0)
        for (int i = 0; i < 7; i++) out[i] = res[i];
}

/* per-doc header fields: errors, stats, roofline work counters */
template <class HT>
__global__ void k_hdr(Store<HT> st, int64_t ndocs, int32_t* err, int32_t* err_op, int32_t* stats4, int64_t* work3) {
    int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndocs) return;
    const DocHdr& h = st.doc(d).t->h;
    if (err) err[d] = h.err;
    if (err_op) err_op[d] = h.errOp;
    if (stats4) {
        stats4[4 * d + 0] = h.nleaf;
        stats4[4 * d + 1] = h.hwSlots;
        stats4[4 * d + 2] = h.hwHeap;
        stats4[4 * d + 3] = h.opsDone;
    }
    if (work3) {
        work3[3 * d + 0] = h.seqOps;
        work3[3 * d + 1] = h.sumR;
        work3[3 * d + 2] = h.sumW;
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
    int profile = 0;
    bool lds = false; /* small profile staged in LDS for the whole replay (MT_REPLAY_LDS=1) */
    int waves = 7;    /* occupancy target of the HBM-resident kernel (MT_REPLAY_WAVES=6|7|8) */
    int mat_skel = 2; /* config-5 profile: 2 SkelLite in LDS, 1 Skel, 0 none (MT_REPLAY_MAT_SKEL) */
    Store<HotSmall> s0;
    Store<HotMid> s1;
    Store<HotBig> s2;
    Store<HotMat> s3;
    Store<HotHuge> s4;
    void* mem = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    bool staged = false;
    DevBuf ops, op_off, text, text_off, props, props_off, kv, kv_off, tmp, local_ids, prof;
    int32_t min_seq0 = 0, cur_seq0 = 0;
    bool collab = false;
    std::string err;
};

/* call f(store) for the engine's profile */
template <class F>
static int32_t with_store(mt_engine* e, F&& f) {
#ifdef MT_ISA_SMALL /* analysis builds (tools/isa_small.sh): the config-3 profile's kernels only */
    return f(e->s0);
#endif
    if (e->profile == 0) return f(e->s0);
    if (e->profile == 1) return f(e->s1);
    if (e->profile == 3) return f(e->s3);
    if (e->profile == 4) return f(e->s4);
    return f(e->s2);
}

static int32_t hip_fail(mt_engine* e, hipError_t st, const char* what) {
    if (e) e->err = std::string(what) + ": " + hipGetErrorString(st);
    return MT_E_HIP;
}
#define HIPCHK(e, x)                                        \
    do {                                                    \
        hipError_t st_ = (x);                               \
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

static dim3 docs_grid(int64_t n) { return dim3((unsigned)n); }
static dim3 flat_grid(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

static int32_t launch_init(mt_engine* e) {
    return with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_init<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs);
        int32_t rc = launch_check(e, "k_init");
        if (rc || !e->collab) return rc;
        hipLaunchKernelGGL((k_start_collab<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs,
                           (const int32_t*)e->local_ids.p, e->min_seq0, e->cur_seq0);
        return launch_check(e, "k_start_collab");
    });
}

extern "C" {

int32_t mt_engine_create(int32_t device, int64_t ndocs, const mt_caps* caps, mt_engine** out) {
    if (!out || !caps || ndocs < 1 || ndocs > (int64_t)0x7fffffff) return MT_E_ARG;
    *out = nullptr;
    Caps k = {caps->acap, caps->mcap, caps->gcap};
    int prof = profile_for(caps->ncap);
    if (!caps_valid(k) || prof < 0 || caps->ccap > 254) return MT_E_ARG; /* short ids are bytes; 0xFF = LocalClientId */
    mt_engine* e = new mt_engine();
    e->device = device;
    e->ndocs = ndocs;
    const char* g = getenv("MT_REPLAY_LDS");
    e->lds = g && g[0] == '1';
    /* Occupancy of the HBM-resident small-profile kernel: documents are replayed one per wave and
     * a document's events are sequential, so a batch runs in "rounds" of 1,024 x waves documents
     * (256 CUs x 4 SIMDs). 7 waves/SIMD is fastest per wave (8 spills registers: 168 vs 174 Mops/s
     * at 32k docs), but a small batch (a strong-scaled shard: 8,192 or 16,384 docs per GPU) is
     * better served by 8, which runs it in 1 or 2 full rounds instead of a last partial one. */
    const char* wv = getenv("MT_REPLAY_WAVES");
    e->waves = wv ? atoi(wv) : (ndocs <= 16384 ? 8 : 7);
    const char* ms = getenv("MT_REPLAY_MAT_SKEL");
    e->mat_skel = ms ? atoi(ms) : 2;
    e->profile = prof;
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
    DevBuf* bufs[] = {&e->ops,    &e->op_off, &e->text, &e->text_off, &e->props,     &e->props_off,
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
    rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_start_collab<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs,
                           (const int32_t*)e->local_ids.p, min_seq, cur_seq);
        return launch_check(e, "k_start_collab");
    });
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
    /* every pool reference of every event must be in bounds before the kernel dereferences it */
    for (int64_t d = 0; d < nd; d++) {
        for (int64_t i = op_off[d]; i < op_off[d + 1]; i++) {
            const mt_op_rec& o = ops[i];
            int kind = o.kind & MT_OP_KIND_MASK;
            if (kind == MT_OP_INSERT && o.seg_kind == MT_SEG_TEXT &&
                text_off[d] + (int64_t)o.text_off + o.text_len > text_units)
                return MT_E_ARG;
            /* snapshot-load records carry the segment length in pos2 (mt_oplog.h) */
            if ((kind == MT_OP_RELOAD || kind == MT_OP_APPEND) && o.seg_kind == MT_SEG_TEXT &&
                (o.pos2 < 0 || text_off[d] + (int64_t)o.text_off + o.pos2 > text_units))
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
    return launch_init(e);
}

int32_t mt_engine_run(mt_engine* e) {
    if (!e || !e->staged) return MT_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
#ifdef MT_PROF
    if (ensure(e, e->prof, sizeof(uint64_t) * PH_N * e->ndocs)) return MT_E_NOMEM;
#endif
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    int32_t rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        auto launch = [&](auto kern) {
            hipLaunchKernelGGL(kern, docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs,
                               (const mt_op_rec*)e->ops.p, (const int64_t*)e->op_off.p, (const uint16_t*)e->text.p,
                               (const int64_t*)e->text_off.p, (const mt_props_rec*)e->props.p,
                               (const int64_t*)e->props_off.p, (const mt_kv*)e->kv.p, (const int64_t*)e->kv_off.p,
                               (uint64_t*)e->prof.p);
        };
        if constexpr (std::is_same_v<HT, HotSmall>) {
            /* Default: the hot image stays in HBM (skeleton and heap in LDS) and the kernel is built
             * for 7 waves per SIMD, so 7,168 documents are in flight (28 per CU): at one wavefront per
             * document the replay is bound by the latency of its dependent accesses, and occupancy
             * hides more of it than full LDS residency (4 documents per CU) saves. With the leaf-line
             * layout 7 beats 6 and 8 (174 / 161 / 168 Mops/s at 32k docs; 8 spills registers;
             * tools/gpu_occupancy.sh). MT_REPLAY_LDS=1 selects the fully LDS-staged form. */
#ifdef MT_ISA_SMALL
            launch(k_replay<HT, false, 7>);
#else
            if (e->lds)
                launch(k_replay<HT, true>);
            else if (e->waves == 8)
                launch(k_replay<HT, false, 8>);
            else if (e->waves == 6)
                launch(k_replay<HT, false, 6>);
            else
                launch(k_replay<HT, false, 7>);
#endif
        } else if constexpr (std::is_same_v<HT, HotMat>) {
            /* Default (MT_REPLAY_MAT_SKEL=2): only SkelLite (4.5 KB) in LDS, 7 waves per SIMD
             * (116 Mops/s at 16k replicas). =1 stages the whole Skel (10.7 KB), which caps residency
             * at 14 documents per CU through LDS (103 Mops/s); =0 stages nothing (104 Mops/s). */
            if (e->mat_skel == 1)
                launch(k_replay<HT, false, 4>);
            else if (e->mat_skel == 2)
                launch(k_replay<HT, false, 7, 2>);
            else
                launch(k_replay<HT, false, 7, 0>);
        } else if constexpr (HT::TILED) {
            launch(k_replay_tiled<HT>);
        } else {
            launch(k_replay<HT, false>);
        }
        return launch_check(e, "k_replay");
    });
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
    rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_hdr<HT>), flat_grid(n), dim3(256), 0, e->stream, st, n, de, deo, ds, dw);
        return launch_check(e, "k_hdr");
    });
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
    rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_digest<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs,
                           (uint64_t*)e->tmp.p);
        return launch_check(e, "k_digest");
    });
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
    int32_t rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_dump<HT>), dim3(1), dim3(WG), 0, e->stream, st, doc, dbuf, out ? cap : 0, dn);
        return launch_check(e, "k_dump");
    });
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
    rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_length<HT>), dim3(1), dim3(WG), 0, e->stream, st, doc, ref_seq, long_client,
                           (int32_t*)e->tmp.p);
        return launch_check(e, "k_length");
    });
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
    int32_t rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_text<HT>), dim3(1), dim3(WG), 0, e->stream, st, doc, ref_seq, long_client, dbuf,
                           out ? cap : 0, dn);
        return launch_check(e, "k_text");
    });
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
    rc = with_store(e, [&](auto& st) {
        using HT = typename std::decay_t<decltype(st)>::Hot;
        hipLaunchKernelGGL((k_seg<HT>), dim3(1), dim3(WG), 0, e->stream, st, doc, mode, a, b, ref_seq, long_client,
                           (int32_t*)e->tmp.p);
        return launch_check(e, "k_seg");
    });
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
