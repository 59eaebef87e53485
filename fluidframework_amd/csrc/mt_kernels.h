/*
 * mt_kernels.h — the CDNA4 (gfx950) kernels of the replay engine and their per-profile launchers.
 *
 * One 64-lane wavefront replays one document: control flow is wave-uniform, and the
 * data-parallel parts of every op — the perspective prefix scan that replaces the reference's
 * root-to-leaf walk (mergeTree.ts:2378-2507, nodeLength 1692-1732), range marking
 * (nodeMap 2936-2998), stable-id lookup and text copies — run across the 64 lanes with
 * DPP/permute shuffles and 64-bit ballots (mt_wave.h). Documents are independent, so the grid
 * is one workgroup per document and the machine is filled by documents.
 *
 * Each profile's kernels are instantiated in a translation unit of their own (prof_*.hip, and one
 * per k_replay occupancy variant), so the library builds in parallel; mt_replay.hip holds the C ABI
 * and dispatches through the engine's ProfOps table.
 */
#pragma once
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
/* local[d] = doc d's local long id, local[ndocs + d] / local[2 ndocs + d] its minSeq / currentSeq */
__global__ __launch_bounds__(WG) void k_start_collab(Store<HT> st, int64_t ndocs, const int32_t* local) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    r.start_collab(local[d], local[ndocs + d], local[2 * ndocs + d]);
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
    DocHdr zh; /* the image's header fields (the replica keeps the hot ones in registers) */
    int16_t lorder[HT::N], lpos[HT::N], nparent[HT::N];
    int8_t nchild[HT::N], nlevel[HT::N], nscour[HT::N];
    int32_t hseq[HT::H];
    int16_t hrid[HT::H];
    uint8_t hgen[HT::H];
    uint8_t l2s[HT::C];  /* long -> short client id */
    uint16_t s2l[HT::C]; /* short -> long */
};
/* The scan-critical subset of the skeleton (document order, child counts, parents): staged alone
 * where the whole Skel would cap residency through LDS (config-5 profile). */
template <class HT>
struct SkelLite {
    DocHdr zh; /* the image's header fields */
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
    constexpr int C = HT::C, NH = (int)(sizeof(DocHdr) / 4);
    if (in) {
        wave_copy((int32_t*)&k.zh, (const int32_t*)&z.h, NH);
        wave_copy(k.lorder, z.lorder, N), wave_copy(k.lpos, z.lpos, N), wave_copy(k.nparent, z.nparent, N);
        wave_copy(k.nchild, z.nchild, N), wave_copy(k.nlevel, z.nlevel, N), wave_copy(k.nscour, z.nscour, N);
        wave_copy(k.hseq, z.hseq, H), wave_copy(k.hrid, z.hrid, H), wave_copy(k.hgen, z.hgen, H);
        wave_copy(k.l2s, z.l2s, C), wave_copy(k.s2l, z.s2l, C);
    } else {
        wave_copy((int32_t*)&z.h, (const int32_t*)&k.zh, NH);
        wave_copy(z.lorder, k.lorder, N), wave_copy(z.lpos, k.lpos, N), wave_copy(z.nparent, k.nparent, N);
        wave_copy(z.nchild, k.nchild, N), wave_copy(z.nlevel, k.nlevel, N), wave_copy(z.nscour, k.nscour, N);
        wave_copy(z.hseq, k.hseq, H), wave_copy(z.hrid, k.hrid, H), wave_copy(z.hgen, k.hgen, H);
        wave_copy(z.l2s, k.l2s, C), wave_copy(z.s2l, k.s2l, C);
    }
}

template <class HT>
__device__ inline void skel_lite_move(SkelLite<HT>& k, HT& z, bool in) {
    constexpr int N = HT::N, NH = (int)(sizeof(DocHdr) / 4);
    if (in) {
        wave_copy((int32_t*)&k.zh, (const int32_t*)&z.h, NH);
        wave_copy(k.lorder, z.lorder, N), wave_copy(k.lpos, z.lpos, N), wave_copy(k.nparent, z.nparent, N);
        wave_copy(k.nchild, z.nchild, N);
    } else {
        wave_copy((int32_t*)&z.h, (const int32_t*)&k.zh, NH);
        wave_copy(z.lorder, k.lorder, N), wave_copy(z.lpos, k.lpos, N), wave_copy(z.nparent, k.nparent, N);
        wave_copy(z.nchild, k.nchild, N);
    }
}

/* Per-launch extras of the replay kernels: the profiling build's per-document phase clocks, and the dispatch
 * order (workgroup b replays document order[b]; the hardware dispatches workgroups in index order as slots free
 * up, so a longest-first order is list scheduling by cost, mt_engine_set_order). */
struct ReplayAux {
    uint64_t* prof;
    const int32_t* order;
    int64_t doc0; /* a launch over documents [doc0, doc0 + grid): the chunked submit (mt_engine_submit_run) */
    int32_t compact; /* the staged pools are indexed by launch position, not by document (mt_engine_submit_docs:
                        `order` lists the documents with records) */
    const uint8_t* vkind; /* value kinds (mt_engine_set_value_kinds), nvk entries */
    int32_t nvk;
};
__device__ inline int64_t aux_doc(const ReplayAux& a) {
    const int64_t b = a.doc0 + (int64_t)blockIdx.x;
    return a.order ? a.order[b] : b;
}
/* the entry of the staged offset arrays that holds document d's pools */
__device__ inline int64_t aux_pool(const ReplayAux& a, int64_t d) {
    return a.compact ? a.doc0 + (int64_t)blockIdx.x : d;
}
/* the document's replay start / end on the constant-rate clock (s_memrealtime, 100 MHz), kept in its image header
 * (DocHdr.tStart / tEnd: no register stays live for it through the replay; mt_engine_doc_times) */
/* Stamped into the header copy the replay writes back (the LDS-staged DocHdr where one is staged): a direct HBM store
 * by lane 0 beside the other lanes' staging copies of the same header could be overwritten by the stale copy. */
__device__ inline void doc_stamp(DocHdr& h, int end) {
    if (threadIdx.x == 0) {
        int64_t now = (int64_t)__builtin_amdgcn_s_memrealtime();
        if (end)
            h.tEnd = now;
        else
            h.tStart = now;
    }
}

/* K1-K4 fused: the whole event stream of a document, one wave per document. LDS = true stages the
 * whole small-profile hot image in LDS; otherwise the image stays in HBM and only the skeleton and
 * the heap (Skel, 3.5 KB for the small profile) are staged. */
/* VAR tags a build variant compiled with other flags in its own translation unit (1: compiler-chosen
 * inlining): the kernel's name must differ, since a host launch resolves the kernel by name. */
/* DL: the delta-event build (engines created with caps.dcap > 0) */
#ifdef MT_NUM_SGPR /* experiment: an explicit SGPR budget for the flat kernel */
#define MT_SGPR_ATTR __attribute__((amdgpu_num_sgpr(MT_NUM_SGPR)))
#else
#define MT_SGPR_ATTR
#endif
template <class HT, bool LDS, int MINW = 1, int SKM = 1, int VAR = 0, bool DL = false, bool LOAD = true> /* SKM: 1 Skel, 2 SkelLite, 0 none */
__global__ __launch_bounds__(WG, MINW) MT_SGPR_ATTR void k_replay(Store<HT> st, int64_t ndocs, const mt_op_rec* ops,
                                              const int64_t* op_off, const uint16_t* text, const int64_t* text_off,
                                              const mt_props_rec* props, const int64_t* props_off, const mt_kv* kv,
                                              const int64_t* kv_off, ReplayAux aux) {
    if ((int64_t)blockIdx.x >= ndocs) return;
    const int64_t d = aux_doc(aux);
    uint64_t* prof = aux.prof;
    (void)prof;
#ifdef MT_PROF
    __shared__ uint64_t sprof[PH_N]; /* the replica's phase clocks (LDS, not registers) */
    for (int i = threadIdx.x; i < PH_N; i += WG) sprof[i] = 0;
    __syncthreads();
#define MT_PROF_ATTACH(r) (r).prof = sprof
#else
#define MT_PROF_ATTACH(r) (void)0
#endif
    Pools p;
    const int64_t pi = aux_pool(aux, d);
    p.ops = ops + op_off[pi];
    p.nops = op_off[pi + 1] - op_off[pi];
    p.text = text + text_off[pi];
    p.props = props + props_off[pi];
    p.kv = kv + kv_off[pi];
    p.vkind = aux.vkind;
    p.nvk = aux.nvk;
    Doc<HT> v = st.doc(d);
    if constexpr (LDS) {
        __shared__ __attribute__((aligned(16))) HT hot;
        HT* g = v.t;
        copy_image(&hot, g);
        __syncthreads();
        doc_stamp(hot.h, 0);
        v.t = &hot;
        Replica<WaveGPU, HT, DL, LOAD> r(v, WaveGPU());
        MT_PROF_ATTACH(r);
        r.replay(p);
        r.commit();
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
        doc_stamp(hot.h, 1);
        __syncthreads();
        copy_image(g, &hot);
    } else if constexpr (SKM == 2) {
        __shared__ __attribute__((aligned(16))) SkelLite<HT> sk;
        skel_lite_move(sk, *v.t, true);
        __syncthreads();
        doc_stamp(sk.zh, 0);
        Replica<WaveGPU, HT, DL, LOAD> r(v, WaveGPU());
        MT_PROF_ATTACH(r);
        r.lo = sk.lorder, r.lp = sk.lpos, r.npar = sk.nparent, r.nch = sk.nchild;
        r.zh = &sk.zh;
        r.replay(p);
        r.commit();
        doc_stamp(sk.zh, 1);
        __syncthreads();
        skel_lite_move(sk, *v.t, false);
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    } else if constexpr (SKM == 1 && sizeof(Skel<HT>) <= 12288) {
        static_assert(sizeof(DocHdr) % 4 == 0, "the header is copied in dwords");
        __shared__ __attribute__((aligned(16))) Skel<HT> sk;
        skel_move(sk, *v.t, true);
        __syncthreads();
        doc_stamp(sk.zh, 0);
        Replica<WaveGPU, HT, DL, LOAD> r(v, WaveGPU());
        MT_PROF_ATTACH(r);
        r.lo = sk.lorder, r.lp = sk.lpos, r.npar = sk.nparent, r.nch = sk.nchild, r.nlev = sk.nlevel;
        r.nsc = sk.nscour, r.hsq = sk.hseq, r.hrd = sk.hrid, r.hgn = sk.hgen;
        r.zh = &sk.zh, r.l2s = sk.l2s, r.s2l = sk.s2l;
        r.replay(p);
        r.commit();
        doc_stamp(sk.zh, 1);
        __syncthreads();
        skel_move(sk, *v.t, false);
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    } else {
        doc_stamp(v.t->h, 0);
        Replica<WaveGPU, HT, DL, LOAD> r(v, WaveGPU());
        MT_PROF_ATTACH(r);
        r.replay(p);
        r.commit();
        doc_stamp(v.t->h, 1);
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    }
}

/* Config 4 (large documents, the tiled profile): one workgroup per document, which has the CU's LDS to
 * itself (155 KB): the position-search scratch (per-chunk window deltas, all zero between searches, and each
 * window row's chunk position / leaf index / perspective length) and, for the duration of the replay, the
 * rope's chunk arrays and the window set (with each row's last-seen slot). The rows, the leaf summaries,
 * the per-leaf rope links and the zamboni heap stay in HBM (~0.2 GB per 1M-op document). An LDS copy of the
 * heap (~60 entries in use at lag 64) measured slower: a heap that can be in either memory is reached through
 * flat accesses, which wait for both counters (r04j A/B: 10.75 -> 10.33M ops/s at 256 x 300k). */
#ifndef MT_PF_HELPERS
#define MT_PF_HELPERS 0 /* prefetch helper waves per config-4 document (0: one wave per document; 1 and 2
                           * measured 2.4 % and 3.2 % slower at 256 x 300k, profiles/r04f_ab) */
#endif
/* waves besides the replaying one in a config-4 workgroup: the prefetch helpers, or the window helper (MT_WIN_HELPER,
 * mt_core.h win_helper) */
#ifndef MT_WIN_HELPER
#define MT_WIN_HELPER 2 /* mt_core.h */
#endif
#define MT_TILED_HELPERS (MT_WIN_HELPER ? 1 : MT_PF_HELPERS)
#ifndef MT_PF_AHEAD
#define MT_PF_AHEAD 2 /* records ahead of the replaying wave each helper looks */
#endif
/* The helper waves of a config-4 workgroup (k_replay_tiled). A document's events are one dependent chain, so
 * the other SIMDs of the document's CU cannot share the replay; they run ahead of it instead: for the records
 * after the one being applied, a helper resolves each position approximately from the current summaries
 * (chunk scan over the staged LDS summaries without the window deltas, then the chunk's leaf summaries) and
 * loads what the replay will read there — the chunk's leaf-summary line, the leaf's 128-byte line and its
 * neighbour's, the leaf's row ids and child count, and the first 16 bytes of its rows' cold records — and,
 * for the zamboni that follows, the leaf of the row at the heap's top. Those reads then hit the L2 / MALL when
 * the replay makes them. Helpers only read (the summaries they scan may be mid-update: an approximate answer
 * only changes what is prefetched); every index is clamped to its array; they exit when the replay is done. */
template <class HT>
__device__ void tiled_prefetch(Doc<HT> v, const mt_op_rec* ops, int64_t nops, const volatile int32_t* cur,
                               const volatile int32_t* done, const int32_t* lcord, const int32_t* lcst,
                               const int32_t* lccnt, int32_t* sink) {
    constexpr int NCH = HT::TL::NCH, N = HT::N, S = HT::S;
    const HT* t = v.t;
    const auto& tl = t->tl;
    const typename HT::Cold* cold = v.cold();
    WaveGPU w;
    const int32_t lane = w.lane(), helper = (int32_t)(threadIdx.x / WG) - 1;
    uint32_t acc = 0;
    int64_t last = -1;
    auto touch_leaf = [&](int32_t leaf) {
        leaf = leaf < 0 ? 0 : (leaf >= N ? N - 1 : leaf);
        const int32_t* line = (const int32_t*)&t->lf[leaf];
        int32_t j = lane & 7;
        int32_t r = t->rid[leaf * 8 + j];
        r = r < 0 ? 0 : (r >= S ? S - 1 : r);
        uint32_t x = lane < 32 ? (uint32_t)line[lane] : (uint32_t)t->nchild[leaf];
        const uint32_t* cr = (const uint32_t*)&cold[r];
        x ^= lane < 8 ? cr[0] ^ cr[1] ^ cr[2] ^ cr[3] : (uint32_t)t->rleaf[r] ^ t->rgen[r];
        acc ^= x ^ (uint32_t)r;
    };
    while (!*done) {
        int64_t k = (int64_t)*cur + 1 + helper * MT_PF_AHEAD;
        if (k <= last) k = last + 1;
        if (k >= nops || k > (int64_t)*cur + (helper + 1) * MT_PF_AHEAD) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        last = k;
        mt_op_rec op = ops[k];
        int32_t kind = op.kind & MT_OP_KIND_MASK;
        if (kind > MT_OP_ANNOTATE || (op.kind & (MT_OPF_LOCAL | MT_OPF_TREE))) continue;
        int32_t nch = tl.nchunk;
        nch = nch < 1 ? 1 : (nch > NCH ? NCH : nch);
        for (int32_t e = 0; e < (kind == MT_OP_INSERT ? 1 : 2); e++) {
            int32_t pos = e ? op.pos2 : op.pos1;
            int32_t run = 0, cp = nch - 1;
            for (int32_t b = 0; b < nch; b += WG) { /* chunk scan over the staged STABLE summaries */
                int32_t i = b + lane;
                int32_t x = i < nch ? lcst[i] : 0;
                int32_t tot;
                int32_t q = run + w.excl_scan(x, &tot);
                uint64_t m = w.ballot(i < nch && q + x >= pos);
                if (m) {
                    int32_t l = WaveGPU::ffs(m);
                    cp = b + l;
                    run = w.bcast(q, l);
                    break;
                }
                run += tot;
            }
            int32_t c = lcord[cp];
            c = c < 0 ? 0 : (c >= NCH ? NCH - 1 : c);
            int32_t cnt = lccnt[c];
            cnt = cnt < 1 ? 1 : (cnt > 64 ? 64 : cnt);
            int32_t x = lane < cnt ? tl.cls[c][lane] : 0; /* the chunk's leaf summaries: one line */
            int32_t tot;
            int32_t q = run + w.excl_scan(x, &tot);
            uint64_t m = w.ballot(lane < cnt && q + x >= pos);
            int32_t li = m ? WaveGPU::ffs(m) : cnt - 1;
            int32_t leaf = tl.cleaf[c][li];
            touch_leaf(leaf);
            touch_leaf(tl.cleaf[c][li + 1 < cnt ? li + 1 : li]);
        }
        if (t->h.heapN > 0) { /* the zamboni after it: the leaf of the row at the heap's top */
            int32_t r = t->hrid[0];
            r = r < 0 ? 0 : (r >= S ? S - 1 : r);
            touch_leaf(t->rleaf[r]);
        }
    }
    if (acc == 0x9e3779b9u && lane == 0) *sink = (int32_t)acc; /* keeps the loads */
}

/* NARROW (the default config-4 kernel): the zamboni heap in LDS too (~60 entries in use at lag 64: every pop and
 * push an LDS pass instead of an HBM round trip), beside a window set of MT_NARROW_W entries; a document whose
 * heap or window set would outgrow them latches E_CAPACITY and the engine replays it in the wide variant
 * (NARROW = false: the heap in HBM, the full window set) — capacity promotion (mt_replay.hip). */
template <class HT, bool DL = false, bool NARROW = false>
__global__ __launch_bounds__(WG * (1 + MT_TILED_HELPERS)) void k_replay_tiled(Store<HT> st, int64_t ndocs, const mt_op_rec* ops,
                                                     const int64_t* op_off, const uint16_t* text,
                                                     const int64_t* text_off, const mt_props_rec* props,
                                                     const int64_t* props_off, const mt_kv* kv, const int64_t* kv_off,
                                                     ReplayAux aux) {
    static_assert(HT::TILED, "tiled profile only");
    typedef Replica<WaveGPU, HT, DL, true, NARROW> R;
    constexpr int NCH = HT::TL::NCH, WCAP = R::WCAPR, HL = NARROW ? R::HCAPR : 1;
    __shared__ int32_t cdel[NCH];
    __shared__ int32_t wcp[WCAP], wvs[WCAP];
    __shared__ uint8_t wlx[WCAP];
    __shared__ DocHdr zhs; /* the image's header fields, staged for the replay */
    /* the rope's chunk arrays and the window set, staged for the replay (written back at the end) */
    constexpr int NG = HT::TL::NG;
    __shared__ int32_t lcord[NCH], lcst[NCH], lcpos[NCH], lccnt[NCH], lwrid[WCAP];
    __shared__ int32_t lgst[NG], lgdel[NG]; /* chunk-group sums of lcst and of cdel */
    __shared__ uint16_t lkeys[HT::K];       /* the property key table */
    __shared__ __attribute__((aligned(16))) uint8_t lwgen[WCAP];
    __shared__ int32_t lwslot[WCAP];
    __shared__ int32_t lhseq[HL]; /* NARROW: the zamboni heap */
    __shared__ typename HT::IX lhrid[HL];
    __shared__ uint8_t lhgen[HL];
    __shared__ int32_t pfcur, pfdone, pfsink; /* the replaying wave's record, its end, the helpers' sink */
#if MT_WIN_HELPER
    __shared__ typename R::WinMail wmail; /* the window helper's mailbox */
#endif
#ifdef MT_PROF
    __shared__ uint64_t sprof[PH_N];
    for (int i = threadIdx.x; i < PH_N; i += blockDim.x) sprof[i] = 0;
#endif
    if ((int64_t)blockIdx.x >= ndocs) return;
    const int64_t d = aux_doc(aux);
    uint64_t* prof = aux.prof;
    (void)prof;
    Doc<HT> v = st.doc(d);
    auto& tl = v.t->tl;
    const bool replayer = threadIdx.x < WG;
    /* what the staged arrays cannot hold: nothing is staged, the replica latches E_CAPACITY */
    const bool fits = !NARROW || (tl.wN <= WCAP && v.t->h.heapN <= HL);
    const int32_t nheap = NARROW ? v.t->h.heapN : 0;
    if (replayer && fits) {
        for (int i = threadIdx.x; i < NCH; i += WG) cdel[i] = 0;
        for (int i = threadIdx.x; i < NG; i += WG) lgdel[i] = 0;
        wave_copy(lgst, tl.gst, NG);
        wave_copy(lkeys, v.t->keys, HT::K);
        wave_copy((int32_t*)&zhs, (const int32_t*)&v.t->h, (int)(sizeof(DocHdr) / 4));
        wave_copy(lcord, tl.cord, NCH);
        wave_copy(lcst, tl.cst, NCH);
        wave_copy(lcpos, tl.cpos, NCH);
        wave_copy(lccnt, tl.ccnt, NCH);
        wave_copy(lwrid, tl.wrid, WCAP);
        wave_copy((int32_t*)lwgen, (const int32_t*)tl.wgen, WCAP / 4);
        wave_copy(lwslot, tl.wslot, WCAP);
        if constexpr (NARROW) {
            wave_copy(lhseq, v.t->hseq, nheap);
            wave_copy(lhrid, v.t->hrid, nheap);
            wave_copy(lhgen, v.t->hgen, nheap);
        }
    }
    if (threadIdx.x == 0) { /* every path: helper waves read these after the barrier */
        pfcur = 0;
        pfdone = fits ? 0 : 1;
#if MT_WIN_HELPER
        wmail.req = wmail.done = wmail.quit = 0;
#endif
    }
    __syncthreads();
    if (replayer && fits) doc_stamp(zhs, 0);
    Pools p;
    const int64_t pi = aux_pool(aux, d);
    p.ops = ops + op_off[pi];
    p.nops = op_off[pi + 1] - op_off[pi];
    p.text = text + text_off[pi];
    p.props = props + props_off[pi];
    p.kv = kv + kv_off[pi];
    p.vkind = aux.vkind;
    p.nvk = aux.nvk;
    if (!replayer) {
#if MT_WIN_HELPER
        if (threadIdx.x < 2 * WG) { /* the window helper: the replaying wave's LDS views of the set and the rope */
            R hr(v, WaveGPU());
            hr.tcpos = lcpos;
            hr.twrid = lwrid;
            hr.twgen = lwgen;
            hr.twslot = lwslot;
            hr.wm = &wmail;
            hr.win_helper(&pfdone);
        }
#else
        tiled_prefetch<HT>(v, p.ops, p.nops, &pfcur, &pfdone, lcord, lcst, lccnt, &pfsink);
#endif
    } else if (!fits) {
        doc_stamp(v.t->h, 0);
        R r(v, WaveGPU());
        r.fail(E_CAPACITY);
        r.commit();
        doc_stamp(v.t->h, 1);
    } else {
        R r(v, WaveGPU());
        MT_PROF_ATTACH(r);
        r.cdel = cdel;
        r.wcp = wcp;
        r.wvs = wvs;
        r.wlx = wlx;
        r.zh = &zhs;
        r.tcord = lcord;
        r.tcst = lcst;
        r.tgst = lgst;
        r.gdel = lgdel;
        r.keys = lkeys;
        r.tcpos = lcpos;
        r.tccnt = lccnt;
        r.twrid = lwrid;
        r.twgen = lwgen;
        r.twslot = lwslot;
        if constexpr (NARROW) {
            r.hsq = lhseq;
            r.hrd = lhrid;
            r.hgn = lhgen;
        }
        if (MT_PF_HELPERS > 0) r.pfcur = &pfcur;
#if MT_WIN_HELPER
        r.wm = &wmail;
#endif
        r.replay(p);
        r.commit();
        doc_stamp(zhs, 1);
        if (threadIdx.x == 0) *(volatile int32_t*)&pfdone = 1;
#ifdef MT_PROF
        if (prof && threadIdx.x == 0)
            for (int i = 0; i < PH_N; i++) prof[d * PH_N + i] = r.prof[i];
#endif
    }
#if MT_WIN_HELPER == 2
    if (replayer) { /* the end: the helper's last barrier (win_helper) */
        if (threadIdx.x == 0) wmail.quit = 1;
        __syncthreads();
    }
#endif
    __syncthreads();
    if (replayer && fits) {
        wave_copy((int32_t*)&v.t->h, (const int32_t*)&zhs, (int)(sizeof(DocHdr) / 4));
        wave_copy(tl.cord, lcord, NCH);
        wave_copy(tl.cst, lcst, NCH);
        wave_copy(tl.gst, lgst, NG);
        wave_copy(v.t->keys, lkeys, HT::K);
        wave_copy(tl.cpos, lcpos, NCH);
        wave_copy(tl.ccnt, lccnt, NCH);
        wave_copy(tl.wrid, lwrid, WCAP);
        wave_copy((int32_t*)tl.wgen, (const int32_t*)lwgen, WCAP / 4);
        wave_copy(tl.wslot, lwslot, WCAP);
        if constexpr (NARROW) {
            int32_t n = zhs.heapN <= HL ? zhs.heapN : HL;
            wave_copy(v.t->hseq, lhseq, n);
            wave_copy(v.t->hrid, lhrid, n);
            wave_copy(v.t->hgen, lhgen, n);
        }
    }
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

/* A read under a remote perspective (refSeq, client) is answered only where the reference's block
 * PartialSequenceLengths and the leaf visibility predicate the engine sums agree: refSeq >= minSeq (the
 * partials fold everything at or below the window into minLength, partialLengths.ts:489-518) and refSeq at
 * or past every refSeq that client has sent an op under (`floor`, tracked by the host from the records:
 * later entries of that client are added whole, getBranchPartialLength 456-486, which counts a removal of
 * a segment inserted after refSeq that the predicate does not — the "invalid combination" of
 * partialLengths.ts:672-681). The local client (cachedLength) and a non-collaborating replica are always
 * answered. Measured against the reference on 7,600 perspectives: every one this rule answers is equal
 * (tests/test_ref_persp.py). */
template <class R>
__device__ inline bool persp_refused(const R& r, int32_t ref_seq, int32_t long_client, int32_t floor) {
    if (long_client < 0 || !r.h.collaborating || long_client == r.h.localLong) return false;
    return ref_seq < r.h.minSeq || ref_seq < floor;
}

template <class HT>
__global__ __launch_bounds__(WG) void k_length(Store<HT> st, int64_t doc, int32_t ref_seq, int32_t long_client,
                                              int32_t floor, int32_t* out) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int32_t v;
    if (persp_refused(r, ref_seq, long_client, floor)) {
        if (threadIdx.x == 0) out[0] = 0, out[1] = 1;
        return;
    }
    if (long_client < 0) {
        v = r.length_local();
    } else {
        int32_t sh = r.short_of(long_client);
        v = r.length(ref_seq, sh < 0 ? 0x7fff : sh);
    }
    if (threadIdx.x == 0) out[0] = v, out[1] = 0;
}

template <class HT>
__global__ __launch_bounds__(WG) void k_text(Store<HT> st, int64_t doc, int32_t ref_seq, int32_t long_client,
                                            int32_t floor, int32_t start, int32_t end, const uint16_t* ph,
                                            int32_t pl, uint16_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    if (persp_refused(r, ref_seq, long_client, floor)) {
        if (threadIdx.x == 0) *n = -E_UNSUPPORTED;
        return;
    }
    int32_t sh;
    if (long_client < 0) {
        sh = r.h.localShort;
        ref_seq = r.h.currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff;
    }
    /* pl < 0: SharedSequence.getItems(start, end) in the local view (the C ABI's mt_engine_get_items) */
    int64_t m = pl < 0 ? r.get_items(start, end, out, cap) : r.get_text_range(ref_seq, sh, start, end, ph, pl, out, cap);
    if (threadIdx.x == 0) *n = m;
}

/* Per-document segment queries (one workgroup); out[0] = status (1 found / 0 none / 2 several markers /
 * 3 refused perspective), then by mode:
 *   0 getContainingSegment(a = pos): mt_seg_ref fields {rid, gen, offset, length, seq, client, removedSeq,
 *     removedClient, ordinal} in out[1..9]
 *   1 getPosition(a = rid, b = gen): out[1]
 *   2 posFromRelativePos' marker (a = marker-id key, b = value): its position, out[1]
 *   3 HandleCache.getHandle(a = pos): out[1]
 *   4 a remote client's position a under (ref_seq, long_client) in the local view (resolveRemoteClientPosition,
 *     mergeTree.ts:2140-2160; PermutationVector.adjustPosition, permutationvector.ts:185-196): found: out[1] =
 *     getPosition(segment) + offset, out[2] = the segment's removal flag; none: out[3] = getLength under the
 *     remote perspective, out[4] = the local length
 *   5 getMarkerFromId (a = key, b = value): mt_seg_ref fields of the marker, as mode 0
 *   6 PermutationVector.handleToPosition (a = handle, b = localSeq; permutationvector.ts:198-253): the segment
 *     whose allocated handles hold a, findReconnectionPostition(segment, localSeq) + its offset, out[1] */
template <class R>
__device__ inline void seg_fields(R& r, int32_t s, int32_t off, int32_t* res) {
    int32_t rid = r.z.rid[s], rs = r.z.rseq(s);
    res[0] = 1;
    res[1] = rid;
    res[2] = r.z.rgen[rid];
    res[3] = off;
    res[4] = r.z.len(s);
    res[5] = r.z.seq(s);
    res[6] = r.long_of_cli(s);
    res[7] = rs;
    res[8] = rs == NOREM ? 0 : r.long_of_rcli(s);
    res[9] = r.ordinal_of(s);
}
#define MT_SEGQ_N 10
template <class HT>
__global__ __launch_bounds__(WG) void k_seg(Store<HT> st, int64_t doc, int32_t mode, int32_t a, int32_t b,
                                           int32_t ref_seq, int32_t long_client, int32_t floor, int32_t* out) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int32_t res[MT_SEGQ_N] = {0, -1, 0, 0, 0, 0, 0, 0, 0, 0};
    if (persp_refused(r, ref_seq, long_client, floor)) { /* res[0] = 3: refused (MT_E_UNSUPPORTED) */
        res[0] = 3;
        if (threadIdx.x == 0)
            for (int i = 0; i < MT_SEGQ_N; i++) out[i] = res[i];
        return;
    }
    int32_t sh;
    if (long_client < 0) {
        sh = r.h.localShort;
        ref_seq = r.h.currentSeq;
    } else {
        sh = r.short_of(long_client);
        if (sh < 0) sh = 0x7fff; /* a client the replica has not seen: sequenced content only */
    }
    if (mode == 0) {
        int32_t off = 0;
        int32_t s = r.containing(a, ref_seq, sh, &off);
        if (s >= 0) seg_fields(r, s, off, res);
    } else if (mode == 1) {
        int32_t s = (a >= 0 && a < HT::S) ? r.slot_of(a, b) : -1;
        if (s >= 0) {
            res[0] = 1;
            res[1] = r.position_of(s, ref_seq, sh);
        }
    } else if (mode == 3) { /* HandleCache.getHandle(a): the PermutationSegment's start + offset, or unallocated */
        int32_t off = 0;
        int32_t s = r.containing(a, ref_seq, sh, &off);
        if (s >= 0) {
            uint32_t st = (r.z.flags(s) & RF_PERM) ? r.cold(s).toff : 0u;
            res[0] = 1;
            res[1] = st ? (int32_t)st + off : INT32_MIN;
        }
    } else if (mode == 4) {
        int32_t off = 0;
        int32_t s = r.containing(a, ref_seq, sh, &off);
        if (s >= 0) {
            res[0] = 1;
            res[1] = r.local_pos(s) + off;
            res[2] = r.z.rseq(s) != NOREM;
        } else {
            res[3] = r.length(ref_seq, sh);
            res[4] = r.length_local();
        }
    } else if (mode == 6) {
        int32_t s = -1, off = 0;
        /* assert(localSeq <= collabWindow.localSeq) (permutationvector.ts:199 -> client.ts:676): res[0] stays 0 */
        const bool inRange = b <= r.zh->localSeq;
        for (int32_t k = 0; inRange && s < 0 && r.kvalid(k); k = r.knext(k)) { /* walkAllSegments: the first match */
            int32_t n = r.leaf_at(k), c = r.nch[n];
            int32_t j = threadIdx.x;
            bool hit = false;
            int32_t q = n * MAXN + (j & (MAXN - 1));
            if (j < c && j < MAXN && (r.z.flags(q) & RF_PERM)) {
                int32_t h0 = (int32_t)r.cold(q).toff;
                hit = h0 != 0 && h0 <= a && a < h0 + r.z.len(q);
            }
            uint64_t m = r.w.ballot(hit);
            if (m) {
                s = n * MAXN + r.w.ffs(m);
                off = a - (int32_t)r.cold(s).toff;
            }
        }
        if (s >= 0) {
            res[0] = 1;
            res[1] = r.recon_pos(s, b) + off;
        }
    } else { /* modes 2 and 5: the marker whose property a (the marker-id key) is value b; res[0] = 2 if several */
        int32_t s = r.marker_by_id(a, b);
        if (s == -2) {
            res[0] = 2;
        } else if (s >= 0 && mode == 5) {
            seg_fields(r, s, 0, res);
        } else if (s >= 0) {
            res[0] = 1;
            res[1] = r.position_of(s, ref_seq, sh);
        }
    }
    if (threadIdx.x == 0)
        for (int i = 0; i < MT_SEGQ_N; i++) out[i] = res[i];
}

/* every segment's handle in walkAllSegments order (the canonical dump's record order): out[2i] = row id,
 * out[2i+1] = its generation; *n = the segment count (writes at most cap pairs) */
template <class HT>
__global__ __launch_bounds__(WG) void k_segids(Store<HT> st, int64_t doc, int32_t* out, int64_t cap, int64_t* n) {
    Replica<WaveGPU, HT> r(st.doc(doc), WaveGPU());
    int64_t base = 0;
    for (int32_t k = 0; r.kvalid(k); k = r.knext(k)) {
        int32_t lf = r.leaf_at(k), c = r.nch[lf];
        int32_t j = threadIdx.x;
        if (j < c && j < MAXN && base + j < cap) {
            int32_t rid = r.z.rid[lf * MAXN + j];
            out[2 * (base + j)] = rid;
            out[2 * (base + j) + 1] = r.z.rgen[rid];
        }
        base += c;
    }
    if (threadIdx.x == 0) *n = base;
}

/* local references: per doc their count and LocalReference.toPosition() of each (-1 detached) */
template <class HT>
__global__ __launch_bounds__(WG) void k_refpos(Store<HT> st, int64_t ndocs, int32_t rcap, int32_t* nref, int32_t* pos) {
    int64_t d = blockIdx.x;
    if (d >= ndocs) return;
    Replica<WaveGPU, HT> r(st.doc(d), WaveGPU());
    int32_t n = r.d.dstate()->nref;
    for (int32_t i = 0; i < n; i++) {
        int32_t p = r.ref_position(i);
        if (threadIdx.x == 0) pos[d * rcap + i] = p;
    }
    if (threadIdx.x == 0) nref[d] = n;
}

/* per-doc header fields: errors, stats, roofline work counters */
template <class HT>
__global__ void k_hdr(Store<HT> st, int64_t ndocs, int32_t* err, int32_t* err_op, int32_t* stats4, int64_t* work3,
                      int64_t* times2) {
    int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ndocs) return;
    const DocHdr& h = st.doc(d).t->h;
    if (times2) {
        times2[2 * d] = h.tStart;
        times2[2 * d + 1] = h.tEnd;
    }
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

struct ProfOps;

struct mt_engine {
    const ProfOps* ops = nullptr; /* the profile's launchers (one translation unit per profile) */
    /* capacity promotion (mt_engine_sync): the documents a replay left with E_CAPACITY replay again, from
     * their staged logs, in an engine of the next profile (`over`); per-document queries route there */
    bool promote = true;
    bool ran = false;                 /* a replay was launched since the last sync */
    bool fresh = true;                /* no replay since create / reset: the staged log is each replica's whole history */
    bool ran_fresh = false;           /* the last launched replay started from such a state */
    bool forwarded = false;           /* the last replay also ran the promoted documents' records in `over` */
    mt_engine* over = nullptr;
    std::vector<int32_t> pro;         /* doc -> index in `over`, -1: not promoted */
    std::vector<int64_t> pro_docs;    /* index in `over` -> doc */
    std::vector<int64_t> h_op_off, h_text_off, h_props_off, h_kv_off; /* host copies of the staged offsets */
    std::vector<int32_t> h_local;     /* start_collab's local long ids, then per doc minSeq, then currentSeq */
    mt_caps caps0 = {};               /* creation capacities */
    bool borrowed = false;            /* text / props / kv point into the parent's staged pools */
    int device;
    int64_t ndocs;
    int32_t dcap = 0; /* delta event log words per document (0: off) */
    int32_t rcap = 0; /* local references per document (0: none) */
    int32_t pcap = 0; /* PermutationVector handles per document (0: none) */
    bool fx = false;  /* delta events or local references: the client-feature replay build */
    bool loads = false; /* the staged batch holds snapshot-load records (the config-2/3 kernel's full build) */
    int profile = 0;
    int waves = 8;    /* occupancy target of the HBM-resident small-profile kernel */
    bool wide = false; /* tiled profile: the variant with the heap in HBM and the full window set (promotion target) */
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
    DevBuf ops_buf, op_off, text, text_off, props, props_off, kv, kv_off, tmp, local_ids, prof;
    DevBuf order;    /* dispatch order of the replay kernel (empty: document order) */
    bool collab = false;
    std::string err;
    /* perspective floors (persp_refused): per document, the greatest refSeq each long client has sent a
     * sequenced op under (long id, refSeq pairs), and a floor for every client (a snapshot load's currentSeq:
     * the loaded window's ops are not in the log). `staged` is built by mt_engine_submit from the staged
     * records, `applied` covers every record replayed since create / reset. */
    struct Persp {
        int32_t all = INT32_MIN;
        int32_t segk = 0; /* segment kinds the document's records inserted: 1 TextSegment, 2 SubSequence (never both) */
        std::vector<std::pair<int32_t, int32_t>> ref;
        void note(int32_t c, int32_t r) {
            for (auto& x : ref)
                if (x.first == c) {
                    if (r > x.second) x.second = r;
                    return;
                }
            ref.emplace_back(c, r);
        }
        void merge(const Persp& o) {
            if (o.all > all) all = o.all;
            segk |= o.segk;
            for (auto& x : o.ref) note(x.first, x.second);
        }
        int32_t floor(int32_t c) const {
            int32_t f = all;
            for (auto& x : ref)
                if (x.first == c && x.second > f) f = x.second;
            return f;
        }
    };
    std::vector<Persp> persp_staged, persp_applied;
    /* the replay launch's document range and stream (mt_engine_run: all documents on `stream`; the chunked
     * mt_engine_submit_run: one range per chunk, alternating between `stream` and `stream2`) */
    int64_t run_d0 = 0, run_n = -1;
    int64_t chunk = 0; /* documents per chunk of mt_engine_submit_run (0: automatic) */
    /* a staged batch of some documents only (mt_engine_submit_docs): their ids (`sub`, increasing; nsub = -1: every
     * document); the staged offsets then hold one entry per listed document */
    int64_t nsub = -1;
    DevBuf sub;
    std::vector<int64_t> h_sub;
    /* the host's value kinds (mt_engine_set_value_kinds) */
    DevBuf vkind;
    int32_t nvk = 0;
    std::vector<uint8_t> h_vkind;
    hipStream_t run_stream = nullptr;
    /* mt_engine_submit_run: the copy stream, the second compute stream, and pinned staging buffers for pageable
     * sources (each with the event of the last copy out of it) */
    hipStream_t cstream = nullptr, stream2 = nullptr;
    hipEvent_t evs = nullptr, evc = nullptr, ev2 = nullptr;
    struct Pin {
        void* p = nullptr;
        hipEvent_t ev = nullptr;
    };
    static constexpr int NPIN = 3;
    Pin pin[NPIN];
    int pin_i = 0;
};

static inline int32_t hip_fail(mt_engine* e, hipError_t st, const char* what) {
    if (e) e->err = std::string(what) + ": " + hipGetErrorString(st);
    return MT_E_HIP;
}
#define HIPCHK(e, x)                                        \
    do {                                                    \
        hipError_t st_ = (x);                               \
        if (st_ != hipSuccess) return hip_fail(e, st_, #x); \
    } while (0)

static inline int32_t launch_check(mt_engine* e, const char* what) {
    hipError_t st = hipGetLastError();
    if (st != hipSuccess) return hip_fail(e, st, what);
    return MT_OK;
}

static inline dim3 docs_grid(int64_t n) { return dim3((unsigned)n); }
static inline dim3 flat_grid(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

/* The store-dependent launches of one profile. Device pointers come from the engine's buffers. */
struct ProfOps {
    int32_t (*init)(mt_engine* e);                                    /* k_init (+ k_start_collab) */
    int32_t (*start_collab)(mt_engine* e); /* k_start_collab from local_ids (ids, minSeq, currentSeq per doc) */
    int32_t (*replay)(mt_engine* e);                                  /* k_replay over the staged batch */
    int32_t (*hdr)(mt_engine* e, int32_t* de, int32_t* deo, int32_t* ds, int64_t* dw, int64_t* dt);
    int32_t (*digest)(mt_engine* e, uint64_t* dout);
    int32_t (*dump)(mt_engine* e, int64_t doc, uint8_t* dbuf, int64_t cap, int64_t* dn);
    /* the reads take the perspective floor of persp_refused (the host's per-client refSeq bound) */
    int32_t (*length)(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t floor, int32_t* dout);
    int32_t (*text)(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t floor, int32_t start,
                    int32_t end, const uint16_t* dph, int32_t pl, uint16_t* dbuf, int64_t cap, int64_t* dn);
    int32_t (*seg)(mt_engine* e, int64_t doc, int32_t mode, int32_t a, int32_t b, int32_t ref_seq,
                   int32_t long_client, int32_t floor, int32_t* dout);
    int32_t (*refpos)(mt_engine* e, int32_t* dn, int32_t* dpos);
    int32_t (*segids)(mt_engine* e, int64_t doc, int32_t* dout, int64_t cap, int64_t* dn);
};
/* each profile's table (host functions, defined in its mt_prof_*.hip) */
const ProfOps* ops_small();
const ProfOps* ops_mat();
const ProfOps* ops_mid();
const ProfOps* ops_big();
const ProfOps* ops_huge();

template <class HT>
static inline Store<HT>& store_of(mt_engine* e) {
    if constexpr (std::is_same_v<HT, HotSmall>) return e->s0;
    else if constexpr (std::is_same_v<HT, HotMid>) return e->s1;
    else if constexpr (std::is_same_v<HT, HotBig>) return e->s2;
    else if constexpr (std::is_same_v<HT, HotMat>) return e->s3;
    else return e->s4;
}

/* one replay kernel over the staged batch (a document per workgroup) */
template <class HT, class K>
static inline int32_t launch_replay(mt_engine* e, K kern, int block = WG) {
    const int64_t n = e->run_n >= 0 ? e->run_n : e->nsub >= 0 ? e->nsub : e->ndocs;
    if (n <= 0) return MT_OK;
    const int32_t* order = e->nsub >= 0 ? (const int32_t*)e->sub.p : (const int32_t*)e->order.p;
    hipLaunchKernelGGL(kern, docs_grid(n), dim3(block), 0, e->run_stream ? e->run_stream : e->stream, store_of<HT>(e),
                       e->ndocs, (const mt_op_rec*)e->ops_buf.p, (const int64_t*)e->op_off.p, (const uint16_t*)e->text.p,
                       (const int64_t*)e->text_off.p, (const mt_props_rec*)e->props.p, (const int64_t*)e->props_off.p,
                       (const mt_kv*)e->kv.p, (const int64_t*)e->kv_off.p,
                       ReplayAux{(uint64_t*)e->prof.p, order, e->run_d0, e->nsub >= 0 ? 1 : 0,
                                 (const uint8_t*)e->vkind.p, e->nvk});
    return launch_check(e, "k_replay");
}

/* the launchers every profile shares (replay is the profile's own) */
template <class HT>
struct Launch {
    static int32_t init(mt_engine* e) {
        Store<HT>& st = store_of<HT>(e);
        hipLaunchKernelGGL((k_init<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs);
        int32_t rc = launch_check(e, "k_init");
        if (rc || !e->collab) return rc;
        hipLaunchKernelGGL((k_start_collab<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, st, e->ndocs,
                           (const int32_t*)e->local_ids.p);
        return launch_check(e, "k_start_collab");
    }
    static int32_t start_collab(mt_engine* e) {
        hipLaunchKernelGGL((k_start_collab<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, store_of<HT>(e),
                           e->ndocs, (const int32_t*)e->local_ids.p);
        return launch_check(e, "k_start_collab");
    }
    static int32_t hdr(mt_engine* e, int32_t* de, int32_t* deo, int32_t* ds, int64_t* dw, int64_t* dt) {
        hipLaunchKernelGGL((k_hdr<HT>), flat_grid(e->ndocs), dim3(256), 0, e->stream, store_of<HT>(e), e->ndocs, de,
                           deo, ds, dw, dt);
        return launch_check(e, "k_hdr");
    }
    static int32_t digest(mt_engine* e, uint64_t* dout) {
        hipLaunchKernelGGL((k_digest<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, store_of<HT>(e), e->ndocs,
                           dout);
        return launch_check(e, "k_digest");
    }
    static int32_t dump(mt_engine* e, int64_t doc, uint8_t* dbuf, int64_t cap, int64_t* dn) {
        hipLaunchKernelGGL((k_dump<HT>), dim3(1), dim3(WG), 0, e->stream, store_of<HT>(e), doc, dbuf, cap, dn);
        return launch_check(e, "k_dump");
    }
    static int32_t length(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t floor,
                          int32_t* dout) {
        hipLaunchKernelGGL((k_length<HT>), dim3(1), dim3(WG), 0, e->stream, store_of<HT>(e), doc, ref_seq,
                           long_client, floor, dout);
        return launch_check(e, "k_length");
    }
    static int32_t text(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t floor, int32_t start,
                        int32_t end, const uint16_t* dph, int32_t pl, uint16_t* dbuf, int64_t cap, int64_t* dn) {
        hipLaunchKernelGGL((k_text<HT>), dim3(1), dim3(WG), 0, e->stream, store_of<HT>(e), doc, ref_seq, long_client,
                           floor, start, end, dph, pl, dbuf, cap, dn);
        return launch_check(e, "k_text");
    }
    static int32_t seg(mt_engine* e, int64_t doc, int32_t mode, int32_t a, int32_t b, int32_t ref_seq,
                       int32_t long_client, int32_t floor, int32_t* dout) {
        hipLaunchKernelGGL((k_seg<HT>), dim3(1), dim3(WG), 0, e->stream, store_of<HT>(e), doc, mode, a, b, ref_seq,
                           long_client, floor, dout);
        return launch_check(e, "k_seg");
    }
    static int32_t refpos(mt_engine* e, int32_t* dn, int32_t* dpos) {
        hipLaunchKernelGGL((k_refpos<HT>), docs_grid(e->ndocs), dim3(WG), 0, e->stream, store_of<HT>(e), e->ndocs,
                           e->rcap, dn, dpos);
        return launch_check(e, "k_refpos");
    }
    static int32_t segids(mt_engine* e, int64_t doc, int32_t* dout, int64_t cap, int64_t* dn) {
        hipLaunchKernelGGL((k_segids<HT>), dim3(1), dim3(WG), 0, e->stream, store_of<HT>(e), doc, dout, cap, dn);
        return launch_check(e, "k_segids");
    }
    static ProfOps table(int32_t (*replay)(mt_engine*)) {
        return ProfOps{init, start_collab, replay, hdr, digest, dump, length, text, seg, refpos, segids};
    }
};
