/*
 * mt_core.h — the merge-tree replay core, single source for the HIP kernel (one wavefront per
 * document) and for the host build that the generator and the CPU spec tests use.
 *
 * Representation ("leaf slabs"). The reference keeps a B-tree of MergeBlocks with at most
 * MaxNodesInBlock-1 = 7 children (mergeTree.ts:329-382). Segment boundaries depend on the exact
 * leaf-block partition (zamboni merges only inside a leaf, mergeTree.ts:1322-1398; inserts tie
 * at leaf ends, 2464-2478), so the block skeleton is kept, but flattened for a wavefront:
 *   - every block is a node; a LEAF node owns a slab of 8 row slots (7 children + the transient
 *     8th the reference uses before splitting, mergeTree.ts:2487-2503);
 *   - rows are stored structure-of-arrays by slot (slot = node * 8 + child index);
 *   - `lorder` lists leaf nodes in document order, so document order = (lorder[k], j);
 *   - interior nodes keep parent / child lists only for split propagation and pack.
 * Position resolution replaces the root-to-leaf walk with a wavefront prefix scan of
 * perspective-visible lengths over all slots in document order (nodeLength, 1692-1732); the
 * PartialSequenceLengths summaries are not needed because the scan sums leaves directly.
 *
 * Wave abstraction: W::N lanes execute every function; control flow and all "scalar" values are
 * uniform across lanes. Cross-lane work goes through W (exclusive scan, ballot, broadcast). The
 * host build uses W::N = 1 so the same code runs serially.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifndef MT_A32 /* element addressing by 32-bit offsets from the block base (HotT::at32), per array group: 1 leaf lines,
                  2 row ids / leaves / generations / kids, 4 cold rows, 8 the free-id stack and the membership logs */
#define MT_A32 0
#endif

#include <type_traits>

#include "../../include/mt_oplog.h"

#ifdef __HIPCC__
#ifdef MT_NO_FORCE_INLINE /* analysis builds: let the compiler choose what to inline */
#define MT_HD __host__ __device__
#else
#define MT_HD __host__ __device__ __attribute__((always_inline))
#endif
#define MT_DEV __device__
#else
#define MT_HD
#define MT_DEV
#endif

namespace mt {

enum : int32_t {
    UNIVERSAL_SEQ = 0,
    UNASSIGNED_SEQ = -1,
    NOREM = INT32_MIN, /* rseq when not removed */
    NONE = INT32_MIN,
    MAXN = 8,          /* MaxNodesInBlock (mergeTree.ts:333) */
    GRANULARITY = 256, /* TextSegmentGranularity (mergeTree.ts:1093) */
    NOVL = 8,          /* removedClientOverlap entries per row held inline; more go to the overflow pool */
    OVB = 64,          /* overflow blocks per document (8 overlap entries each) */
};
enum : uint8_t { LOCAL_CLIENT = 0xFF }; /* short id of LocalClientId (-1) */
/* A short id is a byte of the leaf lines: slots 0..252 name clients (s2l: their long ids), RETIRED_CLIENT marks a
 * row whose client's slot was recycled (its long id then lives in the document's retired-client table, by row id),
 * 0xFE is a client the replica has not seen. See Replica::reclaim_shorts. */
enum : uint8_t { RETIRED_CLIENT = 0xFD, MAX_SLOTS = 0xFD };
enum : uint16_t { FREE_SLOT = 0xFFFF }; /* s2l of a recycled slot (no long id takes 0xFFFF: NonCollabClient) */

/* error codes (mt_engine.h MT_E_*) */
enum : int32_t {
    E_OK = 0,
    E_INSERT_FAILED = 1, /* mergeTree.ts:2243-2249 */
    E_ASSERT = 2,
    E_INVALID_RANGE = 3, /* reserved: a local op getValidOpRange rejects (client.ts:486-548) is a no-op */
    E_UNSUPPORTED = 4,
    E_CAPACITY = 5,
};

/* row flag bits */
enum : uint8_t {
    RF_MARKER = 1,
    RF_PROPS = 2, /* properties !== undefined (and propertyManager exists) */
    RF_LSEQ = 4,
    RF_LRSEQ = 8,
    RF_OVL = 16, /* removedClientOverlap is non-empty (its list lives in the cold row) */
    RF_NLK = 32, /* RF_NL is known: a cache of the text's last unit, so zamboni rarely reads it */
    RF_NL = 64,  /* the text ends with "\n" (textSegment.ts:64 canAppend) */
    RF_PERM = 128, /* PermutationSegment (permutationvector.ts:36-122): no text, handle unallocated */
    RF_NOTEXT = RF_MARKER | RF_PERM,
};

/* runtime capacities that are not part of the LDS image */
struct Caps {
    int32_t acap; /* text arena half-size (UTF-16 units); arena holds 2 halves */
    int32_t mcap; /* segment-group membership log entries */
    int32_t gcap; /* pending segment groups (local ops in flight) */
    int32_t dcap; /* delta event log words (0 = delta events off; mt_oplog.h MT_DELTA_*) */
    int32_t rcap; /* local references (0 = none; mt_oplog.h MT_OP_REF) */
    int32_t pcap; /* PermutationVector handle-table entries (0 = none; mt_oplog.h MT_OP_NOOP | MT_OPF_LOCAL) */
};

/* delta event stream state at the head of a document's delta region (mt_oplog.h) */
struct alignas(16) DState {
    int64_t n;   /* words emitted (may exceed dcap: later words are hashed, not stored) */
    uint64_t h;  /* FNV-1a-64 of every emitted word */
    int32_t seq; /* seq of the record being applied (-1: local edit) */
    int32_t on;  /* 0 while a snapshot-load record applies */
    int32_t nref;  /* local references created */
    int32_t ncoll; /* segments holding a LocalReferenceCollection (LColl) */
    int32_t hlen;  /* PermutationVector's HandleTable: the length of its `handles` array (handletable.ts:23) */
    int32_t _pad[3];
};
/* a local reference (localReference.ts:20-117): the row id of its segment (-1: detached), its offset
 * in the segment and its ReferenceType */
struct alignas(16) LRef {
    int32_t rid, off, type;
    int32_t ek; /* the refsByOffset entry it sits in was created by addLocalRef (0: has an `at` list) or by
                   a tombstone slide (1: `before` / `after` only) */
    /* a removed reference (rid <= REF_FROZEN) also keeps the refsByOffset ENTRY it left: removeLocalRef only
     * splices the reference out of the entry's lists (localReference.ts:225-264), so the entry stays defined,
     * with its shape, in its collection and moves with that collection's splits and appends as the live
     * references do: erid = the row id of the collection holding it now (-1: gone with the collection), eoff
     * its offset there, ekd its kind (as ek) */
    int32_t erid, eoff, ekd, _pad;
};
enum : int32_t {
    REF_DETACHED = -1,
    REF_SAVED = -2, /* on a row the current remove took (mergeTree.ts:2673-2676) */
    REF_GHOST = -3, /* addLocalReference threw: refsByOffset[offset].at is undefined (localReference.ts:195-201) */
    /* removeLocalReference took it out of its segment's collection (localReference.ts:225-264): the
     * LocalReference keeps `segment` and `offset` (toPosition still answers) but no longer follows splits,
     * appends or slides. Stored as rid = REF_FROZEN - (the row id), ek = the row's generation then. */
    REF_FROZEN = -16,
};
/* a segment's LocalReferenceCollection: its row id and refsByOffset.length, which is what an append adds
 * to the offsets of the references it takes over (localReference.ts:211-223). That length follows the
 * JavaScript array, not the segment: set at creation, cut by a split, extended by appends and by
 * assignments past its end, and left alone when the segment grows by a reference-free append. */
struct LColl {
    int32_t rid, len;
};

/* per-document scalar header */
struct DocHdr {
    int32_t root, nleaf, freeHead, nfree;
    int32_t currentSeq, minSeq, localSeq, collaborating;
    int32_t localShort, localLong, nclients, nextSid;
    int32_t heapN, memN, gqHead, gqN;
    int32_t arenaTop, arenaSide, err, errOp;
    int32_t nkeys, opsDone, hwSlots, hwHeap;
    int32_t nrows, seqOps, nfreeRid, gcEpoch; /* rows in the table; sequenced msgs applied */
    int32_t localLen;      /* root.cachedLength: Client.getLength() (client.ts:1051) */
    int32_t heapTop;       /* maxSeq of the heap's root (valid when heapN > 0) */
    int32_t loadPos;       /* snapshot load: the next position of the open loadBody batch (mt_oplog.h) */
    int32_t ovTop, ovFree; /* overlap overflow pool: next never-used block, free-list head (0 = none) */
    int32_t gidNext;       /* id of the next pending segment group (ids increase along the queue) */
    int32_t mkMask;        /* property key slots an annotate changed on a marker (marker_keys_annotated) */
    int32_t ndv; /* derived property values (mt_oplog.h MT_VALUE_DERIVED): bits 0-7 the STRCAT entries, 8-15 the
                    consensus-object entries, bit 16 a NaN was made; nonzero bits 8-16: some row may hold a value
                    matchProperties never matches. Bit 24 (DV_RUN): a SubSequence document (mt_oplog.h MT_SEG_RUN: its
                    text-bearing rows are SubSequence rows, whose canAppend has MaxRun 128 and no newline rule) */
    int64_t sumR, sumW; /* roofline counters: sum over sequenced msgs of rows before the op and
                           rows written by it (BASELINE.md A(op) = 16 R + 32 W) */
    int64_t tStart, tEnd; /* the last replay kernel's start / end for this document (s_memrealtime ticks) */
};
enum : int32_t { DV_RUN = 1 << 24 };
/* the int32 fields of DocHdr the replica keeps in registers while it runs; the rarely used ones
 * (nclients, nextSid, errOp, nkeys, hwSlots, gcEpoch, loadPos, ovTop, ovFree, and since round 2 root,
 * nfree, freeHead, nfreeRid, hwHeap, seqOps) stay in the image and are read and written there (z.h),
 * which keeps the replay loop's scalar registers for the fields every event touches. The last six
 * took the config-3 kernel from 227 to 79 VGPR spills and from 164.8M to 184.7M ops/s
 * (profiles/r02_spill_variants.txt). Since round 3 the replay kernels stage the image's header in LDS
 * (Replica::zh), so eight more fields the local-edit, ack, arena and zamboni paths use (localSeq, gqHead,
 * gqN, memN, arenaSide, heapTop, sumR, sumW) live there too: SGPR spills 1,637 -> 686 and +3 % on config 3
 * (profiles/r03_ab_*.json). */
#define MT_HDR_FIELDS(X)                                                                          \
    X(nleaf) X(currentSeq) X(minSeq) X(collaborating)   \
    X(localShort) X(localLong) X(heapN) X(arenaTop) X(err) \
    X(opsDone) X(nrows) X(localLen)
/* the register header: only these fields, so a stale read of one that lives in the image does not compile */
struct RegHdr {
#define MT_HF(f) int32_t f;
    MT_HDR_FIELDS(MT_HF)
#undef MT_HF
};

/* Cold per-row data, indexed by a row id that does not move when the row's slot moves. K = the
 * profile's property key slots per document. */
template <int K>
struct alignas(16) ColdRowT {
    int32_t lseq, lrseq;
    uint32_t toff; /* text offset in the arena; a marker's refType */
    uint8_t prw;   /* pendingRewriteCount */
    uint8_t gc;    /* arena-GC epoch that last moved this row's text (0 = never) */
    uint16_t ovx;  /* first overflow block of removedClientOverlap past the inline 8 (0 = none) */
    uint16_t pv[K]; /* property values per doc key slot (0 = absent); 16-byte aligned: compared and
                       cleared 16 bytes at a time. pv, pk and prw are meaningful only while the row's
                       RF_PROPS flag is set (add_props clears them when it sets the flag). */
    uint64_t ovl;  /* removedClientOverlap: the first 8 short ids (+1), push order */
    uint8_t pk[K];  /* pendingKeyUpdateCount per key slot */
};
static_assert(sizeof(ColdRowT<8>) % 16 == 0 && sizeof(ColdRowT<24>) % 16 == 0, "cold rows are 16-byte granular");
static_assert(offsetof(ColdRowT<8>, lrseq) == 4 && offsetof(ColdRowT<8>, toff) == 8 && offsetof(ColdRowT<8>, prw) == 12 &&
                  offsetof(ColdRowT<8>, ovx) == 14 && offsetof(ColdRowT<24>, ovx) == 14,
              "insert_segments writes lseq, lrseq, toff and {prw, gc, ovx} as one 16-byte unit");
static_assert((2 * 8) % 16 == 0 && (2 * 24) % 16 == 0, "pv spans whole 16-byte units");

/* Position index of the large-document profile ("tiled", config 4: >100k live rows).
 *
 * Leaf order is a two-level rope instead of one dense array (a dense `lorder` costs O(leaves) per
 * leaf split): chunks of <= 64 leaves, kept in document order by `cord` (chunk ids by position).
 * Each row is STABLE (settled at the current MSN and not removed: visible with its full length in
 * every perspective the protocol can use, refSeq >= minSeq, and in the local one), W (in the
 * collaboration window: seq or removedSeq above minSeq, or local-pending; evaluated exactly per
 * op) or DEAD (removed at or below minSeq: invisible everywhere). Summaries hold only STABLE
 * lengths: `lst` per leaf, `cst` per chunk position — the flattened, window-free part of the
 * reference's PartialSequenceLengths (partialLengths.ts:218-274 `fromLeaves` splits a block's rows
 * the same way: segments at or below minSeq fold into `minLength`, newer ones into partials).
 * The W rows are a small set (`wrid`) re-evaluated under each op's perspective and scattered onto
 * the chunk summaries; a position search is then chunk scan -> leaf scan -> row scan. */
template <int N, bool T>
struct TileState {
    static constexpr int NCH = 1, WCAP = 1;
};
template <int N>
struct TileState<N, true> {
    static constexpr int CH = 64;       /* leaves per chunk */
    static constexpr int NCH = N / 64;  /* chunk capacity (a 1M-op config-4 document peaks at ~2,100 chunks);
                                           the tiled kernel stages the chunk arrays in LDS */
    static constexpr int WCAP = 4096;   /* window-set capacity (rows; under 100 in use at lag 64, ~1,200 at lag 8,000) */
    int32_t nchunk, wN, cfree, nfreeChunk;
    int32_t lst[N];         /* leaf node -> sum of its STABLE rows' lengths */
    int32_t lch[N];         /* leaf node -> chunk id */
    uint8_t lix[N];         /* leaf node -> index in its chunk */
    uint8_t xf[N * 8];      /* slot -> XF_* state of the row it holds */
    uint16_t ph[N * 8];     /* slot -> a 16-bit hash of its row's property values (RF_PROPS rows; moves with the row):
                               scour's append test reads the cold values only where the hashes match */
    int32_t cord[NCH];      /* chunk ids in document order */
    int32_t cst[NCH];       /* sum of lst over the chunk at each position */
    static constexpr int NG = NCH / 64; /* chunk groups: positions [64 g, 64 g + 64) */
    int32_t gst[NG];        /* sum of cst over each group (a chunk search scans the groups, then one group) */
    int32_t cpos[NCH];      /* chunk id -> position (free chunks: next free id) */
    int32_t ccnt[NCH];      /* chunk id -> leaf count */
    int32_t cleaf[NCH][CH]; /* chunk id -> its leaves in order */
    int32_t cls[NCH][CH];   /* chunk id -> its leaves' lst, in the same order (a chunk search reads one line) */
    int32_t wrid[WCAP];     /* window set: row ids */
    uint8_t wgen[WCAP];     /* their generations when added */
    int32_t wslot[WCAP];    /* the slot each was last seen in (a hint: rows move; checked before use) */
    /* host-build scratch of a position search (the GPU kernel uses LDS instead) */
    int32_t sdel[NCH];
    int32_t sgdel[NG];
    int32_t swcp[WCAP], swvs[WCAP];
    uint8_t swlx[WCAP];
};
enum : uint8_t { XF_STABLE = 1, XF_W = 2 };

/* Hot per-document state with compile-time capacities: everything the per-op scans and the
 * tree skeleton touch. */
template <int N_, int C_ = 256, bool TILED_ = false, int K_ = 8>
struct HotT {
    static constexpr int K = K_;     /* property key slots per document */
    typedef ColdRowT<K_> Cold;
    static constexpr int N = N_;     /* B-tree nodes */
    static constexpr int S = N_ * 8; /* row slots (8 per leaf node) */
    static constexpr int H = N_ + 64; /* zamboni heap entries (config 3 peaks at 109) */
    static constexpr int C = C_;     /* clients */
    static constexpr bool TILED = TILED_;
    typedef typename std::conditional<TILED_, int32_t, int16_t>::type IX; /* node / row-id type */
    typedef TileState<N_, TILED_> TL;
    DocHdr h;
    /* The scan columns of one leaf's 8 slots share one 128-byte line (leaf-major SoA): a
     * perspective scan that visits a leaf touches one cache line, not one line per column.
     * len is 0 in every slot that holds no row (rows always have len >= 1), so a scan needs no
     * child count; the int32 columns are read 4 slots at a time (16-byte reads). */
    struct alignas(128) Leaf {
        int32_t len[8], seq[8], rseq[8];
        uint8_t b[8][4]; /* per slot {cli, rcli, flags, ng}: a quad's byte columns in one 16-byte read */
    };
    Leaf lf[N];
    /* Per-lane element addresses as the image base + a 32-bit byte offset (the offset in 32-bit arithmetic, then
     * zero-extended): the GPU compiler keeps the one base pointer (an SGPR pair) and issues each load / store with a
     * 32-bit per-lane offset (global_load ... v_off, s_base), where a member array indexed directly becomes a
     * 64-bit address per lane from a base of its own (a hoisted SGPR pair per array, which the 8-waves-per-SIMD
     * kernel spills). A small negative index stays inside the document's block, as before. */
    template <class T>
    MT_HD T& at32(int32_t off) { return *(T*)((uint8_t*)this + (uint64_t)(uint32_t)off); }
    MT_HD static int32_t lfo(int s, int f) { return (int32_t)offsetof(HotT, lf) + (s >> 3) * 128 + f + (s & 7) * 4; }
#if MT_A32 & 1
    MT_HD int32_t& len(int s) { return at32<int32_t>(lfo(s, 0)); }
    MT_HD int32_t& seq(int s) { return at32<int32_t>(lfo(s, 32)); }
    MT_HD int32_t& rseq(int s) { return at32<int32_t>(lfo(s, 64)); }
    MT_HD uint8_t& cli(int s) { return at32<uint8_t>(lfo(s, 96)); }
    MT_HD uint8_t& rcli(int s) { return at32<uint8_t>(lfo(s, 97)); }
    MT_HD uint8_t& flags(int s) { return at32<uint8_t>(lfo(s, 98)); }
    MT_HD uint8_t& ng(int s) { return at32<uint8_t>(lfo(s, 99)); }
    MT_HD const int32_t* bytes4(int s) { return &at32<const int32_t>(lfo(s, 96)); }
#else
    MT_HD int32_t& len(int s) { return lf[s >> 3].len[s & 7]; }
    MT_HD int32_t& seq(int s) { return lf[s >> 3].seq[s & 7]; }
    MT_HD int32_t& rseq(int s) { return lf[s >> 3].rseq[s & 7]; }
    MT_HD uint8_t& cli(int s) { return lf[s >> 3].b[s & 7][0]; }
    MT_HD uint8_t& rcli(int s) { return lf[s >> 3].b[s & 7][1]; }
    MT_HD uint8_t& flags(int s) { return lf[s >> 3].b[s & 7][2]; }
    MT_HD uint8_t& ng(int s) { return lf[s >> 3].b[s & 7][3]; }
    MT_HD const int32_t* bytes4(int s) { return (const int32_t*)&lf[s >> 3].b[s & 7][0]; }
#endif
    IX rid[S];   /* slot -> row id (stable identity of a segment; cold data index) */
    IX rleaf[S]; /* row id -> leaf node currently holding it */
    uint8_t rgen[S]; /* row id -> generation, bumped when the id is freed */
#if MT_A32 & 2
    MT_HD IX& RID(int s) { return at32<IX>((int32_t)offsetof(HotT, rid) + s * (int32_t)sizeof(IX)); }
    MT_HD IX& RLEAF(int r) { return at32<IX>((int32_t)offsetof(HotT, rleaf) + r * (int32_t)sizeof(IX)); }
    MT_HD uint8_t& RGEN(int r) { return at32<uint8_t>((int32_t)offsetof(HotT, rgen) + r); }
    MT_HD IX& KIDS(int i) { return at32<IX>((int32_t)offsetof(HotT, kids) + i * (int32_t)sizeof(IX)); }
#else
    MT_HD IX& RID(int s) { return rid[s]; }
    MT_HD IX& RLEAF(int r) { return rleaf[r]; }
    MT_HD uint8_t& RGEN(int r) { return rgen[r]; }
    MT_HD IX& KIDS(int i) { return kids[i]; }
#endif
    IX nparent[N], lorder[N], lpos[N]; /* lorder / lpos: dense leaf order (not used when TILED) */
    IX kids[N * 8];
    int8_t nchild[N], nlevel[N], nscour[N];
    int8_t _pad[(16 - (3 * N) % 16) % 16];
    int32_t hseq[H];
    IX hrid[H];  /* segment (row id) queued for scouring */
    uint8_t hgen[H];  /* its row-id generation when queued: a mismatch means it was unlinked */
    uint16_t s2l[C];  /* short client id -> long id (client.ts:637-661) */
    uint8_t l2s[C];   /* long id (< C) -> short id, 0xFF = not seen yet */
    uint16_t keys[K_]; /* property key id of each doc key slot */
    uint16_t ovn[OVB];  /* overlap overflow pool: next block of a chain (0 = end) / of the free list */
    int8_t _pad2[(16 - (2 * K_ + 2 * OVB) % 16) % 16];
    uint64_t ovp[OVB];  /* 8 more removedClientOverlap entries (short id + 1) per block */
    /* derived property values (incr / consensus, mt_oplog.h MT_VALUE_DERIVED): STRCAT entries {base id | k << 16}
     * (String(base) + "undefined" x k) and consensus objects' seqs, interned by content per document */
    int32_t dvs[128];
    int32_t dvc[128];
    TileState<N_, TILED_> tl;
};

/* LDS-sized profile for config 2/3 documents (39.5 KB <= 160 KB / 4: 4 documents per CU; the
 * node high-water of config-3 documents has a tail reaching ~180 nodes) and larger
 * global-memory profiles. */
typedef HotT<192> HotSmall;
typedef HotT<640> HotMat; /* config 5: PermutationVector replicas peak at ~540 nodes */
typedef HotT<2048, 256, false, 24> HotMid; /* the larger profiles hold 24 property keys per document */
typedef HotT<16384, 256, false, 24> HotBig;
typedef HotT<(1 << 18), 256, true, 24> HotHuge; /* config 4: tiled position index, 32-bit ids (1M-op docs: ~112k nodes) */

struct alignas(16) I4 {
    int32_t x[4];
};
struct alignas(4) B4 {
    uint8_t x[4];
};
/* 16-byte / 4-byte column reads. memcpy, not a pointer cast: the columns are members of the leaf
 * line struct, and an I4/B4-typed load of them would be "no alias" for type-based alias analysis,
 * letting the compiler move it above a store to the same slot. */
MT_HD inline I4 ld4(const int32_t* p) { /* p 16-byte aligned */
    I4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 16), sizeof v);
    return v;
}
MT_HD inline void st4(void* p, const I4& v) { /* p 16-byte aligned */
    __builtin_memcpy(__builtin_assume_aligned(p, 16), &v, sizeof v);
}
MT_HD inline bool eq4(const I4& a, const I4& b) {
    return a.x[0] == b.x[0] && a.x[1] == b.x[1] && a.x[2] == b.x[2] && a.x[3] == b.x[3];
}
MT_HD inline B4 ldb4(const uint8_t* p) { /* p 4-byte aligned */
    B4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), sizeof v);
    return v;
}

MT_HD constexpr int64_t align256c(int64_t x) { return (x + 255) & ~(int64_t)255; }

/* Per-document view: the hot image (LDS or global) plus the document's global block. The block is
 * [hot image | cold rows | free row-id stack | text arena (2 halves) | membership log gid | rid |
 * pending-group ring]; the first three offsets are compile-time constants of the profile and the
 * rest follow from the caps, so a replica keeps one block pointer (and the caps) in registers
 * instead of one pointer per region. */
template <class HT>
struct Doc {
    typedef typename HT::IX IX_;
    HT* t;      /* hot image: the block itself, or its LDS copy */
    uint8_t* b; /* the document's global block */
    Caps caps;
    static constexpr int64_t OFF_COLD = align256c((int64_t)sizeof(HT));
    static constexpr int64_t OFF_FRID = align256c(OFF_COLD + (int64_t)sizeof(typename HT::Cold) * HT::S);
    /* retired clients by row id: {client long id, removedClient long id} of a row whose short-id byte is
     * RETIRED_CLIENT (written by reclaim_shorts, copied by splits, read by the dump and the segment queries) */
    static constexpr int64_t OFF_RCL = align256c(OFF_FRID + (int64_t)sizeof(typename HT::IX) * HT::S);
    static constexpr bool HAS_RCL = HT::N > 640; /* the profiles that recycle short ids (Replica::RECLAIM) */
    static constexpr int64_t OFF_ARENA = align256c(OFF_RCL + (HAS_RCL ? 4 * (int64_t)HT::S : 0));
    MT_HD static int64_t off_mgid(const Caps& c) { return OFF_ARENA + align256c(4 * (int64_t)c.acap); }
    MT_HD static int64_t off_mrid(const Caps& c) { return off_mgid(c) + align256c(4 * (int64_t)c.mcap); }
    MT_HD static int64_t off_gq(const Caps& c) { return off_mrid(c) + align256c(4 * (int64_t)c.mcap); }
    /* client-feature region (only when c.dcap > 0 or c.rcap > 0): DState, dcap delta-log words, rcap
     * local references */
    MT_HD static bool has_fx(const Caps& c) { return c.dcap > 0 || c.rcap > 0 || c.pcap > 0; }
    MT_HD static int64_t off_gql(const Caps& c) { return off_gq(c) + align256c(4 * (int64_t)c.gcap); }
    MT_HD static int64_t off_dl(const Caps& c) { return off_gql(c) + align256c(4 * (int64_t)c.gcap); }
    MT_HD static int64_t off_refs(const Caps& c) {
        return off_dl(c) + (int64_t)sizeof(DState) + ((4 * (int64_t)c.dcap + 15) & ~(int64_t)15);
    }
    MT_HD static int64_t off_coll(const Caps& c) { return off_refs(c) + (int64_t)sizeof(LRef) * c.rcap; }
    MT_HD static int32_t coll_cap(const Caps& c) { return 4 * c.rcap; }
    /* PermutationVector's HandleTable (handletable.ts:19-87): handles[0] = the free-list head, then pcap
     * entries (0 = allocated, else the next free handle) */
    MT_HD static int64_t off_ht(const Caps& c) {
        return (off_coll(c) + (int64_t)sizeof(LColl) * coll_cap(c) + 15) & ~(int64_t)15;
    }
    MT_HD static int64_t stride(const Caps& c) {
        return has_fx(c) ? align256c(off_ht(c) + 4 * ((int64_t)c.pcap + 1)) : off_dl(c);
    }
    MT_HD DState* dstate() const { return (DState*)(b + off_dl(caps)); }
    MT_HD int32_t* dlog() const { return (int32_t*)(b + off_dl(caps) + (int64_t)sizeof(DState)); }
    MT_HD LRef* refs() const { return (LRef*)(b + off_refs(caps)); }
    MT_HD LColl* colls() const { return (LColl*)(b + off_coll(caps)); }
    MT_HD int32_t* ht() const { return (int32_t*)(b + off_ht(caps)); }
    MT_HD typename HT::Cold* cold() const { return (typename HT::Cold*)(b + OFF_COLD); } /* HT::S records */
    /* elements by 32-bit offsets from the block base (HotT::at32) */
    template <class T>
    MT_HD T& at32(int32_t off) const { return *(T*)(b + (uint64_t)(uint32_t)off); }
#if MT_A32 & 4
    MT_HD typename HT::Cold& COLD(int32_t r) const {
        return at32<typename HT::Cold>((int32_t)OFF_COLD + r * (int32_t)sizeof(typename HT::Cold));
    }
#else
    MT_HD typename HT::Cold& COLD(int32_t r) const { return cold()[r]; }
#endif
#if MT_A32 & 8
    MT_HD IX_& FRID(int32_t i) const { return at32<IX_>((int32_t)OFF_FRID + i * (int32_t)sizeof(IX_)); }
    MT_HD int32_t& MGID(int32_t i) const { return at32<int32_t>((int32_t)off_mgid(caps) + 4 * i); }
    MT_HD int32_t& MRID(int32_t i) const { return at32<int32_t>((int32_t)off_mrid(caps) + 4 * i); }
    MT_HD int32_t& GQ(int32_t i) const { return at32<int32_t>((int32_t)off_gq(caps) + 4 * i); }
    MT_HD int32_t& GQL(int32_t i) const { return at32<int32_t>((int32_t)off_gql(caps) + 4 * i); }
#else
    MT_HD IX_& FRID(int32_t i) const { return frid()[i]; }
    MT_HD int32_t& MGID(int32_t i) const { return mgid()[i]; }
    MT_HD int32_t& MRID(int32_t i) const { return mrid()[i]; }
    MT_HD int32_t& GQ(int32_t i) const { return gq()[i]; }
    MT_HD int32_t& GQL(int32_t i) const { return gql()[i]; }
#endif
    MT_HD typename HT::IX* frid() const { return (typename HT::IX*)(b + OFF_FRID); } /* free row-id stack */
    MT_HD uint16_t* arena() const { return (uint16_t*)(b + OFF_ARENA); } /* 2 * acap */
    MT_HD uint32_t& RCL(int32_t r) const { return ((uint32_t*)(b + OFF_RCL))[r]; } /* lo: client, hi: removedClient */
    MT_HD int32_t* mgid() const { return (int32_t*)(b + off_mgid(caps)); }
    MT_HD int32_t* mrid() const { return (int32_t*)(b + off_mrid(caps)); } /* row id of each membership entry */
    MT_HD int32_t* gq() const { return (int32_t*)(b + off_gq(caps)); }
    MT_HD int32_t* gql() const { return (int32_t*)(b + off_gql(caps)); } /* each queued group's SegmentGroup.localSeq */
};

/* Op pools of one document. */
struct Pools {
    const mt_op_rec* ops;
    int64_t nops;
    const uint16_t* text;
    const mt_props_rec* props;
    const mt_kv* kv;
    const uint8_t* vkind = nullptr; /* per value id its MT_VKIND_* (mt_engine_set_value_kinds), nvk entries */
    int32_t nvk = 0;
};

/* Phase clock for the profiling build only (-DMT_PROF, tools/phase_profile.py): shader-clock
 * cycles accumulated per phase in registers and written out per document. */
enum { PH_APPLY, PH_ZAMBONI, PH_FIND, PH_MAP, PH_SPLIT, PH_ACK, PH_TEXT, PH_HEAP, PH_SCOUR, PH_PACK, PH_APPEND,
       PH_CAND, PH_S1, PH_S2, PH_S3, PH_P1, PH_P2, PH_INSROW, PH_LEAFINS,
       PH_WIN, PH_TFIND, PH_LFIND, PH_ROPE, PH_RESTAT, /* tiled profile */
       PH_VISIT, PH_PLACE, /* a range op's visit; an insert's row set-up after placement */
       PH_C_INS, PH_C_RANGE, PH_C_WROWS, PH_C_WMISS, PH_C_SCOUR, PH_C_PACK, /* event counts, not cycles */
       PH_C_HEAPN, PH_C_POP, PH_C_PUSH,
       PH_N };
#if defined(MT_PROF) && defined(__HIP_DEVICE_COMPILE__)
struct ProfScope { /* no live register across the scope: the LDS counter takes -start at entry and +end at exit */
    uint64_t* acc;
    __device__ ProfScope(uint64_t* a) : acc(a) {
        if (acc) *acc -= __builtin_amdgcn_s_memtime();
    }
    __device__ ~ProfScope() {
        if (acc) *acc += __builtin_amdgcn_s_memtime();
    }
};
/* the clocks live in LDS (the replay kernels point prof at a __shared__ array; other kernels leave it null): an
 * array of PH_N 64-bit counters held in registers spilled the profiled config-3 kernel to 900 B of scratch per lane */
#ifdef MT_PROF_NOSCOPE
#define MT_PROF_SCOPE(i)
#else
#define MT_PROF_SCOPE(i) ProfScope _ps##i(prof ? &prof[i] : nullptr)
#endif
#define MT_PROF_COUNT(i, n) (prof ? (void)(prof[i] += (uint64_t)(n)) : (void)0)
#else
#define MT_PROF_SCOPE(i)
#define MT_PROF_COUNT(i, n)
#endif

/* ------------------------------------------------------------------------------------------
 * Replica: all operations of one document replica, executed by one wave.
 * ---------------------------------------------------------------------------------------- */
/* DL: this build emits delta events (mt_oplog.h) when the engine has a delta log; the hot replay
 * kernels are built without (DL = false), so the emission costs them no registers or code */
/* LOAD: applies snapshot-load records (mt_oplog.h MT_OP_RELOAD / COLLAB / APPEND); the plain config-2/3 replay
 * kernel is built without them (its scalar registers: SGPR spills 1,321 -> 1,041, +2.2 % on config 3, r04s) and
 * the engine runs a batch that holds any with the full build */
/* NARROW: the tiled kernel's variant that keeps the zamboni heap in LDS beside a narrower window set (MT_NARROW_H /
 * MT_NARROW_W entries, mt_kernels.h k_replay_tiled); a document that outgrows either latches E_CAPACITY and replays
 * again in the wide variant (capacity promotion, mt_replay.hip) */
#ifndef MT_NARROW_W
#define MT_NARROW_W 2048
#endif
#ifndef MT_NARROW_H
#define MT_NARROW_H 2048
#endif
template <class W, class HT, bool DL = false, bool LOAD = true, bool NARROW = false>
struct Replica {
    typedef typename HT::IX IX;
    static constexpr bool TILED = HT::TILED;
    static constexpr int WCAPR = NARROW ? MT_NARROW_W : HT::TL::WCAP; /* window-set entries */
    static constexpr int HCAPR = NARROW ? MT_NARROW_H : HT::H;        /* zamboni heap entries */
    /* short-id recycling (reclaim_shorts) is built into the larger profiles only: a config-2/3/5 document that meets
     * its 254th client latches E_CAPACITY and replays again in HotMid (capacity promotion, mt_replay.hip), so the
     * small kernels carry none of it */
    static constexpr bool RECLAIM = Doc<HT>::HAS_RCL;
    Doc<HT> d;
    HT& z; /* the hot image */
    W w;

    RegHdr h; /* the header fields held in registers (SGPRs on the GPU) while the replica runs; the rest: zh */
#ifdef MT_PROF
    uint64_t* prof = nullptr; /* LDS (the replay kernels), or none */
#endif

    /* The tree skeleton's small per-node arrays and the zamboni heap are reached through these
     * pointers: they point into the image by default, and the HBM-resident GPU kernel points them
     * at LDS copies for the duration of a replay (latency-critical, 3.5 KB per document). */
    /* the image's rarely-used header fields (DocHdr, z.h) and the client tables (l2s / s2l): reached through
     * these, so the HBM-resident replay kernel can stage them in LDS with the skeleton (every sequenced
     * message reads l2s and bumps seqOps: no vector-memory round trip for either) */
    DocHdr* zh;
    uint16_t* keys; /* the document's property key table (z.keys; the tiled replay kernel stages it in LDS) */
    uint8_t* l2s;
    uint16_t* s2l;
    IX* lo;  /* lorder */
    IX* lp;  /* lpos */
    IX* npar;
    int8_t* nch;
    int8_t* nlev;
    int8_t* nsc;
    int32_t* hsq;
    IX* hrd;
    uint8_t* hgn;
    /* tiled profile: scratch of a position search — per-chunk window deltas (all zero between
     * searches) and per window row its chunk position, leaf index and perspective length. The image
     * holds host copies; the GPU kernel points them at LDS. */
    int32_t* cdel;
    int32_t* wcp;
    int32_t* wvs;
    uint8_t* wlx;
    /* tiled profile: the rope's chunk arrays (document order, summaries, positions, leaf counts) and the
     * window set, reached through these: they point into the image by default, and the tiled replay kernel
     * points them at LDS copies for the duration of a replay (every position search and summary update
     * reads them: ~3 dependent vector-memory round trips per search fewer) */
    int32_t* tcord;
    int32_t* tcst;
    int32_t* tgst; /* chunk-group sums of tcst (TileState::gst) */
    int32_t* gdel; /* chunk-group sums of cdel */
    int32_t* tcpos;
    int32_t* tccnt;
    int32_t* twrid;
    uint8_t* twgen;
    int32_t* twslot;
    int64_t cur; /* index of the record being applied in the current Pools (snapshot reload reads ahead) */
    int32_t* pfcur = nullptr; /* tiled kernel: where the prefetch helper waves read `cur` (LDS) */
    /* tiled kernel built with MT_WIN_HELPER: the LDS mailbox of the second wave that evaluates the window set's second
     * block of entries while this wave does the first (win_pass, win_helper) */
    struct WinMail {
        int32_t req, done, n, refSeq, client, minSeq, local, quit;
        int32_t s[64], lc[64], lx[64], len[64], rseq[64], v[64], cp[64], st[64];
    };
    WinMail* wm = nullptr;
    int32_t wmseq = 0;
    /* an upper bound of every maxSeq in the zamboni heap (INT32_MAX: unknown), set when a replay starts: an
     * entry at or above it cannot move up, so heap_add appends it without reading its ancestors */
    int32_t hmax = INT32_MAX;
    int32_t zq = 0, zms = 0; /* zamboniSegments calls queued by the record being applied, the first's minSeq */
    bool runOnly = false;      /* range_op_tiled: find and split only, leaving the run's first / last slot in */
    int32_t runA = -1, runB = -1; /* runA / runB for remove_run (no visit) */
    const uint8_t* vk = nullptr; /* the value kinds of the replay's Pools (combine_value) */
    int32_t nvk = 0;

    MT_HD Replica(const Doc<HT>& doc, const W& wave)
        : d(doc), z(*doc.t), w(wave), zh(&z.h), keys(z.keys), l2s(z.l2s), s2l(z.s2l), lo(z.lorder), lp(z.lpos), npar(z.nparent), nch(z.nchild), nlev(z.nlevel),
          nsc(z.nscour), hsq(z.hseq), hrd(z.hrid), hgn(z.hgen), cdel(nullptr), wcp(nullptr), wvs(nullptr),
          wlx(nullptr), tcord(nullptr), tcst(nullptr), tgst(nullptr), gdel(nullptr), tcpos(nullptr), tccnt(nullptr), twrid(nullptr), twgen(nullptr), twslot(nullptr),
          cur(0) {
        if constexpr (TILED) {
            cdel = z.tl.sdel;
            wcp = z.tl.swcp;
            wvs = z.tl.swvs;
            wlx = z.tl.swlx;
            tcord = z.tl.cord;
            tcst = z.tl.cst;
            tgst = z.tl.gst;
            gdel = z.tl.sgdel;
            tcpos = z.tl.cpos;
            tccnt = z.tl.ccnt;
            twrid = z.tl.wrid;
            twgen = z.tl.wgen;
            twslot = z.tl.wslot;
        }
        load_hdr();
    }

    MT_HD void load_hdr() {
#define MT_HF(f) h.f = w.uniform(zh->f);
        MT_HDR_FIELDS(MT_HF)
#undef MT_HF

    }
    /* write the register header back to the image; every mutating entry point ends with it */
    MT_HD void commit() {
#define MT_HF(f) zh->f = h.f;
        MT_HDR_FIELDS(MT_HF)
#undef MT_HF

        w.sync();
    }

    MT_HD typename HT::Cold& cold(int32_t s) const { return d.COLD(z.RID(s)); }
    /* cold row of slot a into slot b's row, 16 bytes per load / store */
    MT_HD void copy_cold(int32_t b, int32_t a) {
        const int32_t* src = (const int32_t*)&cold(a);
        int32_t* dst = (int32_t*)&cold(b);
        I4 v[sizeof(typename HT::Cold) / 16];
        for (int i = 0; i < (int)(sizeof(typename HT::Cold) / 16); i++) v[i] = ld4(src + 4 * i);
        for (int i = 0; i < (int)(sizeof(typename HT::Cold) / 16); i++) st4(dst + 4 * i, v[i]);
    }

    /* the first error latches (the reference throws); apply() records the failing record's index in
     * zh->errOp once, after the record, instead of a store at every one of the many inlined fail sites */
    MT_HD void fail(int32_t e) {
        if (h.err == E_OK) h.err = e;
    }

    /* ---- node allocation ------------------------------------------------------------- */
    MT_HD int32_t alloc_node(int8_t level) {
        int32_t n = zh->freeHead;
        if (n < 0) {
            fail(E_CAPACITY);
            return -1;
        }
        zh->freeHead = npar[n];
        zh->nfree--;
        npar[n] = -1;
        nch[n] = 0;
        nlev[n] = level;
        nsc[n] = -1; /* needsScour undefined */
        if constexpr (TILED) z.tl.lst[n] = 0;
        clear_slots(n * MAXN, MAXN);
        return n;
    }
    /* mark `cnt` slots from `s` as holding no row */
    MT_HD void clear_slots(int32_t s, int32_t cnt) {
        w.sync();
        for (int32_t b = 0; b < cnt; b += W::N) {
            int32_t i = b + w.lane();
            if (i < cnt) z.len(s + i) = 0;
        }
        w.sync();
    }
    MT_HD void free_node(int32_t n) {
        npar[n] = (IX)zh->freeHead;
        nch[n] = 0;
        zh->freeHead = n;
        zh->nfree++;
    }

    /* ---- init -------------------------------------------------------------------------- */
    MT_HD void init() {
        /* node 0 = empty root leaf (initialNode, mergeTree.ts:1159-1163) */
        int32_t ncap = HT::N;
        for (int32_t b = 0; b < ncap; b += W::N) {
            int32_t n = b + w.lane();
            if (n < ncap) {
                npar[n] = (IX)(n + 1 < ncap ? n + 1 : -1);
                nch[n] = 0;
                nlev[n] = 0;
                nsc[n] = -1;
            }
        }
        for (int32_t b = 0; b < HT::S; b += W::N) {
            int32_t i = b + w.lane();
            if (i < HT::S) {
                d.FRID(i) = (IX)(HT::S - 1 - i);
                z.RGEN(i) = 0;
                z.len(i) = 0;
                z.seq(i) = 0;
                z.rseq(i) = 0;
                z.cli(i) = 0;
                z.rcli(i) = 0;
                z.flags(i) = 0;
                z.ng(i) = 0;
                z.RID(i) = 0;
                if constexpr (TILED) z.tl.xf[i] = 0;
            }
        }
        w.sync();
        if constexpr (TILED) rope_init();
        zh->nfreeRid = HT::S;
        zh->gcEpoch = 0;
        zh->freeHead = 1;
        zh->nfree = ncap - 1;
        zh->root = 0;
        npar[0] = -1;
        lo[0] = 0;
        lp[0] = 0;
        h.nleaf = 1;
        h.currentSeq = 0;
        h.minSeq = 0;
        zh->localSeq = 0;
        h.collaborating = 0;
        h.localShort = -1; /* collabWindow.clientId = LocalClientId */
        h.localLong = -1;
        zh->nclients = 0;
        zh->nextSid = 1;
        h.heapN = 0;
        zh->memN = 0;
        zh->gqHead = 0;
        zh->gqN = 0;
        h.arenaTop = 0;
        zh->arenaSide = 0;
        h.err = 0;
        zh->errOp = -1;
        zh->nkeys = 0;
        h.opsDone = 0;
        zh->hwSlots = 0;
        zh->hwHeap = 0;
        h.nrows = 0;
        zh->seqOps = 0;
        zh->sumR = 0;
        zh->sumW = 0;
        h.localLen = 0;
        zh->heapTop = 0;
        zh->loadPos = 0;
        zh->gidNext = 0;
        zh->mkMask = 0;
        zh->ndv = 0;
        zh->ovTop = 1; /* block 0 is the null link */
        zh->ovFree = 0;
        for (int32_t b = 0; b < HT::C; b += W::N) {
            int32_t i = b + w.lane();
            if (i < HT::C) l2s[i] = 0xFF;
        }
        if (Doc<HT>::has_fx(d.caps)) {
            DState* st = d.dstate();
            st->n = 0;
            st->h = MT_FNV_OFFSET;
            st->seq = 0;
            st->on = 1;
            st->nref = 0;
            st->ncoll = 0;
            st->hlen = 1; /* handles = [1] (handletable.ts:23) */
            d.ht()[0] = 1;
        }
        w.sync();
    }

    /* ---- PermutationVector handles (permutationvector.ts:36-122, 157-183, 338-363; handletable.ts) ----
     * A PermutationSegment row keeps its `start` handle in the cold row's toff (0 = Handle.unallocated:
     * valid handles are >= 1). The document's HandleTable (off_ht) allocates lazily at
     * getAllocatedHandle and takes the handles of every unlinked segment back, in the order of the
     * maintenance callbacks. Client-feature build with caps.pcap > 0 only. */
    MT_HD bool ht_on() const {
        if constexpr (DL)
            return d.caps.pcap > 0;
        else
            return false;
    }
    /* HandleTable.allocate (handletable.ts:35-40); 0 and E_CAPACITY when the table is full */
    MT_HD int32_t ht_alloc() {
        int32_t* t = d.ht();
        DState* st = d.dstate();
        int32_t f = t[0], len = st->hlen;
        if (f > d.caps.pcap) {
            fail(E_CAPACITY);
            return 0;
        }
        int32_t nx = f < len ? t[f] : f + 1; /* handles[free] ?? free + 1 */
        w.sync();
        t[0] = nx;
        t[f] = 0;
        if (f >= len) st->hlen = f + 1;
        w.sync();
        return f;
    }
    /* HandleTable.load(handleTableData) (handletable.ts:84-86) of PermutationVector.load (permutationvector.ts:270-
     * 275): entries [pos1, pos1 + text_len / 2) of the summary's `handles` array (each as two UTF-16 units of the
     * text pool, low then high), whose length is pos2 (mt_oplog.h MT_NOOP_HTLOAD) */
    MT_HD void ht_load(const mt_op_rec& op, const Pools& p) {
        if (!ht_on()) {
            fail(E_UNSUPPORTED);
            return;
        }
        int32_t first = op.pos1, len = op.pos2, n = op.text_len / 2;
        if (first < 0 || len < 1 || first + n > len) {
            fail(E_ASSERT);
            return;
        }
        if (len - 1 > d.caps.pcap) {
            fail(E_CAPACITY);
            return;
        }
        int32_t* t = d.ht();
        const uint16_t* u = p.text + op.text_off;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            if (i < n) t[first + i] = (int32_t)((uint32_t)u[2 * i] | ((uint32_t)u[2 * i + 1] << 16));
        }
        w.sync();
        d.dstate()->hlen = len;
        w.sync();
    }
    /* onMaintenance UNLINK (permutationvector.ts:338-363): HandleTable.free (56-59) of start .. start + len - 1
     * in increasing order */
    MT_HD void ht_free_range(int32_t start, int32_t len) {
        int32_t* t = d.ht();
        int32_t nx = t[0];
        w.sync();
        for (int32_t b = 0; b < len; b += W::N) {
            int32_t i = b + w.lane();
            if (i < len) t[start + i] = i == 0 ? nx : start + i - 1;
        }
        if (len > 0) t[0] = start + len - 1;
        w.sync();
    }
    /* the handles of a row zamboni unlinks */
    MT_HD void ht_unlinked(int32_t rid, int32_t len) {
        if ((int32_t)d.COLD(rid).toff != 0) ht_free_range((int32_t)d.COLD(rid).toff, len);
    }
    /* PermutationVector.getAllocatedHandle(pos) (157-183) in the local view: the handle of the row at pos
     * (getMaybeHandle: start + offset when allocated), else walkSegments(pos, pos + 1, splitRange) splits a
     * one-row segment out at pos and HandleTable.allocate()s its start */
    /* MergeTree.mapRange's splitRange (mergeTree.ts:2830-2838) in the local view (Client.walkSegments,
     * client.ts:276-285): ensureIntervalBoundary at a truthy start, then at a truthy end (one call site) */
    MT_HD void split_range(int32_t a, int32_t b) {
#pragma clang loop unroll(disable)
        for (int32_t i = 0; i < 2; i++) {
            int32_t p = i ? b : a;
            if (p) ensure_boundary(p, h.currentSeq, h.localShort);
        }
    }
    MT_HD void alloc_handle(int32_t pos) {
        if (!ht_on()) {
            fail(E_UNSUPPORTED);
            return;
        }
        if (pos < 0 || pos >= h.localLen) { /* assert(0 <= pos && pos < this.getLength()) */
            fail(E_ASSERT);
            return;
        }
        int32_t off = 0;
        int32_t s = containing(pos, h.currentSeq, h.localShort, &off);
        if (s < 0 || !(z.flags(s) & RF_PERM)) {
            fail(s < 0 ? E_ASSERT : E_UNSUPPORTED);
            return;
        }
        if (cold(s).toff != 0) return; /* isHandleValid(start + offset) */
        split_range(pos, pos + 1); /* walkSegments(pos, pos + 1, ..., splitRange = true) */
        s = containing(pos, h.currentSeq, h.localShort, &off);
        if (s < 0 || off != 0 || z.len(s) != 1) {
            fail(E_ASSERT);
            return;
        }
        int32_t hnd = ht_alloc();
        if (hnd > 0) cold(s).toff = (uint32_t)hnd;
    }

    /* ---- delta events (§8 f3; stream format in mt_oplog.h): the reference's
     * mergeTreeDeltaCallback / mergeTreeMaintenanceCallback, in firing order. Only engines created
     * with caps.dcap > 0 emit; the state lives in the document's delta region, not in registers. */
    MT_HD bool dl_on() const {
        if constexpr (!DL)
            return false;
        else
            return d.caps.dcap > 0 && d.dstate()->on;
    }
    MT_HD void dput(int32_t v) {
        DState* st = d.dstate();
        int64_t n = st->n;
        uint64_t hh = st->h;
        for (int i = 0; i < 4; i++) {
            hh ^= (uint8_t)((uint32_t)v >> (8 * i));
            hh *= MT_FNV_PRIME;
        }
        if (n < d.caps.dcap) d.dlog()[n] = v;
        st->n = n + 1;
        st->h = hh;
    }
    MT_HD void dhead(int32_t op) {
        dput(op);
        dput(d.dstate()->seq);
    }
    MT_HD void dtail(int32_t nseg) { /* end of the segment list, then its count */
        dput(MT_DELTA_END);
        dput(nseg);
    }
    MT_HD void dseg(int32_t pos, int32_t len) {
        dput(pos);
        dput(len);
        dput(0);
    }
    /* ---- local references (§8 f4; mt_oplog.h MT_OP_REF, localReference.ts) ------------------- */
    MT_HD bool refs_on() const {
        if constexpr (!DL)
            return false;
        else
            return d.caps.rcap > 0 && d.dstate()->nref > 0;
    }
    /* the references on row id `from` at offset >= o0 move to row id `to`, offset + delta (split:
     * LocalReferenceCollection.split, localReference.ts:225-241; append: 211-223; to < 0 marks them) */
    MT_HD int32_t refs_move(int32_t from, int32_t o0, int32_t to, int32_t delta) {
        LRef* R = d.refs();
        int32_t n = d.dstate()->nref, moved = 0;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            bool mv = i < n && R[i].rid == from && R[i].off >= o0;
            if (mv) {
                R[i].rid = to;
                R[i].off += delta;
            }
            moved += w.sum(mv ? 1 : 0);
            /* the entries removed references left ride along; a collection that goes away (to < 0: the
             * segment was removed or unlinked) takes them with it */
            if (i < n && R[i].rid <= REF_FROZEN && R[i].erid == from && R[i].eoff >= o0) {
                R[i].erid = to >= 0 ? to : -1;
                R[i].eoff += delta;
            }
        }
        w.sync();
        return moved;
    }
    /* the LocalReferenceCollection of row id `rid`: its index in the table, or -1 */
    MT_HD int32_t coll_find(int32_t rid) {
        LColl* C = d.colls();
        int32_t n = d.dstate()->ncoll;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            uint64_t m = w.ballot(i < n && C[i].rid == rid);
            if (m) return b + W::ffs(m);
        }
        return -1;
    }
    /* `new LocalReferenceCollection(segment)` unless it has one: refsByOffset.length = its length now */
    MT_HD int32_t coll_get(int32_t rid, int32_t len) {
        int32_t i = coll_find(rid);
        if (i >= 0) return i;
        DState* st = d.dstate();
        i = st->ncoll;
        if (i >= Doc<HT>::coll_cap(d.caps)) {
            fail(E_CAPACITY);
            return -1;
        }
        LColl c = {rid, len};
        d.colls()[i] = c;
        st->ncoll = i + 1;
        return i;
    }
    MT_HD void coll_drop(int32_t rid) { /* segment.localRefs = undefined, or the segment left the tree */
        refs_move(rid, INT32_MIN, REF_DETACHED, 0); /* the entries of removed references go with it */
        int32_t i = coll_find(rid);
        if (i < 0) return;
        DState* st = d.dstate();
        int32_t n = st->ncoll - 1;
        d.colls()[i] = d.colls()[n];
        st->ncoll = n;
    }
    MT_HD int32_t refs_on_row(int32_t rid) { /* LocalReferenceCollection.refCount of the row's collection */
        LRef* R = d.refs();
        int32_t n = d.dstate()->nref, c = 0;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            c += w.sum(i < n && R[i].rid == rid ? 1 : 0);
        }
        return c;
    }
    /* splitAt -> localRefs.split(pos, next) (mergeTree.ts:561-563, localReference.ts:225-241): a
     * non-empty collection hands its references at offsets >= pos, and refsByOffset.splice(pos) of its
     * array, to a new collection of the right part */
    MT_HD void refs_split(int32_t lrid, int32_t rrid, int32_t pos) {
        int32_t i = coll_find(lrid);
        if (i < 0 || refs_on_row(lrid) == 0) return;
        int32_t cl = d.colls()[i].len;
        refs_move(lrid, pos, rrid, -pos);
        int32_t j = coll_get(rrid, 0);
        if (j < 0) return;
        d.colls()[j].len = cl > pos ? cl - pos : 0;
        if (cl > pos) d.colls()[i].len = pos;
    }
    /* TextSegment / PermutationSegment.append -> LocalReferenceCollection.append(seg1, seg2)
     * (textSegment.ts:78, permutationvector.ts:98, localReference.ts:126-133, 211-223), before seg1's
     * length (len1) changes; seg2 leaves the tree */
    MT_HD void refs_append(int32_t rid1, int32_t rid2, int32_t len1) {
        int32_t j = coll_find(rid2);
        if (j >= 0 && refs_on_row(rid2) > 0) {
            int32_t cl2 = d.colls()[j].len;
            int32_t i = coll_get(rid1, len1);
            if (i < 0) return;
            j = coll_find(rid2); /* the table may have moved */
            int32_t cl1 = d.colls()[i].len;
            refs_move(rid2, INT32_MIN, rid1, cl1);
            d.colls()[i].len = cl1 + cl2;
        }
        coll_drop(rid2);
    }
    /* the kind (LRef.ek) of the refsByOffset entry at `off` of row `rid`'s collection, -1 if none */
    MT_HD int32_t entry_kind(int32_t rid, int32_t off) {
        LRef* R = d.refs();
        int32_t n = d.dstate()->nref, k = -1;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            uint64_t m = w.ballot(i < n && R[i].rid == rid && R[i].off == off);
            if (m && k < 0) k = R[b + W::ffs(m)].ek;
            uint64_t e = w.ballot(i < n && R[i].rid <= REF_FROZEN && R[i].erid == rid && R[i].eoff == off);
            if (e && k < 0) k = R[b + W::ffs(e)].ekd; /* an entry whose references were all removed */
        }
        return k;
    }
    /* new LocalReference(segment, offset) + addLocalReference for getContainingSegment(pos) (local view) */
    MT_HD void add_ref(int32_t pos, int32_t type) {
        DState* st = d.dstate();
        int32_t n = st->nref;
        if (n >= d.caps.rcap) {
            fail(E_CAPACITY);
            return;
        }
        int32_t off = 0;
        int32_t s = containing(pos, h.currentSeq, h.localShort, &off);
        LRef r = {s >= 0 ? (int32_t)z.RID(s) : REF_DETACHED, s >= 0 ? off : 0, type, 0, -1, 0, 0, 0};
        if (s >= 0 && entry_kind(r.rid, off) == 1) { /* the reference's addLocalRef throws here: the tree */
            r.rid = REF_GHOST;                            /* is untouched and the reference is not kept */
            d.refs()[n] = r;
            st->nref = n + 1;
            return;
        }
        if (s >= 0) { /* addLocalRef: refsByOffset[offset] = ... (localReference.ts:190-202) */
            int32_t i = coll_get(r.rid, z.len(s));
            if (i < 0) return;
            if (d.colls()[i].len < off + 1) d.colls()[i].len = off + 1;
        }
        d.refs()[n] = r;
        st->nref = n + 1;
    }
    /* Client.removeLocalReference (client.ts:299-301) -> MergeTree.removeLocalReference (mergeTree.ts:
     * 2761-2769) -> LocalReferenceCollection.removeLocalRef (localReference.ts:225-264) of reference i: found
     * in its segment's refsByOffset[offset] lists, it leaves the collection (refCount--; the array keeps its
     * length; hierRefCount only counts labelled references, which MT_OP_REF does not make). A detached
     * reference (segment undefined: the reference's call throws before touching the tree), one whose add
     * threw, or one already removed is not in any collection: no-op. */
    MT_HD void remove_ref(int32_t i) {
        if (i < 0 || i >= d.dstate()->nref) {
            fail(E_ASSERT);
            return;
        }
        LRef r = d.refs()[i];
        if (r.rid < 0) return;
        if (w.lane() == 0) {
            d.refs()[i].rid = REF_FROZEN - r.rid;
            d.refs()[i].ek = z.RGEN(r.rid);
            d.refs()[i].erid = r.rid; /* the entry it leaves stays (localReference.ts:225-264) */
            d.refs()[i].eoff = r.off;
            d.refs()[i].ekd = r.ek;
        }
        w.sync();
    }
    /* the slot of a reference's segment, -1 when it has none in the tree (detached, ghost, or a removed
     * reference whose segment left the tree: appended into its neighbour or unlinked, `parent` undefined) */
    MT_HD int32_t ref_slot(const LRef& r) {
        if (r.rid >= 0) return slot_of(r.rid, -1);
        if (r.rid <= REF_FROZEN) return slot_of(REF_FROZEN - r.rid, r.ek);
        return -1;
    }
    /* after a remove took rows holding references (markRangeRemoved, mergeTree.ts:2703-2732): under the
     * op's perspective, SlideOnRemove references go to offset 0 of the segment at `start`
     * (addBeforeTombstones) or, past the end, to the last offset of the last segment (addAfterTombstones);
     * the others, or all of them in an empty document, detach */
    MT_HD void refs_slide(int32_t start, int32_t refSeq, int32_t client) {
        int32_t L = length(refSeq, client), tgt = REF_DETACHED, toff = 0, off = 0, ci = -1, need = 0;
        if (start < L) {
            int32_t s = containing(start, refSeq, client, &off);
            if (s >= 0) {
                tgt = z.RID(s);
                ci = coll_get(tgt, z.len(s));
                need = 1; /* refsByOffset[0] */
            }
        } else if (L > 0) {
            int32_t s = containing(L - 1, refSeq, client, &off);
            if (s >= 0) {
                tgt = z.RID(s);
                toff = z.len(s) - 1;
                ci = coll_get(tgt, z.len(s));
                need = z.len(s); /* refsByOffset[cachedLength - 1] */
            }
        }
        LRef* R = d.refs();
        int32_t n = d.dstate()->nref, nslide = 0;
        int32_t ek = tgt >= 0 ? entry_kind(tgt, toff) : -1; /* sliding into an existing entry keeps its kind */
        if (ek < 0) ek = 1;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            bool slide = false;
            if (i < n && R[i].rid == REF_SAVED) {
                slide = (R[i].type & MT_REF_SLIDE_ON_REMOVE) && tgt >= 0;
                R[i].rid = slide ? tgt : REF_DETACHED;
                R[i].off = slide ? toff : 0;
                if (slide) R[i].ek = ek;
            }
            nslide += w.sum(slide ? 1 : 0);
        }
        w.sync();
        if (nslide > 0 && ci >= 0 && d.colls()[ci].len < need) d.colls()[ci].len = need;
    }
    MT_HD int32_t kprev(int32_t k) const { /* the leaf position before k (k > 0) */
        if constexpr (TILED)
            return (k & 63) ? k - 1 : ((((k >> 6) - 1) << 6) | (tccnt[tcord[(k >> 6) - 1]] - 1));
        else
            return k - 1;
    }
    /* Client.insertAtReferencePositionLocal (client.ts:217-245) -> MergeTree.insertAtReferencePosition
     * (mergeTree.ts:2033-2130): split the reference's segment at its offset unless the offset or the
     * segment's local length is 0, walk left over zero-length rows (leftExcursion, 2313-2344) taking
     * every one breakTie(0, 0, ...) accepts, and insert the new local segment right before that row. */
    /* true if the insert happens: at leaf coordinate *atT (the caller's insert_segments) */
    MT_HD bool insert_at_ref(const mt_op_rec& op, int32_t* atT) {
        if (op.pos1 < 0 || op.pos1 >= d.dstate()->nref) {
            fail(E_ASSERT);
            return false;
        }
        LRef r = d.refs()[op.pos1];
        if ((r.rid < 0 && r.rid > REF_FROZEN) || seg_len(op) <= 0)
            return false; /* DetachedPosition / a zero-length segment: no-op */
        int32_t s = ref_slot(r);
        if (s < 0) { /* a removed reference whose segment left the tree: not modelled */
            if (r.rid <= REF_FROZEN) fail(E_UNSUPPORTED);
            return false;
        }
        int32_t rs0 = z.rseq(s);
        int32_t off = (rs0 != NOREM && rs0 != 0) ? 0 : r.off; /* getOffset() */
        if (off != 0 && local_len(s) != 0) {
            /* Past the segment's end (an append adds refsByOffset.length, not the length, to the offsets
             * it takes over, localReference.ts:211-223) a text segment splits off an empty segment, which
             * split_row models. A PermutationSegment would take a negative length and grow its left part
             * (permutationvector.ts:103-114), and a Marker does not split, so the reference's
             * assert(splitSeg.next) throws (mergeTree.ts:2082-2083): neither is modelled. */
            if (off >= z.len(s) && (z.flags(s) & RF_NOTEXT)) {
                fail(E_UNSUPPORTED);
                return false;
            }
            int32_t rs = -1;
            if (split_row(kpos(s / MAXN) * MAXN + (s & (MAXN - 1)), off, &rs) < 0 || rs < 0) return false;
            s = rs;
        }
        int32_t st = s, k = kpos(s / MAXN), j = s & (MAXN - 1);
        for (;;) {
            if (j == 0) {
                if (k == 0) break;
                k = kprev(k);
                j = nch[leaf_at(k)];
                continue;
            }
            j--;
            int32_t q = leaf_at(k) * MAXN + j;
            if (local_len(q) != 0) break;
            if (break_tie(q, h.currentSeq, h.localShort)) st = q;
        }
        *atT = kpos(st / MAXN) * MAXN + (st & (MAXN - 1));
        return true;
    }
    /* LocalReference.toPosition (localReference.ts:62-68): getPosition(segment) + getOffset() (0 on a
     * removed segment: `removedSeq` truthy), -1 when detached */
    MT_HD int32_t ref_position(int32_t i) {
        LRef r = d.refs()[i];
        if (r.rid == REF_GHOST) return -2;
        int32_t s = ref_slot(r);
        if (s < 0) return -1;
        int32_t rs = z.rseq(s);
        return local_pos(s) + (rs != NOREM && rs != 0 ? 0 : r.off);
    }

    /* Client.getPosition(segment) (client.ts:291): the local view */
    MT_HD int32_t local_pos(int32_t s) { return position_of(s, h.currentSeq, h.localShort); }
    /* the propertyDeltas addProperties (segmentPropertiesManager.ts:35-111) returns for row s and this
     * annotate, read before the row changes: nd, then (key << 16 | previous value) by key id */
    MT_HD bool prop_delta(int32_t s, int32_t kid, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t seq, bool collab,
                          int32_t* val) {
        const bool rewrite = comb == MT_COMBINE_REWRITE;
        bool has = z.flags(s) & RF_PROPS;
        int32_t cv = 0, pd = 0;
        if (has)
            for (int32_t k = 0; k < zh->nkeys; k++)
                if (keys[k] == kid) {
                    cv = cold(s).pv[k];
                    pd = cold(s).pk[k];
                }
        bool inNew = false, truthy = false;
        for (int32_t j = 0; j < nkv; j++)
            if (kv[j].key == kid) {
                inNew = true;
                truthy = kv[j].value != 0 && !(kv[j].value & MT_VALUE_FALSY);
            }
        bool in = false, del = false;
        if (rewrite && cv != 0 && !truthy && (seq == UNASSIGNED_SEQ || pd == 0)) { /* rewrite deletes it */
            in = del = true;
            *val = cv;
        }
        /* shouldModifyKey: a combining op modifies every key (segmentPropertiesManager.ts:59-65) */
        if (inNew && (comb >= MT_COMBINE_INCR || !(collab && seq != UNASSIGNED_SEQ && pd != 0))) { /* deltas[key] = previous ?? null */
            in = true;
            *val = del ? 0 : cv;
        }
        return in;
    }
    MT_HD void prop_deltas(int32_t s, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t seq, bool collab) {
        if ((z.flags(s) & RF_PROPS) && cold(s).prw > 0 && seq != UNASSIGNED_SEQ && collab) {
            dput(-1); /* outstanding local rewrites: addProperties returns undefined */
            return;
        }
        for (int pass = 0; pass < 2; pass++) {
            int32_t last = -1, nd = 0;
            for (;;) { /* candidate keys (the doc's key slots and the op's keys) in id order */
                int32_t best = 0x7fffffff;
                for (int32_t k = 0; k < zh->nkeys; k++)
                    if (keys[k] > last && keys[k] < best) best = keys[k];
                for (int32_t j = 0; j < nkv; j++)
                    if (kv[j].key > last && kv[j].key < best) best = kv[j].key;
                if (best == 0x7fffffff) break;
                last = best;
                int32_t v = 0;
                if (!prop_delta(s, best, kv, nkv, comb, seq, collab, &v)) continue;
                nd++;
                if (pass) dput((int32_t)(((uint32_t)best << 16) | ((uint32_t)v & 0xFFFF)));
            }
            if (!pass) dput(nd);
        }
    }

    /* ---- clients (client.ts:637-661) --------------------------------------------------- */
    MT_HD int32_t short_of(int32_t longId) {
        if ((uint32_t)longId < (uint32_t)HT::C) {
            int32_t s = l2s[longId];
            return s == 0xFF ? -1 : s;
        }
        const int32_t n = zh->nclients;
        if constexpr (!RECLAIM) {
            for (int32_t i = 0; i < n; i++)
                if (s2l[i] == longId) return i;
            return -1;
        }
        for (int32_t b = 0; b < n; b += W::N) { /* a wave pass per 64 slots (long ids past the l2s table) */
            int32_t i = b + w.lane();
            uint64_t m = w.ballot(i < n && (int32_t)s2l[i] == longId);
            if (m) return b + W::ffs(m);
        }
        return -1;
    }
    /* client.ts:637-661 getOrAddShortClientId. The reference numbers clients without bound; here a client takes a
     * slot (0..252), and when every slot is taken the slots no row of the collaboration window needs are recycled
     * (reclaim_shorts) — so a document may see any number of clients, at most 253 of them with rows in the window
     * at once (E_CAPACITY past that). */
    MT_HD int32_t get_or_add_short(int32_t longId) {
        int32_t s = short_of(longId);
        if (s >= 0) return s;
        int32_t n = zh->nclients;
        int32_t slot = -1;
        if (n < MAX_SLOTS && n < HT::C) {
            slot = n;
            zh->nclients = n + 1;
        } else {
            if constexpr (RECLAIM) {
                slot = free_slot();
                if (slot < 0 && reclaim_shorts()) slot = free_slot();
            }
            if (slot < 0) {
                fail(E_CAPACITY);
                return 0;
            }
        }
        s2l[slot] = (uint16_t)longId;
        if ((uint32_t)longId < (uint32_t)HT::C) l2s[longId] = (uint8_t)slot;
        return slot;
    }
    MT_HD int32_t free_slot() {
        const int32_t n = zh->nclients;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            uint64_t m = w.ballot(i < n && s2l[i] == FREE_SLOT);
            if (m) return b + W::ffs(m);
        }
        return -1;
    }
    /* Recycle the short ids no row of the collaboration window needs. A short id is only ever compared for
     * equality, and only where a row's seq or removedSeq lies in the window (above minSeq, or local-pending): a
     * settled row is visible, or removed, under every perspective the protocol admits (refSeq >= minSeq), whatever
     * its client (the visibility predicate, mergeTree.ts:1692-1732; breakTie compares seqs). So the slots of clients
     * with no window row, no removedClientOverlap entry and not the local client are freed; a settled row holding
     * one keeps its long ids in the retired-client table (Doc::RCL, by row id) and the byte RETIRED_CLIENT, which
     * no client's byte equals. Returns whether a slot was freed. Rare (a document's 254th client), rolled. */
    MT_HD bool reclaim_shorts() {
        uint64_t act[4] = {0, 0, 0, 0};
        auto mark = [&](uint32_t b) {
            if (b < MAX_SLOTS) act[b >> 6] |= 1ull << (b & 63);
        };
        if (h.localShort >= 0) mark((uint32_t)h.localShort);
        const int32_t minSeq = h.minSeq;
        /* the values lanes hold, each distinct one marked once (a ballot loop, no atomics) */
        auto mark_lanes = [&](bool has, uint32_t v) {
            uint64_t m = w.ballot(has);
            while (m) {
                uint32_t x = (uint32_t)w.bcast((int32_t)v, W::ffs(m));
                mark(x);
                has = has && v != x;
                m = w.ballot(has);
            }
        };
#pragma clang loop unroll(disable)
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            const int32_t n = leaf_at(k), c = nch[n];
            for (int32_t j0 = 0; j0 < c; j0 += W::N) { /* a lane per row of the leaf */
                const int32_t j = j0 + w.lane();
                const bool row = j < c;
                const int32_t s = n * MAXN + (row ? j : 0);
                int32_t sq = 0, rs = NOREM;
                uint32_t b4 = 0;
                if (row) {
                    sq = z.seq(s);
                    rs = z.rseq(s);
                    b4 = ld_bytes4(s);
                }
                const bool rem = rs != NOREM;
                const bool win = row && (sq == UNASSIGNED_SEQ || sq > minSeq ||
                                         (rem && (rs == UNASSIGNED_SEQ || rs > minSeq)) || (((b4 >> 16) & 0xFF) & RF_OVL));
                mark_lanes(win, b4 & 0xFF);
                mark_lanes(win && rem, (b4 >> 8) & 0xFF);
                uint64_t ov = w.ballot(win && (((b4 >> 16) & 0xFF) & RF_OVL));
                while (ov) { /* removedClientOverlap lists: every entry stays */
                    int32_t l = W::ffs(ov);
                    ov &= ov - 1;
                    int32_t so = n * MAXN + j0 + l;
#pragma clang loop unroll(disable)
                    for (int32_t q = 0, e; (e = ovl_at(so, q)) >= 0; q++) mark((uint32_t)e);
                }
            }
        }
        bool freed = false;
        for (int32_t sl = 0; sl < zh->nclients; sl++)
            if (!((act[sl >> 6] >> (sl & 63)) & 1) && s2l[sl] != FREE_SLOT) freed = true;
        if (!freed) return false;
        /* retire the settled rows' bytes of the slots about to be freed */
#pragma clang loop unroll(disable)
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            const int32_t n = leaf_at(k), c = nch[n];
            for (int32_t j0 = 0; j0 < c; j0 += W::N) {
                const int32_t j = j0 + w.lane();
                const bool row = j < c;
                const int32_t s = n * MAXN + (row ? j : 0);
                const uint32_t b4 = row ? ld_bytes4(s) : 0;
                const uint32_t cb = b4 & 0xFF, rb = (b4 >> 8) & 0xFF;
                const bool rem = row && z.rseq(s) != NOREM;
                const bool rc = row && cb < MAX_SLOTS && !((act[cb >> 6] >> (cb & 63)) & 1);
                const bool rr = rem && rb < MAX_SLOTS && !((act[rb >> 6] >> (rb & 63)) & 1);
                w.sync();
                if (rc || rr) {
                    int32_t r = (int32_t)z.RID(s);
                    uint32_t e = d.RCL(r);
                    if (rc) e = (e & 0xFFFF0000u) | (uint32_t)s2l[cb];
                    if (rr) e = (e & 0xFFFFu) | ((uint32_t)s2l[rb] << 16);
                    d.RCL(r) = e;
                    st_bytes4(s, (b4 & 0xFFFF0000u) | (rc ? (uint32_t)RETIRED_CLIENT : cb) |
                                     ((rr ? (uint32_t)RETIRED_CLIENT : rb) << 8));
                }
                w.sync();
            }
        }
        for (int32_t sl = 0; sl < zh->nclients; sl++) {
            if (((act[sl >> 6] >> (sl & 63)) & 1) || s2l[sl] == FREE_SLOT) continue;
            int32_t lo = s2l[sl];
            if ((uint32_t)lo < (uint32_t)HT::C) l2s[lo] = 0xFF;
            s2l[sl] = FREE_SLOT;
        }
        w.sync();
        return true;
    }
    /* startOrUpdateCollaboration (client.ts:1053-1073) + startCollaboration (mergeTree.ts:1287) */
    MT_HD void start_collab(int32_t longId, int32_t minSeq, int32_t curSeq) {
        if (h.localLong >= 0 || longId < 0) return; /* longId < 0: stays detached (a snapshot load follows) */
        h.localLong = longId;
        h.localShort = get_or_add_short(longId);
        h.minSeq = minSeq;
        h.currentSeq = curSeq;
        h.collaborating = 1;
    }

    /* ---- row helpers ------------------------------------------------------------------- */
    MT_HD bool is_local(int32_t client) const {
        return !h.collaborating || client == h.localShort;
    }
    /* nodeLength of a leaf (mergeTree.ts:1692-1732); local perspective -> localNetLength */
    /* the scan columns of one slot, read together (four independent loads, one round trip) */
    struct RowView {
        int32_t len, seq, rseq;
        uint32_t b4; /* {cli, rcli, flags, ng} */
    };
    MT_HD RowView row_view(int32_t s) const {
        RowView r;
        r.len = z.len(s);
        r.seq = z.seq(s);
        r.rseq = z.rseq(s);
        r.b4 = ld_bytes4(s);
        return r;
    }
    /* the byte a row's client / removedClient must equal to be this client's own: a short id (0..253) as is,
     * LocalClientId (-1) as LOCAL_CLIENT, and anything else (0x7fff: a client the replica has never seen) as 0xFE,
     * which no short id takes (get_or_add_short hands out at most 254), so such a client owns no row */
    MT_HD static uint32_t client_byte(int32_t client) {
        return (uint32_t)client < (uint32_t)MAX_SLOTS ? (uint32_t)client : (client == -1 ? (uint32_t)LOCAL_CLIENT : 0xFEu);
    }
    MT_HD int32_t vis_of(int32_t s, const RowView& r, int32_t refSeq, int32_t client) const {
        return vis_of_l(s, r, refSeq, client, is_local(client));
    }
    /* vis_of with the local-perspective test decided by the caller (the window helper wave, win_block) */
    MT_HD int32_t vis_of_l(int32_t s, const RowView& r, int32_t refSeq, int32_t client, bool local) const {
        if (local) return r.rseq == NOREM ? r.len : 0;
        /* the tests of quad_vis_of: short id bytes against the client's byte, one unsigned compare per seq */
        const uint32_t uc = client_byte(client);
        const uint32_t ur1 = refSeq >= 0 ? (uint32_t)refSeq + 1u : 0u;
        uint32_t cq = r.b4 & 0xFFu, rcq = (r.b4 >> 8) & 0xFFu, fq = (r.b4 >> 16) & 0xFFu;
        if (!(cq == uc || (uint32_t)r.seq < ur1)) return 0;
        if (r.rseq != NOREM) {
            if (rcq == uc) return 0;
            if ((fq & RF_OVL) && ovl_has(s, client)) return 0; /* cold read: rare */
            if ((uint32_t)r.rseq < ur1) return 0;
        }
        return r.len;
    }
    MT_HD int32_t vis(int32_t s, int32_t refSeq, int32_t client) const {
        return vis_of(s, row_view(s), refSeq, client);
    }
    /* localNetLength (mergeTree.ts:1195-1206) */
    MT_HD int32_t local_len(int32_t s) const { return z.rseq(s) == NOREM ? z.len(s) : 0; }

    MT_HD int32_t slot_at(int32_t t) const { /* t = k*8+j over the leaf order; -1 if not a row */
        int32_t k = t >> 3, j = t & 7;
        if (!kvalid(k)) return -1;
        int32_t n = leaf_at(k);
        return j < nch[n] ? n * MAXN + j : -1;
    }

    /* ---- leaf order: the dense `lorder`, or the tiled rope (TileState) ------------------ */
    /* A leaf position k is an index into lorder, or (chunk position << 6 | index in chunk) when
     * TILED; positions increase in document order (with gaps when tiled). */
    MT_HD int32_t leaf_at(int32_t k) const {
        if constexpr (TILED)
            return z.tl.cleaf[tcord[k >> 6]][k & 63];
        else
            return lo[k];
    }
    MT_HD int32_t kpos(int32_t n) const {
        if constexpr (TILED)
            return (tcpos[z.tl.lch[n]] << 6) | z.tl.lix[n];
        else
            return lp[n];
    }
    MT_HD bool kvalid(int32_t k) const {
        if constexpr (TILED)
            return k >= 0 && (k >> 6) < z.tl.nchunk && (k & 63) < tccnt[tcord[k >> 6]];
        else
            return k < h.nleaf;
    }
    MT_HD int32_t knext(int32_t k) const {
        if constexpr (TILED)
            return (k & 63) + 1 < tccnt[tcord[k >> 6]] ? k + 1 : ((k >> 6) + 1) << 6;
        else
            return k + 1;
    }

    /* copy every column of row a to row b (same doc) */
    /* move row a's slot contents to slot b (hot columns + its cold row id) */
    MT_HD void copy_row(int32_t b, int32_t a) {
        if constexpr (TILED) {
            z.tl.xf[b] = z.tl.xf[a];
            z.tl.ph[b] = z.tl.ph[a];
        }
        z.len(b) = z.len(a);
        z.seq(b) = z.seq(a);
        z.rseq(b) = z.rseq(a);
        z.RID(b) = z.RID(a);
        st_bytes4(b, ld_bytes4(a));
    }
    /* a slot's {cli, rcli, flags, ng} bytes as one dword (one memory access instead of four) */
    MT_HD uint32_t ld_bytes4(int32_t a) const {
        uint32_t v;
        __builtin_memcpy(&v, __builtin_assume_aligned(&z.cli(a), 4), 4);
        return v;
    }
    MT_HD void st_bytes4(int32_t b, uint32_t v) { __builtin_memcpy(__builtin_assume_aligned(&z.cli(b), 4), &v, 4); }
    /* a row's slot contents held in registers */
    struct HotRow {
        int32_t len, seq, rseq;
        IX rid;
        uint8_t cli, rcli, flags, ng;
        uint8_t xf; /* tiled profile: XF_* */
        uint16_t ph; /* tiled profile: the property hash (TileState::ph) */
    };
    MT_HD HotRow load_row(int32_t a) const {
        HotRow r;
        r.len = z.len(a);
        r.seq = z.seq(a);
        r.rseq = z.rseq(a);
        r.rid = z.RID(a);
        uint32_t b4 = ld_bytes4(a);
        r.cli = (uint8_t)b4;
        r.rcli = (uint8_t)(b4 >> 8);
        r.flags = (uint8_t)(b4 >> 16);
        r.ng = (uint8_t)(b4 >> 24);
        r.xf = 0;
        r.ph = 0;
        if constexpr (TILED) {
            r.xf = z.tl.xf[a];
            r.ph = z.tl.ph[a];
        }
        return r;
    }
    MT_HD void store_row(int32_t b, const HotRow& r) {
        z.len(b) = r.len;
        z.seq(b) = r.seq;
        z.rseq(b) = r.rseq;
        z.RID(b) = r.rid;
        st_bytes4(b, (uint32_t)r.cli | ((uint32_t)r.rcli << 8) | ((uint32_t)r.flags << 16) | ((uint32_t)r.ng << 24));
        if constexpr (TILED) {
            z.tl.xf[b] = r.xf;
            z.tl.ph[b] = r.ph;
        }
    }
    /* shift slab rows [j, c) of leaf n right by one slot (wave-parallel: read all, then write) */
    MT_HD void slab_shift_right(int32_t n, int32_t j, int32_t c) {
        if (W::N >= MAXN) {
            int32_t l = w.lane();
            bool mv = l >= j && l < c;
            HotRow r;
            if (mv) r = load_row(n * MAXN + l);
            w.sync();
            if (mv) store_row(n * MAXN + l + 1, r);
            w.sync();
        } else {
            for (int32_t i = c; i > j; i--) copy_row(n * MAXN + i, n * MAXN + i - 1);
        }
    }
    /* copy `cnt` rows between non-overlapping slot ranges */
    MT_HD void move_rows(int32_t dst, int32_t src, int32_t cnt) {
        for (int32_t b = 0; b < cnt; b += W::N) {
            int32_t i = b + w.lane();
            if (i < cnt) store_row(dst + i, load_row(src + i));
        }
        w.sync();
    }
    /* shift lorder[from, n) by delta entries and fix lpos; chunk order never overwrites an
     * entry before it is read */
    MT_HD void lorder_shift(int32_t from, int32_t n, int32_t delta) {
        int32_t cnt = n - from;
        if (delta == 0 || cnt <= 0) return;
        int32_t nch = (cnt + W::N - 1) / W::N;
        for (int32_t c = 0; c < nch; c++) {
            int32_t b = delta > 0 ? (nch - 1 - c) * W::N : c * W::N;
            int32_t i = from + b + w.lane();
            bool ok = i < n;
            int32_t x = ok ? lo[i] : 0;
            w.sync();
            if (ok) {
                lo[i + delta] = (IX)x;
                lp[x] = (IX)(i + delta);
            }
            w.sync();
        }
    }
    /* cold row ids */
    MT_HD int32_t alloc_rid() {
        int32_t n = zh->nfreeRid;
        if (n <= 0) {
            fail(E_CAPACITY);
            return 0;
        }
        zh->nfreeRid = n - 1;
        return d.FRID(n - 1); /* (a read-ahead of the next entry measured slower: r04l, r04m) */
    }
    MT_HD void free_rid(int32_t r) {
        z.RGEN(r)++;
        d.FRID(zh->nfreeRid++) = (IX)r;
    }
    /* record leaf n as the holder of its first `cnt` rows */
    MT_HD void set_leaf_of_rows(int32_t n, int32_t cnt) {
        for (int32_t b = 0; b < cnt; b += W::N) {
            int32_t j = b + w.lane();
            int32_t r = j < cnt ? z.RID(n * MAXN + j) : -1;
            if (r >= 0) z.RLEAF(r) = (IX)n;
        }
        w.sync();
    }
    /* slot of a live row id (its leaf is rleaf[rid]); -1 if the id was freed since `gen` */
    MT_HD int32_t slot_of(int32_t rid, int32_t gen) {
        int32_t g = z.RGEN(rid), leaf = z.RLEAF(rid); /* both reads in one round trip */
        if (gen >= 0 && g != (uint8_t)gen) return -1;
        int32_t c = nch[leaf];
        if (W::N == 1) {
            for (int32_t j = 0; j < c; j++)
                if (z.RID(leaf * MAXN + j) == rid) return leaf * MAXN + j;
            return -1;
        }
        int32_t j = w.lane();
        int32_t r = z.RID(leaf * MAXN + (j & (MAXN - 1))); /* with the child count: one round trip */
        uint64_t m = w.ballot(j < c && r == rid);
        return m ? leaf * MAXN + W::ffs(m) : -1;
    }

    /* slot_of(ra, -1) and slot_of(rb, -1) with both lookups' reads issued together (two round trips, not four) */
    MT_HD void slot_of2(int32_t ra, int32_t rb, int32_t* sa, int32_t* sb) {
        if constexpr (W::N >= 2 * MAXN) {
            int32_t la = z.RLEAF(ra), lb = z.RLEAF(rb);
            int32_t ca = nch[la], cb = nch[lb];
            const int32_t j = w.lane();
            const bool first = j < MAXN;
            int32_t lf = first ? la : lb;
            int32_t r = j < 2 * MAXN ? (int32_t)z.RID(lf * MAXN + (j & (MAXN - 1))) : -1;
            uint64_t m = w.ballot(j < 2 * MAXN && (j & (MAXN - 1)) < (first ? ca : cb) && r == (first ? ra : rb));
            uint64_t ma = m & 0xFFull, mb = (m >> MAXN) & 0xFFull;
            *sa = ma ? la * MAXN + W::ffs(ma) : -1;
            *sb = mb ? lb * MAXN + W::ffs(mb) : -1;
        } else {
            *sa = slot_of(ra, -1);
            *sb = slot_of(rb, -1);
        }
    }

    /* ---- tiled profile: rope of leaves, STABLE summaries, window set ------------------- */
    MT_HD void rope_init() {
        auto& t = z.tl;
        constexpr int NCH = HT::TL::NCH;
        for (int32_t b = 0; b < NCH; b += W::N) {
            int32_t i = b + w.lane();
            if (i < NCH) {
                tcpos[i] = i + 1; /* free list */
                tccnt[i] = 0;
                t.sdel[i] = 0;
            }
        }
        w.sync();
        for (int32_t b = 0; b < HT::TL::NG; b += W::N) {
            int32_t g = b + w.lane();
            if (g < HT::TL::NG) {
                tgst[g] = 0;
                t.sgdel[g] = 0;
            }
        }
        t.nchunk = 1;
        tcord[0] = 0;
        tcpos[0] = 0;
        tcst[0] = 0;
        tccnt[0] = 1;
        t.cleaf[0][0] = 0;
        t.cfree = 1;
        t.nfreeChunk = NCH - 1;
        t.lch[0] = 0;
        t.lix[0] = 0;
        t.lst[0] = 0;
        t.cls[0][0] = 0;
        t.wN = 0;
        w.sync();
    }
    MT_HD int32_t chunk_alloc() {
        auto& t = z.tl;
        int32_t c = t.cfree;
        if (c >= HT::TL::NCH) {
            fail(E_CAPACITY);
            return -1;
        }
        t.cfree = tcpos[c];
        t.nfreeChunk--;
        tccnt[c] = 0;
        return c;
    }
    MT_HD void chunk_free(int32_t c) {
        auto& t = z.tl;
        tcpos[c] = t.cfree;
        t.cfree = c;
        t.nfreeChunk++;
    }
    /* a chunk summary changes by d: its group's sum with it */
    MT_HD void cst_add(int32_t p, int32_t d) {
        tcst[p] += d;
        tgst[p >> 6] += d;
    }
    /* the group sums from position p's group on, after chunk positions moved (a chunk split or freed: rare) */
    MT_HD void gst_rebuild(int32_t p) {
        int32_t nc = z.tl.nchunk;
        for (int32_t g = p >> 6; g < HT::TL::NG; g++) {
            int32_t v = 0;
            for (int32_t b = 0; b < 64; b += W::N) {
                int32_t i = 64 * g + b + w.lane();
                v += w.sum(i < nc && b + w.lane() < 64 ? tcst[i] : 0);
            }
            w.sync();
            tgst[g] = v;
            w.sync();
            if (64 * g + 64 >= nc) { /* the groups past the last chunk are empty */
                for (int32_t b = g + 1; b < HT::TL::NG; b += W::N)
                    if (b + w.lane() < HT::TL::NG) tgst[b + w.lane()] = 0;
                w.sync();
                break;
            }
        }
    }
    /* move chunk positions [from, nchunk) by delta (+1 / -1) with their summaries; fix cpos */
    MT_HD void cord_shift(int32_t from, int32_t delta) {
        auto& t = z.tl;
        int32_t n = t.nchunk, cnt = n - from;
        if (cnt <= 0) return;
        int32_t np = (cnt + W::N - 1) / W::N;
        for (int32_t c = 0; c < np; c++) {
            int32_t b = delta > 0 ? (np - 1 - c) * W::N : c * W::N;
            if (W::N == 1) b = delta > 0 ? cnt - 1 - c : c;
            int32_t i = from + b + (W::N == 1 ? 0 : w.lane());
            bool ok = i < n && i >= from;
            int32_t id = ok ? tcord[i] : 0, sm = ok ? tcst[i] : 0;
            w.sync();
            if (ok) {
                tcord[i + delta] = id;
                tcst[i + delta] = sm;
                tcpos[id] = i + delta;
            }
            w.sync();
        }
    }
    /* shift leaves [i0, cnt) of chunk c by delta (+1 / -1), fixing lix (<= 64 entries) */
    MT_HD void chunk_shift(int32_t c, int32_t i0, int32_t cnt, int32_t delta) {
        auto& t = z.tl;
        if constexpr (W::N >= 64) {
            int32_t i = i0 + w.lane();
            bool ok = i < cnt;
            int32_t lf = ok ? t.cleaf[c][i] : 0, ls = ok ? t.cls[c][i] : 0;
            w.sync();
            if (ok) {
                t.cleaf[c][i + delta] = lf;
                t.cls[c][i + delta] = ls;
                t.lix[lf] = (uint8_t)(i + delta);
            }
            w.sync();
        } else {
            for (int32_t q = 0; q < cnt - i0; q++) {
                int32_t i = delta > 0 ? cnt - 1 - q : i0 + q;
                int32_t lf = t.cleaf[c][i];
                t.cleaf[c][i + delta] = lf;
                t.cls[c][i + delta] = t.cls[c][i];
                t.lix[lf] = (uint8_t)(i + delta);
            }
        }
    }
    /* leaf b goes right after leaf a in document order (a full chunk splits 32 + 32) */
    MT_HD void rope_insert_after(int32_t a, int32_t b) {
        MT_PROF_SCOPE(PH_ROPE);
        auto& t = z.tl;
        constexpr int32_t CH = HT::TL::CH, HALF = CH / 2;
        int32_t c = t.lch[a], i = t.lix[a] + 1;
        if (tccnt[c] >= CH) {
            int32_t c2 = chunk_alloc();
            if (c2 < 0) return;
            int32_t p = tcpos[c];
            cord_shift(p + 1, 1);
            t.nchunk++;
            tcord[p + 1] = c2;
            tcpos[c2] = p + 1;
            int32_t moved = 0;
            for (int32_t bb = 0; bb < HALF; bb += W::N) {
                int32_t l = bb + w.lane();
                int32_t v = 0;
                if (l < HALF) {
                    int32_t lf = t.cleaf[c][HALF + l];
                    v = t.cls[c][HALF + l];
                    t.cleaf[c2][l] = lf;
                    t.cls[c2][l] = v;
                    t.lch[lf] = c2;
                    t.lix[lf] = (uint8_t)l;
                }
                moved += w.sum(v);
            }
            w.sync();
            tccnt[c2] = HALF;
            tccnt[c] = HALF;
            tcst[p + 1] = moved;
            tcst[p] -= moved;
            gst_rebuild(p); /* positions after p moved one up */
            if (i >= HALF) {
                c = c2;
                i -= HALF;
            }
        }
        int32_t cnt = tccnt[c];
        chunk_shift(c, i, cnt, 1);
        int32_t lb = t.lst[b];
        t.cleaf[c][i] = b;
        t.cls[c][i] = lb;
        t.lch[b] = c;
        t.lix[b] = (uint8_t)i;
        tccnt[c] = cnt + 1;
        cst_add(tcpos[c], lb);
        w.sync();
    }
    /* leaf b leaves the document order (its STABLE length leaves its chunk's summary) */
    MT_HD void rope_remove(int32_t b) {
        MT_PROF_SCOPE(PH_ROPE);
        auto& t = z.tl;
        int32_t c = t.lch[b], i = t.lix[b], p = tcpos[c];
        cst_add(p, -t.lst[b]);
        t.lst[b] = 0;
        int32_t cnt = tccnt[c];
        chunk_shift(c, i + 1, cnt, -1);
        tccnt[c] = cnt - 1;
        if (cnt - 1 == 0) {
            cord_shift(p + 1, -1);
            t.nchunk--;
            chunk_free(c);
            gst_rebuild(p); /* positions after p moved one down */
        }
        w.sync();
    }
    /* cls[lch[n]][lix[n]] always equals lst[n] (every update writes both): the new sum goes to both, one read */
    MT_HD void lst_add(int32_t n, int32_t d) {
        auto& t = z.tl;
        int32_t c = t.lch[n], v = t.lst[n] + d;
        t.lst[n] = v;
        t.cls[c][t.lix[n]] = v;
        cst_add(tcpos[c], d);
    }
    /* lst_add with the leaf's chunk, index and sum read ahead by the caller */
    MT_HD void lst_add_known(int32_t n, int32_t c, int32_t ix, int32_t old, int32_t d) {
        auto& t = z.tl;
        t.lst[n] = old + d;
        t.cls[c][ix] = old + d;
        cst_add(tcpos[c], d);
    }
    /* recompute leaf n's STABLE length from its rows */
    MT_HD void leaf_restat(int32_t n) {
        MT_PROF_SCOPE(PH_RESTAT);
        int32_t c = nch[n];
        int32_t v = 0;
        for (int32_t b = 0; b < c; b += W::N) {
            int32_t j = b + w.lane();
            int32_t x = 0;
            if (j < c && (z.tl.xf[n * MAXN + j] & XF_STABLE)) x = z.len(n * MAXN + j);
            v += w.sum(x);
        }
        lst_add(n, v - z.tl.lst[n]);
        w.sync();
    }
    /* leaf_restat of cnt <= 8 distinct leaves at once (a split leaf's halves, a pack's new leaves): lane q reads
     * row q & 7 of leaf q >> 3 and the leaf's old summary and chunk in one pass; the chunk summaries (LDS in
     * the tiled kernel) are updated leaf by leaf */
    MT_HD void leaves_restat(const int32_t* nl, int32_t cnt) {
        if constexpr (W::N >= MAXN * MAXN) {
            MT_PROF_SCOPE(PH_RESTAT);
            auto& t = z.tl;
            int32_t q = w.lane(), i = q >> 3, j = q & (MAXN - 1);
            int32_t n = -1;
            for (int32_t k = 0; k < MAXN; k++)
                if (k == i && k < cnt) n = nl[k];
            int32_t old = n >= 0 ? t.lst[n] : 0, ch = n >= 0 ? t.lch[n] : 0, ix = n >= 0 ? t.lix[n] : 0;
            int32_t c = n >= 0 ? nch[n] : 0;
            int32_t x = 0;
            if (j < c && (t.xf[n * MAXN + j] & XF_STABLE)) x = z.len(n * MAXN + j);
            x += w.shfl_xor(x, 1);
            x += w.shfl_xor(x, 2);
            x += w.shfl_xor(x, 4);
            w.sync();
            if (n >= 0 && j == 0) {
                t.lst[n] = x;
                t.cls[ch][ix] = x;
            }
            for (int32_t k = 0; k < cnt; k++) {
                int32_t dk = w.bcast(x - old, MAXN * k);
                if (dk) cst_add(tcpos[w.bcast(ch, MAXN * k)], dk);
            }
            w.sync();
        } else {
            for (int32_t k = 0; k < cnt; k++) leaf_restat(nl[k]);
        }
    }
    /* a row is settled when its insert and (if any) its removal are sequenced at or below minSeq */
    MT_HD bool settled_of(const RowView& r) const {
        return r.seq != UNASSIGNED_SEQ && r.seq <= h.minSeq &&
               (r.rseq == NOREM || (r.rseq != UNASSIGNED_SEQ && r.rseq <= h.minSeq));
    }
    MT_HD bool settled(int32_t s) const {
        int32_t sq = z.seq(s), rs = z.rseq(s);
        return sq != UNASSIGNED_SEQ && sq <= h.minSeq && (rs == NOREM || (rs != UNASSIGNED_SEQ && rs <= h.minSeq));
    }
    MT_HD void win_add(int32_t rid, int32_t s) {
        auto& t = z.tl;
        if (t.wN >= WCAPR) {
            fail(E_CAPACITY);
            return;
        }
        twrid[t.wN] = rid;
        twgen[t.wN] = z.RGEN(rid);
        twslot[t.wN] = s;
        t.wN++;
    }
    /* row_enter of a row whose id, generation, seq, removedSeq and length the caller holds */
    MT_HD void row_enter_known(int32_t s, int32_t rid, int32_t gen, int32_t seq, int32_t rseq, int32_t len) {
        bool st = seq != UNASSIGNED_SEQ && seq <= h.minSeq && (rseq == NOREM || (rseq != UNASSIGNED_SEQ && rseq <= h.minSeq));
        if (st) {
            z.tl.xf[s] = rseq == NOREM ? XF_STABLE : 0;
            if (rseq == NOREM) lst_add(s / MAXN, len);
        } else {
            z.tl.xf[s] = XF_W;
            auto& t = z.tl;
            if (t.wN >= WCAPR) {
                fail(E_CAPACITY);
                return;
            }
            twrid[t.wN] = rid;
            twgen[t.wN] = (uint8_t)gen;
            twslot[t.wN] = s;
            t.wN++;
        }
    }
    /* a row just placed (insert): STABLE if already settled (non-collaborating edits), else W */
    MT_HD void row_enter(int32_t s) {
        if (settled(s)) {
            z.tl.xf[s] = z.rseq(s) == NOREM ? XF_STABLE : 0;
            if (z.rseq(s) == NOREM) lst_add(s / MAXN, z.len(s));
        } else {
            z.tl.xf[s] = XF_W;
            win_add(z.RID(s), s);
        }
    }
    /* a row just marked removed: leaves the STABLE summaries; W unless the removal is settled */
    MT_HD void row_removed(int32_t s) {
        uint8_t x = z.tl.xf[s];
        if (x & XF_STABLE) {
            lst_add(s / MAXN, -z.len(s));
            x = 0;
        }
        if (!(x & XF_W) && !settled(s)) {
            x = XF_W;
            win_add(z.RID(s), s);
        }
        z.tl.xf[s] = x;
    }
    /* Evaluate the window set under (refSeq, client): rows the MSN has passed settle into the
     * STABLE summaries (or DEAD), entries of freed rows drop out, and every remaining row's chunk
     * position, leaf index and perspective length go to the scratch, its length scattered onto
     * cdel[chunk position]. Returns the sum of those lengths. */
#ifndef MT_FIND2
#define MT_FIND2 1 /* a tiled range op's two ends found in the same passes (tile_find2 / leaf_find2) */
#endif
#ifndef MT_WIN_NB
#define MT_WIN_NB 1 /* wave passes of the window set issued together: 2 covered the ~80-100 rows in one round trip (r04e, 8 -> 2: 8.81 -> 9.66M ops/s at 256 x 300k); since the set's entries and the leaf headers sit in LDS (round 5), one pass at a time is faster (r05zd at 256 x 1M: 2 -> 1: 15.73 -> 15.88M, 4: 14.91M) */
#endif
#ifndef MT_WIN_HELPER /* tiled kernel: a second wave of the document's workgroup evaluates the window set's second block
                          (win_helper) — 2: handed over by two workgroup barriers (r06h at 256 x 300k: 16.21 -> 16.36M
                          ops/s); 1: by polled LDS flags (r06g: 16.23 -> 15.46M, the s_sleep wake-up costs more than the
                          global round trip it hides, tools/wave_sync_probe.hip); 0: one wave */
#define MT_WIN_HELPER 2
#endif
    /* stages 1-3 of win_pass for one block of window entries (lane i = b0 + lane < n) under (refSeq, client) with the
     * given minSeq and local-perspective test: the entry (rd, g), its row's slot s (-1: gone), the row, its leaf's
     * chunk (lc) and index (lx), settle / keep, the perspective length v and the chunk position cp */
    struct WinRow {
        int32_t rd, g, s, lc, lx, v, cp;
        bool settle, keep;
        RowView rv;
    };
    MT_HD WinRow win_block(int32_t b0, int32_t n, int32_t refSeq, int32_t client, int32_t minSeq, bool local) {
        auto& t = z.tl;
        WinRow x;
        int32_t i = b0 + w.lane();
        bool ok = i < n;
        x.rd = ok ? twrid[i] : 0;
        x.g = ok ? twgen[i] : -1;
        x.s = ok ? twslot[i] : 0;
        int32_t c = x.s, l = c / MAXN;
        uint8_t gg = z.RGEN(x.rd);
        IX lr = z.RLEAF(x.rd), cr = z.RID(c);
        int32_t cn = nch[l];
        bool gok = x.g >= 0 && gg == (uint8_t)x.g;
        bool hit = gok & (lr == (IX)l) & ((c & (MAXN - 1)) < cn) & (cr == (IX)x.rd);
        x.rv = row_view(c);
        x.lc = t.lch[l];
        x.lx = t.lix[l];
        if (!hit) x.s = gok ? -2 : -1;
        if (x.s == -2) {
            int32_t lf = z.RLEAF(x.rd);
            int32_t cc = nch[lf];
            x.s = -1;
            for (int32_t j = 0; j < MAXN; j++)
                if (j < cc && z.RID(lf * MAXN + j) == (IX)x.rd) x.s = lf * MAXN + j;
            if (x.s >= 0) {
                x.rv = row_view(x.s);
                x.lc = t.lch[lf];
                x.lx = t.lix[lf];
            }
        }
        const RowView& r = x.rv;
        x.settle = x.s >= 0 && r.seq != UNASSIGNED_SEQ && r.seq <= minSeq &&
                   (r.rseq == NOREM || (r.rseq != UNASSIGNED_SEQ && r.rseq <= minSeq));
        x.keep = x.s >= 0 && !x.settle;
        x.v = x.cp = 0;
        if (x.keep) {
            x.v = vis_of_l(x.s, x.rv, refSeq, client, local);
            x.cp = tcpos[x.lc];
        }
        return x;
    }
    /* the helper wave's loop (k_replay_tiled with MT_WIN_HELPER): each request of the replaying wave (a window pass
     * with more than W::N entries) evaluated on the second block, the results left in the mailbox. Exits when the
     * replaying wave is done (`*quit`). Every wait is bounded. */
    MT_HD void win_helper(const volatile int32_t* quit) {
#ifdef __HIP_DEVICE_COMPILE__
        if constexpr (TILED && W::N == 64) {
            volatile WinMail* m = wm;
#if MT_WIN_HELPER == 2
            for (;;) { /* barrier handoff: every request is two workgroup barriers, matched by win_pass2 */
                __syncthreads(); /* a request (or the end) is posted */
                if (m->quit) return;
                WinRow x = win_block(W::N, m->n, m->refSeq, m->client, m->minSeq, m->local != 0);
                int32_t l = w.lane();
                m->s[l] = x.s, m->lc[l] = x.lc, m->lx[l] = x.lx, m->len[l] = x.rv.len, m->rseq[l] = x.rv.rseq;
                m->v[l] = x.v, m->cp[l] = x.cp, m->st[l] = (x.settle ? 1 : 0) | (x.keep ? 2 : 0);
                __syncthreads(); /* the results are in */
            }
#endif
            int32_t last = 0;
            for (;;) {
                int32_t spins = 0;
                while (m->req == last && !*quit && ++spins < (1 << 26)) __builtin_amdgcn_s_sleep(1);
                if (m->req == last) return; /* done (or a replaying wave gone quiet: stop waiting) */
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                last = m->req;
                WinRow x = win_block(W::N, m->n, m->refSeq, m->client, m->minSeq, m->local != 0);
                int32_t l = w.lane();
                m->s[l] = x.s, m->lc[l] = x.lc, m->lx[l] = x.lx, m->len[l] = x.rv.len, m->rseq[l] = x.rv.rseq;
                m->v[l] = x.v, m->cp[l] = x.cp, m->st[l] = (x.settle ? 1 : 0) | (x.keep ? 2 : 0);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (l == 0) m->done = last;
            }
        }
#else
        (void)quit;
#endif
    }
    MT_HD int32_t win_pass(int32_t refSeq, int32_t client) {
        MT_PROF_SCOPE(PH_WIN);
        auto& t = z.tl;
#if MT_WIN_HELPER && defined(__HIPCC__)
        if constexpr (TILED && W::N == 64) {
            if (wm) return win_pass2(refSeq, client);
        }
#endif
        /* NB passes of the wave at a time, stage by stage: every entry's loads of one stage are issued
         * together (one round trip per stage, not one per stage per pass); the settling and the
         * compaction then run pass by pass, in entry order. Every read of a block precedes its writes,
         * and the compaction only writes entries at or before the ones read. */
        constexpr int NB = W::N >= 64 ? MT_WIN_NB : 1;
        int32_t n = t.wN, wpos = 0, total = 0;
        for (int32_t b0 = 0; b0 < n; b0 += NB * W::N) {
            int32_t rd[NB], g[NB], s[NB], v[NB], cp[NB], lx[NB];
            bool settle[NB], keep[NB];
#pragma unroll
            for (int q = 0; q < NB; q++) { /* the entries (LDS in the tiled kernel) */
                int32_t i = b0 + q * W::N + w.lane();
                bool ok = i < n;
                rd[q] = ok ? twrid[i] : 0;
                g[q] = ok ? twgen[i] : -1;
                s[q] = ok ? twslot[i] : 0;
            }
            /* One round trip when the row is still in the slot it was last seen in: its generation, its leaf,
             * the slot's row id and the leaf's child count check the hint, and the row itself and its leaf's
             * rope links are read in the same pass. */
            RowView rv[NB];
            int32_t lc[NB];
#pragma unroll
            for (int q = 0; q < NB; q++) {
                int32_t c = s[q], l = c / MAXN;
                uint8_t gg = z.RGEN(rd[q]); /* every load of the pass unconditional: they issue together */
                IX lr = z.RLEAF(rd[q]), cr = z.RID(c);
                int32_t cn = nch[l];
                bool gok = g[q] >= 0 && gg == (uint8_t)g[q];
                bool hit = gok & (lr == (IX)l) & ((c & (MAXN - 1)) < cn) & (cr == (IX)rd[q]);
                rv[q] = row_view(c);
                lc[q] = t.lch[l];
                lx[q] = t.lix[l];
                if (!hit) s[q] = gok ? -2 : -1; /* -2: look the row up */
            }
#pragma unroll
            for (int q = 0; q < NB; q++) {
                MT_PROF_COUNT(PH_C_WROWS, __builtin_popcountll(w.ballot(b0 + q * W::N + w.lane() < n)));
                MT_PROF_COUNT(PH_C_WMISS, __builtin_popcountll(w.ballot(s[q] == -2)));
            }
#pragma unroll
            for (int q = 0; q < NB; q++) { /* the rows that moved: leaf, slot, row */
                if (s[q] == -2) {
                    int32_t lf = z.RLEAF(rd[q]);
                    int32_t c = nch[lf];
                    s[q] = -1;
                    for (int32_t j = 0; j < MAXN; j++)
                        if (j < c && z.RID(lf * MAXN + j) == (IX)rd[q]) s[q] = lf * MAXN + j;
                    if (s[q] >= 0) {
                        rv[q] = row_view(s[q]);
                        lc[q] = t.lch[lf];
                        lx[q] = t.lix[lf];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NB; q++) { /* settled, or its perspective length and chunk position */
                settle[q] = s[q] >= 0 && settled_of(rv[q]);
                keep[q] = s[q] >= 0 && !settle[q];
                v[q] = cp[q] = 0;
                if (keep[q]) {
                    v[q] = vis_of(s[q], rv[q], refSeq, client);
                    cp[q] = tcpos[lc[q]];
                }
            }
            for (int q = 0; q < NB; q++) {
                if (b0 + q * W::N >= n) break;
                uint64_t m = w.ballot(settle[q]);
                while (m) { /* a few rows per op: serial, on the values this pass read (row, leaf's chunk) */
                    int32_t l = W::ffs(m);
                    m &= m - 1;
                    int32_t ss = w.bcast(s[q], l);
                    if (w.bcast(rv[q].rseq, l) == NOREM) {
                        t.xf[ss] = XF_STABLE;
                        int32_t dl = w.bcast(rv[q].len, l), lcl = w.bcast(lc[q], l);
                        int32_t nv = t.lst[ss / MAXN] + dl; /* cls mirrors lst: one read */
                        t.lst[ss / MAXN] = nv;
                        t.cls[lcl][w.bcast(lx[q], l)] = nv;
                        cst_add(tcpos[lcl], dl);
                    } else {
                        t.xf[ss] = 0;
                    }
                }
                int32_t tot;
                int32_t off = w.excl_scan(keep[q] ? 1 : 0, &tot);
                w.sync();
                if (keep[q]) {
                    int32_t o = wpos + off;
                    twrid[o] = rd[q];
                    twgen[o] = (uint8_t)g[q];
                    twslot[o] = s[q];
                    wcp[o] = cp[q];
                    wlx[o] = (uint8_t)lx[q];
                    wvs[o] = v[q];
                    if (v[q]) {
                        W::atomic_add(&cdel[cp[q]], v[q]);
                        W::atomic_add(&gdel[cp[q] >> 6], v[q]);
                    }
                }
                w.sync();
                wpos += tot;
                total += w.sum(v[q]);
            }
        }
        t.wN = wpos;
        return total;
    }
#if MT_WIN_HELPER && defined(__HIPCC__)
    /* win_pass with the helper wave: the second block's entries evaluated by the helper while this wave evaluates the
     * first; then both blocks settled and compacted in entry order, as win_pass does, and the rest of the set (more
     * than 2 W::N entries) here. The compaction writes only positions below the entries still to be read. */
    MT_HD int32_t win_pass2(int32_t refSeq, int32_t client) {
        auto& t = z.tl;
        int32_t n = t.wN, wpos = 0, total = 0;
        const bool local = is_local(client);
        volatile WinMail* m = wm;
        const bool split = n > W::N;
        if (split) { /* post the request: the second block, this perspective */
            if (w.lane() == 0) {
                m->n = n, m->refSeq = refSeq, m->client = client, m->minSeq = h.minSeq, m->local = local ? 1 : 0;
            }
#if MT_WIN_HELPER == 2
            __syncthreads(); /* the helper's first barrier of the request */
#else
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wmseq++;
            if (w.lane() == 0) m->req = wmseq;
#endif
        }
        for (int32_t b0 = 0; b0 < n; b0 += W::N) {
            WinRow x;
            if (b0 == W::N && split) { /* the helper's results */
#if MT_WIN_HELPER == 2
                __syncthreads(); /* the helper's second barrier */
#else
                int32_t spins = 0;
                while (m->done != wmseq && ++spins < (1 << 26)) __builtin_amdgcn_s_sleep(1);
                if (m->done != wmseq) { /* the helper never answered: stop here, the document latched */
                    fail(E_ASSERT);
                    return total;
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
                int32_t l = w.lane(), i = b0 + l;
                x.rd = i < n ? twrid[i] : 0;
                x.g = i < n ? twgen[i] : -1;
                x.s = m->s[l], x.lc = m->lc[l], x.lx = m->lx[l], x.rv.len = m->len[l], x.rv.rseq = m->rseq[l];
                x.v = m->v[l], x.cp = m->cp[l];
                int32_t st = m->st[l];
                x.settle = (st & 1) != 0, x.keep = (st & 2) != 0;
            } else {
                x = win_block(b0, n, refSeq, client, h.minSeq, local);
            }
            uint64_t msk = w.ballot(x.settle);
            while (msk) { /* serial, on the values the block read */
                int32_t l = W::ffs(msk);
                msk &= msk - 1;
                int32_t ss = w.bcast(x.s, l);
                if (w.bcast(x.rv.rseq, l) == NOREM) {
                    t.xf[ss] = XF_STABLE;
                    int32_t dl = w.bcast(x.rv.len, l), lcl = w.bcast(x.lc, l);
                    int32_t nv = t.lst[ss / MAXN] + dl;
                    t.lst[ss / MAXN] = nv;
                    t.cls[lcl][w.bcast(x.lx, l)] = nv;
                    cst_add(tcpos[lcl], dl);
                } else {
                    t.xf[ss] = 0;
                }
            }
            int32_t tot;
            int32_t off = w.excl_scan(x.keep ? 1 : 0, &tot);
            w.sync();
            if (x.keep) {
                int32_t o = wpos + off;
                twrid[o] = x.rd;
                twgen[o] = (uint8_t)x.g;
                twslot[o] = x.s;
                wcp[o] = x.cp;
                wlx[o] = (uint8_t)x.lx;
                wvs[o] = x.v;
                if (x.v) {
                    W::atomic_add(&cdel[x.cp], x.v);
                    W::atomic_add(&gdel[x.cp >> 6], x.v);
                }
            }
            w.sync();
            wpos += tot;
            total += w.sum(x.v);
        }
        t.wN = wpos;
        return total;
    }
#endif
    /* zero the chunk deltas of the last win_pass */
    MT_HD void win_clear() {
        int32_t n = z.tl.wN;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            if (i < n) {
                cdel[wcp[i]] = 0;
                gdel[wcp[i] >> 6] = 0;
            }
        }
        w.sync();
    }
    /* The chunk position holding position pos (the first with P < pos <= P + its total, window deltas included)
     * and the total before it: on the GPU the group sums first, then that group's chunks (two LDS passes, not
     * one per 256 chunks); on the host the chunk scan. -1 if pos is beyond the length. */
    MT_HD int32_t chunk_find(int32_t pos, int32_t* runOut) {
        int32_t nc = z.tl.nchunk;
        if constexpr (W::N >= 64) {
            static_assert(HT::TL::NG <= W::N, "one pass over the groups");
            int32_t ng = (nc + 63) >> 6, l = w.lane();
            int32_t v = l < ng ? tgst[l] + gdel[l] : 0;
            int32_t tot;
            int32_t p = w.excl_scan(v, &tot);
            uint64_t m = w.ballot(l < ng && p < pos && pos <= p + v);
            if (!m) return -1;
            int32_t g = W::ffs(m);
            int32_t run = w.bcast(p, g);
            int32_t i = 64 * g + l;
            int32_t x = i < nc ? tcst[i] + cdel[i] : 0;
            int32_t q = run + w.excl_scan(x, &tot);
            m = w.ballot(i < nc && q < pos && pos <= q + x);
            if (!m) {
                fail(E_ASSERT); /* a group's chunks must add up to its sum */
                return -1;
            }
            int32_t c = W::ffs(m);
            *runOut = w.bcast(q, c);
            return 64 * g + c;
        } else {
            int32_t run = 0;
            for (int32_t b = 0; b < nc; b += 4 * W::N) {
                int32_t p0 = b + 4 * w.lane();
                int32_t v[4];
                for (int q = 0; q < 4; q++) v[q] = p0 + q < nc ? tcst[p0 + q] + cdel[p0 + q] : 0;
                int32_t tot;
                int32_t p = run + w.excl_scan(v[0] + v[1] + v[2] + v[3], &tot);
                int32_t hq = -1, hp = 0;
                for (int q = 0; q < 4; q++) {
                    if (hq < 0 && p < pos && pos <= p + v[q]) {
                        hq = q;
                        hp = p;
                    }
                    p += v[q];
                }
                uint64_t m = w.ballot(hq >= 0);
                if (m) {
                    int32_t l = W::ffs(m);
                    *runOut = w.bcast(hp, l);
                    return b + 4 * l + w.bcast(hq, l);
                }
                run += tot;
            }
            return -1;
        }
    }
    /* the sum of every chunk's STABLE total (the group sums; on the host checked against the chunks) */
    MT_HD int32_t stable_total() {
        int32_t total = 0;
        for (int32_t b = 0; b < HT::TL::NG; b += W::N) {
            int32_t g = b + w.lane();
            total += w.sum(g < HT::TL::NG ? tgst[g] : 0);
        }
#ifndef __HIP_DEVICE_COMPILE__
        int32_t chk = 0;
        for (int32_t p = 0; p < z.tl.nchunk; p++) chk += tcst[p];
        if (chk != total) fail(E_ASSERT);
#endif
        return total;
    }
    /* Leaf position k and start offset P of the leaf holding the first row with
     * P < pos <= P + vis, from the chunk and leaf summaries plus the window scratch of the last
     * win_pass (same perspective). -1 if pos is beyond the length. */
    MT_HD int32_t tile_find(int32_t pos, int32_t refSeq, int32_t client, int32_t* Pout, int32_t* Nout) {
        MT_PROF_SCOPE(PH_TFIND);
        auto& t = z.tl;
        int32_t run = 0;
        int32_t cpf = chunk_find(pos, &run);
        if (cpf < 0) return -1;
        /* leaves of the chunk: STABLE lengths + the window rows that sit in them */
        int32_t c = tcord[cpf], cnt = tccnt[c];
        int32_t nw = t.wN;
        int32_t ldel[HT::TL::CH / (W::N < 64 ? W::N : 64) + 1] = {};
        for (int32_t b = 0; b < nw; b += W::N) {
            int32_t i = b + w.lane();
            uint64_t m = w.ballot(i < nw && wcp[i] == cpf);
            while (m) {
                int32_t l = W::ffs(m);
                m &= m - 1;
                int32_t lx = w.bcast(i < nw ? wlx[i] : 0, l);
                int32_t vv = w.bcast(i < nw ? wvs[i] : 0, l);
                if constexpr (W::N >= 64) {
                    if (w.lane() == lx) ldel[0] += vv;
                } else {
                    ldel[lx] += vv;
                }
            }
        }
        for (int32_t b = 0; b < cnt; b += W::N) {
            int32_t l = b + w.lane();
            int32_t v = 0, nl = 0;
            if (l < cnt) { /* the leaf's summary and its node id: one round trip */
                v = t.cls[c][l] + (W::N >= 64 ? ldel[0] : ldel[l]);
                nl = t.cleaf[c][l];
            }
            int32_t tot;
            int32_t p = run + w.excl_scan(v, &tot);
            uint64_t m = w.ballot(l < cnt && p < pos && pos <= p + v);
            if (m) {
                int32_t ll = W::ffs(m);
                *Pout = w.bcast(p, ll);
                *Nout = w.bcast(nl, ll);
                return (cpf << 6) | (b + ll);
            }
            run += tot;
        }
        fail(E_ASSERT); /* the chunk's leaves must add up to its summary */
        return -1;
    }
    /* tile_find of two positions pa <= pb (a range op's first and last rows): both chunks' leaf-summary lines are
     * read in one round trip. Same answers as two tile_find calls. */
    MT_HD void tile_find2(int32_t pa, int32_t pb, int32_t* ka, int32_t* Pa, int32_t* Na, int32_t* kb, int32_t* Pb,
                          int32_t* Nb) {
        MT_PROF_SCOPE(PH_TFIND);
        static_assert(W::N >= HT::TL::CH, "a lane per leaf of a chunk");
        auto& t = z.tl;
        int32_t ra = 0, rb = 0;
        *ka = *kb = -1;
        int32_t cpa = chunk_find(pa, &ra);
        int32_t cpb = chunk_find(pb, &rb);
        if (cpa < 0 || cpb < 0) return;
        int32_t ca = tcord[cpa], cb = tcord[cpb], na = tccnt[ca], nb = tccnt[cb];
        int32_t nw = t.wN;
        int32_t lda = 0, ldb = 0; /* lane l: the window rows' lengths in leaf l of each chunk */
        for (int32_t b = 0; b < nw; b += W::N) {
            int32_t i = b + w.lane();
            int32_t cp = i < nw ? wcp[i] : -1;
            uint64_t m = w.ballot(cp == cpa || cp == cpb);
            while (m) {
                int32_t l = W::ffs(m);
                m &= m - 1;
                int32_t lx = w.bcast(i < nw ? wlx[i] : 0, l);
                int32_t vv = w.bcast(i < nw ? wvs[i] : 0, l);
                int32_t c2 = w.bcast(cp, l);
                if (w.lane() == lx) {
                    if (c2 == cpa) lda += vv;
                    if (c2 == cpb) ldb += vv;
                }
            }
        }
        int32_t l = w.lane();
        int32_t va = 0, la = 0, vb = 0, lb = 0;
        if (l < na) { /* both chunks' leaf summaries and node ids: one round trip */
            va = t.cls[ca][l];
            la = t.cleaf[ca][l];
        }
        if (l < nb) {
            vb = t.cls[cb][l];
            lb = t.cleaf[cb][l];
        }
        va += lda;
        vb += ldb;
        int32_t tot;
        int32_t p = ra + w.excl_scan(l < na ? va : 0, &tot);
        uint64_t m = w.ballot(l < na && p < pa && pa <= p + va);
        if (m) {
            int32_t x = W::ffs(m);
            *Pa = w.bcast(p, x);
            *Na = w.bcast(la, x);
            *ka = (cpa << 6) | x;
        }
        p = rb + w.excl_scan(l < nb ? vb : 0, &tot);
        m = w.ballot(l < nb && p < pb && pb <= p + vb);
        if (m) {
            int32_t x = W::ffs(m);
            *Pb = w.bcast(p, x);
            *Nb = w.bcast(lb, x);
            *kb = (cpb << 6) | x;
        }
        if (*ka < 0 || *kb < 0) fail(E_ASSERT); /* the chunk's leaves must add up to its summary */
    }
    /* leaf_find of two (leaf, position) pairs in one round trip: lanes 0-7 read leaf na's rows, lanes 8-15 leaf
     * nb's. Same answers as two leaf_find calls. */
    MT_HD void leaf_find2(int32_t ka, int32_t na, int32_t Pa, int32_t pa, int32_t kb, int32_t nb, int32_t Pb, int32_t pb,
                          int32_t refSeq, int32_t client, int32_t* ta, int32_t* Poa, int32_t* Sa, int32_t* Va,
                          int32_t* tb, int32_t* Pob, int32_t* Sb, int32_t* Vb, HotRow* rowsA, int32_t* cA) {
        MT_PROF_SCOPE(PH_LFIND);
        static_assert(W::N >= 2 * MAXN, "a lane per row of two leaves");
        int32_t j = w.lane();
        bool A = j < MAXN, B = j >= MAXN && j < 2 * MAXN;
        int32_t n = A ? na : nb;
        int32_t s = n * MAXN + (j & (MAXN - 1));
        HotRow hr = load_row(s); /* lanes 0-7: leaf na's rows in full, for the split of the first row (split_row's pre) */
        RowView r{hr.len, hr.seq, hr.rseq,
                  (uint32_t)hr.cli | ((uint32_t)hr.rcli << 8) | ((uint32_t)hr.flags << 16) | ((uint32_t)hr.ng << 24)};
        *rowsA = hr;
        int32_t c = nch[n];
        *cA = w.bcast(c, 0);
        int32_t v = (A || B) && (j & (MAXN - 1)) < c ? vis_of(s, r, refSeq, client) : 0;
        int32_t tot;
        int32_t p = Pa + w.excl_scan(A ? v : 0, &tot);
        uint64_t m = w.ballot(A && p < pa && pa <= p + v);
        *ta = *tb = -1;
        if (m) {
            int32_t l = W::ffs(m);
            *Poa = w.bcast(p, l);
            *Sa = na * MAXN + l;
            *Va = w.bcast(v, l);
            *ta = ka * MAXN + l;
        }
        p = Pb + w.excl_scan(B ? v : 0, &tot);
        m = w.ballot(B && p < pb && pb <= p + v);
        if (m) {
            int32_t l = W::ffs(m);
            *Pob = w.bcast(p, l);
            *Sb = nb * MAXN + (l - MAXN);
            *Vb = w.bcast(v, l);
            *tb = kb * MAXN + (l - MAXN);
        }
        if (*ta < 0 || *tb < 0) fail(E_ASSERT);
    }
    /* within leaf position k (start offset P): the row t = k*8+j with P < pos <= P + vis */
    /* n: the leaf node at k (tile_find's) */
    /* *Sout / *Vout (optional): the row's slot and its perspective length */
    /* rowsOut / cOut (GPU): every lane's row (lane j: child j & 7) in full and the child count, for a split of the
     * found row that follows without another read of the leaf (split_row's pre) */
    MT_HD int32_t leaf_find(int32_t k, int32_t n, int32_t P, int32_t pos, int32_t refSeq, int32_t client, int32_t* Pout,
                            int32_t* Sout = nullptr, int32_t* Vout = nullptr, HotRow* rowsOut = nullptr,
                            int32_t* cOut = nullptr) {
        MT_PROF_SCOPE(PH_LFIND);
        if constexpr (W::N >= MAXN) { /* lane j: child j; one prefix scan */
            int32_t j = w.lane();
            int32_t s = n * MAXN + (j & (MAXN - 1));
            RowView r;
            if (rowsOut) { /* the whole row in the same pass */
                HotRow hr = load_row(s);
                r = RowView{hr.len, hr.seq, hr.rseq,
                            (uint32_t)hr.cli | ((uint32_t)hr.rcli << 8) | ((uint32_t)hr.flags << 16) | ((uint32_t)hr.ng << 24)};
                *rowsOut = hr;
            } else {
                r = row_view(s); /* the leaf's slab is always in bounds: loaded with the child count */
            }
            int32_t c = nch[n];
            if (cOut) *cOut = c;
            int32_t v = j < c ? vis_of(s, r, refSeq, client) : 0;
            int32_t tot;
            int32_t p = P + w.excl_scan(v, &tot);
            uint64_t m = w.ballot(j < c && p < pos && pos <= p + v);
            if (m) {
                int32_t l = W::ffs(m);
                *Pout = w.bcast(p, l);
                if (Sout) *Sout = n * MAXN + l;
                if (Vout) *Vout = w.bcast(v, l);
                return k * MAXN + l;
            }
            fail(E_ASSERT);
            return -1;
        }
        int32_t run = P, c = nch[n];
        for (int32_t j = 0; j < c; j++) {
            int32_t v = vis(n * MAXN + j, refSeq, client);
            if (run < pos && pos <= run + v) {
                *Pout = run;
                if (Sout) *Sout = n * MAXN + j;
                if (Vout) *Vout = v;
                return k * MAXN + j;
            }
            run += v;
        }
        fail(E_ASSERT);
        return -1;
    }
    /* perspectives the summaries cannot answer: a remote refSeq below minSeq (reads only) */
    MT_HD bool tiles_cover(int32_t refSeq, int32_t client) const {
        return is_local(client) || refSeq >= h.minSeq;
    }
    /* find_reach by a walk over every leaf (any perspective; O(rows)) */
    MT_HD int32_t find_reach_walk(int32_t pos, int32_t refSeq, int32_t client, int32_t* Pout, int32_t* Sout = nullptr,
                                  int32_t* Vout = nullptr) {
        int32_t run = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t n = leaf_at(k), c = nch[n];
            for (int32_t j = 0; j < c; j++) {
                int32_t v = vis(n * MAXN + j, refSeq, client);
                if (run < pos && pos <= run + v) {
                    *Pout = run;
                    if (Sout) *Sout = n * MAXN + j;
                    if (Vout) *Vout = v;
                    return k * MAXN + j;
                }
                run += v;
            }
        }
        return -1;
    }
    MT_HD int32_t find_reach_tiled(int32_t pos, int32_t refSeq, int32_t client, int32_t* Pout, int32_t* Sout,
                                   int32_t* Vout, HotRow* rowsOut = nullptr, int32_t* cOut = nullptr) {
        if (pos <= 0) return -1;
        if (!tiles_cover(refSeq, client)) return find_reach_walk(pos, refSeq, client, Pout, Sout, Vout);
        win_pass(refSeq, client);
        int32_t P;
        int32_t n = 0;
        int32_t k = tile_find(pos, refSeq, client, &P, &n);
        win_clear();
        if (k < 0) return -1;
        return leaf_find(k, n, P, pos, refSeq, client, Pout, Sout, Vout, rowsOut, cOut);
    }
    MT_HD int32_t length_tiled(int32_t refSeq, int32_t client) {
        if (!tiles_cover(refSeq, client)) {
            int32_t total = 0;
            for (int32_t k = 0; kvalid(k); k = knext(k)) {
                int32_t n = leaf_at(k), c = nch[n];
                for (int32_t j = 0; j < c; j++) total += vis(n * MAXN + j, refSeq, client);
            }
            return total;
        }
        int32_t total = win_pass(refSeq, client);
        win_clear();
        return total + stable_total();
    }

    /* ---- perspective scans ------------------------------------------------------------- */
    /* The scans walk the document-order slot space t = k * 8 + j (leaf lorder[k], child j). A lane
     * covers a quad of 4 consecutive slots (half a leaf slab, contiguous in the SoA columns), so one
     * pass of the wave covers 256 slots with one lorder read and one 16-byte read per int32 column,
     * and the position search is a per-lane 4-step prefix plus one wavefront exclusive scan. */
    MT_HD int32_t quad_slot(int32_t t0) const { /* t0 % 4 == 0; -1 past the last leaf */
        int32_t k = t0 >> 3;
        if (k >= h.nleaf) return -1;
        return lo[k] * MAXN + (t0 & 4);
    }
#ifndef MT_SCAN_NB
#define MT_SCAN_NB 1 /* flat-profile position scans: wave blocks (256 slots each) per round trip; 2 and 3 measured
                        * 9 % and 27 % slower on config 3 (r04n: the second block's 16 registers spill at 8 waves) */
#endif
    /* ---- removedClientOverlap: 8 entries inline in the cold row, then chains of 8-entry blocks
     * in a per-document pool (entries are short id + 1; 0 ends a list) ------------------------ */
    MT_HD bool ovl_has(int32_t s, int32_t client) const {
        uint64_t ov = cold(s).ovl;
        for (int32_t b = cold(s).ovx;; b = z.ovn[b]) {
#pragma clang loop unroll(disable)
            for (int k = 0; k < NOVL; k++) { /* a rare path: kept rolled (it is inlined at every visibility test) */
                uint32_t e = (uint32_t)((ov >> (8 * k)) & 0xFF);
                if (e == 0) return false;
                if ((int32_t)e - 1 == client) return true;
            }
            if (!b) return false;
            ov = z.ovp[b];
        }
    }
    /* the k-th entry (short id) of row s's overlap list; -1 past its end */
    MT_HD int32_t ovl_at(int32_t s, int32_t k) const {
        uint64_t ov = cold(s).ovl;
        int32_t b = cold(s).ovx;
        while (k >= NOVL) {
            if (!b) return -1;
            ov = z.ovp[b];
            b = z.ovn[b];
            k -= NOVL;
        }
        uint32_t e = (uint32_t)((ov >> (8 * k)) & 0xFF);
        return e ? (int32_t)e - 1 : -1;
    }
    MT_HD int32_t ovl_count(int32_t s) const {
        int32_t n = 0;
        while (ovl_at(s, n) >= 0) n++;
        return n;
    }
    /* removedClientOverlap.push(client) */
    MT_HD void ovl_push(int32_t s, int32_t client) {
        uint64_t e = (uint64_t)(client + 1);
        int32_t k = 0;
        uint64_t ov = cold(s).ovl;
        while (k < NOVL && ((ov >> (8 * k)) & 0xFF)) k++;
        if (k < NOVL) {
            cold(s).ovl = ov | (e << (8 * k));
            return;
        }
        int32_t b = cold(s).ovx, last = 0;
        while (b) {
            last = b;
            b = z.ovn[b];
        }
        if (last) {
            ov = z.ovp[last];
            for (k = 0; k < NOVL && ((ov >> (8 * k)) & 0xFF); k++) {
            }
            if (k < NOVL) {
                z.ovp[last] = ov | (e << (8 * k));
                return;
            }
        }
        int32_t nb = ovb_alloc();
        if (!nb) return;
        z.ovp[nb] = e;
        if (last)
            z.ovn[last] = (uint16_t)nb;
        else
            cold(s).ovx = (uint16_t)nb;
    }
    /* a split's right part gets its own copy of the left part's overflow chain */
    MT_HD void ovl_clone(int32_t rs, int32_t ls) {
        cold(rs).ovx = 0;
        int32_t prev = 0;
        for (int32_t src = cold(ls).ovx; src; src = z.ovn[src]) {
            int32_t nb = ovb_alloc(); /* a sweep here keeps both chains: rs holds what is linked */
            if (!nb) return;
            z.ovp[nb] = z.ovp[src];
            if (prev)
                z.ovn[prev] = (uint16_t)nb;
            else
                cold(rs).ovx = (uint16_t)nb;
            prev = nb;
        }
    }
    MT_HD int32_t ovb_alloc() {
        if (!zh->ovFree && zh->ovTop >= OVB) ovb_sweep();
        int32_t b;
        if (zh->ovFree) {
            b = zh->ovFree;
            zh->ovFree = z.ovn[b];
        } else if (zh->ovTop < OVB) {
            b = zh->ovTop++;
        } else {
            fail(E_CAPACITY);
            return 0;
        }
        z.ovn[b] = 0;
        z.ovp[b] = 0;
        return b;
    }
    /* blocks no live row's chain reaches (their rows were unlinked or their ids reused) return to
     * the free list */
    MT_HD void ovb_sweep() {
        uint64_t used = 1;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t n = leaf_at(k), c = nch[n];
            for (int32_t j = 0; j < c; j++) {
                int32_t s = n * MAXN + j;
                if (z.flags(s) & RF_OVL)
                    for (int32_t b = cold(s).ovx; b; b = z.ovn[b]) used |= 1ull << b;
            }
        }
        zh->ovFree = 0;
#pragma clang loop unroll(disable)
        for (int32_t b = OVB - 1; b >= 1; b--)
            if (!((used >> b) & 1)) {
                z.ovn[b] = (uint16_t)zh->ovFree;
                zh->ovFree = b;
            }
    }
    /* the scan columns of the 4 slots from s0 (len, rseq; seq and {cli, rcli, flags, ng} unless the
     * perspective is the local view), loaded apart from their use so that a scan can issue several quads'
     * loads in one round trip */
    struct QuadRows {
        I4 L, R, Q, BY;
    };
    /* lanes with s0 < 0 (past the last leaf) and the fields a local perspective does not use are left unset:
     * quad_vis_of reads neither (zeroing them cost 16 moves per scanned block) */
    MT_HD QuadRows quad_load(int32_t s0, bool local) const {
        QuadRows x;
        if (s0 >= 0) {
            x.L = ld4(&z.len(s0));
            x.R = ld4(&z.rseq(s0));
            if (!local) {
                x.Q = ld4(&z.seq(s0));
                x.BY = ld4(z.bytes4(s0));
            }
        }
        return x;
    }
    /* nodeLength (mergeTree.ts:1692-1732) of the 4 slots from s0 under (refSeq, client); 0 for
     * empty slots */
    MT_HD void quad_vis(int32_t s0, int32_t refSeq, int32_t client, int32_t v[4]) const {
        quad_vis_of(s0, quad_load(s0, is_local(client)), refSeq, client, v);
    }
    MT_HD void quad_vis_of(int32_t s0, const QuadRows& x, int32_t refSeq, int32_t client, int32_t v[4]) const {
        if (s0 < 0) {
            v[0] = v[1] = v[2] = v[3] = 0;
            return;
        }
        const I4& L = x.L;
        const I4& R = x.R;
        if (is_local(client)) { /* localNetLength (mergeTree.ts:1195-1206) */
            for (int q = 0; q < 4; q++) v[q] = R.x[q] == NOREM ? L.x[q] : 0;
            return;
        }
        const I4& Q = x.Q;
        const I4& BY = x.BY; /* {cli, rcli, flags, ng} of the 4 slots */
        int32_t ovq = 0;
        /* the same tests in fewer instructions: a short id byte equals the client's (LocalClientId -1 is byte 0xFF,
         * LOCAL_CLIENT), and "s != UNASSIGNED_SEQ && s <= refSeq" is one unsigned compare against refSeq + 1 (0 when
         * refSeq < 0): UNASSIGNED_SEQ (-1) and NOREM (INT32_MIN) are above every bound as unsigned values */
        const uint32_t uc = client_byte(client);
        const uint32_t ur1 = refSeq >= 0 ? (uint32_t)refSeq + 1u : 0u;
        for (int q = 0; q < 4; q++) {
            uint32_t by = (uint32_t)BY.x[q];
            uint32_t cq = by & 0xFFu, rcq = (by >> 8) & 0xFFu, fq = (by >> 16) & 0xFFu;
            int32_t sq = Q.x[q];
            bool ok = L.x[q] > 0 && (cq == uc || (uint32_t)sq < ur1);
            int32_t rs = R.x[q];
            if (ok && rs != NOREM) {
                if (rcq == uc || (uint32_t)rs < ur1)
                    ok = false;
                else if (fq & RF_OVL)
                    ovq |= 1 << q; /* removedClientOverlap: looked up once below, not in each unrolled slot */
            }
            v[q] = ok ? L.x[q] : 0;
        }
        int32_t hid = 0; /* slots a removedClientOverlap entry hides from the client */
#pragma clang loop unroll(disable)
        while (ovq) {
            int32_t q = __builtin_ctz(ovq);
            ovq &= ovq - 1;
            if (ovl_has(s0 + q, client)) hid |= 1 << q;
        }
        for (int q = 0; q < 4; q++)
            if ((hid >> q) & 1) v[q] = 0;
    }
    /* Total length under a perspective (getLength, mergeTree.ts:1610). */
    MT_HD int32_t length(int32_t refSeq, int32_t client) {
        if constexpr (TILED) return length_tiled(refSeq, client);
        int32_t total = 0;
        int32_t T = h.nleaf * MAXN;
        for (int32_t b = 0; b < T; b += 4 * W::N) {
            int32_t v[4];
            quad_vis(quad_slot(b + 4 * w.lane()), refSeq, client, v);
            total += w.sum(v[0] + v[1] + v[2] + v[3]);
        }
        return total;
    }
    /* First row (document order) with P < pos <= P + vis; returns t (lorder coordinate) or -1,
     * and P of that row; *Sout / *Vout (optional): its slot and perspective length. */
    MT_HD int32_t find_reach(int32_t pos, int32_t refSeq, int32_t client, int32_t* Pout, int32_t* Sout = nullptr,
                             int32_t* Vout = nullptr, HotRow* rowsOut = nullptr,
                             int32_t* cOut = nullptr) {
        MT_PROF_SCOPE(PH_FIND);
        if constexpr (TILED) return find_reach_tiled(pos, refSeq, client, Pout, Sout, Vout, rowsOut, cOut);
        int32_t run = 0;
        int32_t T = h.nleaf * MAXN;
        const bool loc = is_local(client);
        constexpr int NB = W::N >= 64 ? MT_SCAN_NB : 1; /* wave blocks whose loads are issued together */
        for (int32_t b0 = 0; b0 < T; b0 += NB * 4 * W::N) {
            int32_t s0[NB];
            QuadRows x[NB];
#pragma unroll
            for (int q = 0; q < NB; q++) s0[q] = quad_slot(b0 + q * 4 * W::N + 4 * w.lane());
#pragma unroll
            for (int q = 0; q < NB; q++) x[q] = quad_load(s0[q], loc);
#pragma unroll
            for (int bq = 0; bq < NB; bq++) {
                int32_t b = b0 + bq * 4 * W::N;
                if (b >= T) return -1;
                int32_t v[4];
                quad_vis_of(s0[bq], x[bq], refSeq, client, v);
                int32_t tot;
                int32_t p = run + w.excl_scan(v[0] + v[1] + v[2] + v[3], &tot);
                int32_t hq = -1, hp = 0, hv = 0;
                for (int q = 0; q < 4; q++) {
                    if (hq < 0 && p < pos && pos <= p + v[q]) {
                        hq = q;
                        hp = p;
                        hv = v[q];
                    }
                    p += v[q];
                }
                uint64_t m = w.ballot(hq >= 0);
                if (m) {
                    int32_t l = W::ffs(m);
                    *Pout = w.bcast(hp, l);
                    if (Sout) *Sout = w.bcast(s0[bq] + hq, l);
                    if (Vout) *Vout = w.bcast(hv, l);
                    return b + 4 * l + w.bcast(hq, l);
                }
                run += tot;
                if (run >= pos && pos > 0) return -1;
            }
        }
        return -1;
    }

    /* ---- structure: inserting a row into a leaf slab --------------------------------- */
    /* Insert an empty row slot at child index j of leaf n (shift right). Returns the slot of
     * the new row, or -1. May split the leaf (and ancestors) afterwards; the returned slot is
     * remapped by `place_after_split` — callers use the returned final slot. */
    MT_HD void node_insert_child(int32_t p, int32_t idx, int32_t child) {
        /* interior node p: insert `child` at idx (insertChildNode, mergeTree.ts:2162-2172) */
        int32_t n = nch[p];
        for (int32_t i = n; i > idx; i--) z.KIDS(p * MAXN + i) = z.KIDS(p * MAXN + i - 1);
        z.KIDS(p * MAXN + idx) = (IX)child;
        nch[p] = (int8_t)(n + 1);
        npar[child] = (IX)p;
    }
    MT_HD int32_t child_index(int32_t p, int32_t child) const {
        for (int32_t i = 0; i < nch[p]; i++)
            if (z.KIDS(p * MAXN + i) == child) return i;
        return -1;
    }
    /* insert leaf `nl` into lorder right after leaf `after` */
    MT_HD void lorder_insert_after(int32_t after, int32_t nl) {
        if constexpr (TILED) {
            rope_insert_after(after, nl);
            h.nleaf++;
            note_leaves();
            return;
        }
        int32_t k = lp[after] + 1;
        int32_t n = h.nleaf;
        lorder_shift(k, n, 1);
        lo[k] = (IX)nl;
        lp[nl] = (IX)k;
        h.nleaf = n + 1;
        note_leaves();
    }
    /* split (mergeTree.ts:2509-2522) of a full node (8 children) into 4 + 4; the new node is
     * inserted after it in its parent, recursively; root split -> updateRoot (1909-1920).
     * Returns the new node. */
    MT_HD int32_t split_node(int32_t n0) {
        int32_t first = -1;
        int32_t n = n0;
        for (;;) { /* iterative: a split may overflow the parent, up to the root */
            int8_t lvl = nlev[n];
            int32_t nn = alloc_node(lvl);
            if (nn < 0) return -1;
            if (first < 0) first = nn;
            if constexpr (W::N >= MAXN) {
                /* children 4..7 move to the new node in one pass, a lane each: rows (with their leaf link,
                 * from the ids just read, and the vacated slots' lengths) or child nodes (with their parent) */
                const int32_t l = w.lane();
                const bool mv = l < 4;
                if (lvl == 0) {
                    HotRow r;
                    if (mv) r = load_row(n * MAXN + 4 + l);
                    w.sync();
                    if (mv) {
                        store_row(nn * MAXN + l, r);
                        if ((int32_t)r.rid >= 0) z.RLEAF(r.rid) = (IX)nn; /* a slot awaiting its row holds -1 */
                        z.len(n * MAXN + 4 + l) = 0;
                    }
                } else {
                    int32_t c = mv ? (int32_t)z.KIDS(n * MAXN + 4 + l) : 0;
                    w.sync();
                    if (mv) {
                        z.KIDS(nn * MAXN + l) = (IX)c;
                        npar[c] = (IX)nn;
                    }
                }
                w.sync();
            } else if (lvl == 0) {
                move_rows(nn * MAXN, n * MAXN + 4, 4);
                set_leaf_of_rows(nn, 4);
                clear_slots(n * MAXN + 4, 4);
            } else {
                for (int32_t i = 0; i < 4; i++) {
                    int32_t c = z.KIDS(n * MAXN + 4 + i);
                    z.KIDS(nn * MAXN + i) = (IX)c;
                    npar[c] = (IX)nn;
                }
            }
            nch[n] = 4;
            nch[nn] = 4;
            if (lvl == 0) lorder_insert_after(n, nn);
            if constexpr (TILED) {
                if (lvl == 0) {
                    int32_t two[2] = {n, nn};
                    leaves_restat(two, 2);
                }
            }
            int32_t p = npar[n];
            if (p < 0) {
                int32_t r = alloc_node((int8_t)(lvl + 1));
                if (r < 0) return -1;
                z.KIDS(r * MAXN + 0) = (IX)n;
                z.KIDS(r * MAXN + 1) = (IX)nn;
                nch[r] = 2;
                npar[n] = (IX)r;
                npar[nn] = (IX)r;
                zh->root = r;
                return first;
            }
            if constexpr (W::N >= MAXN) {
                /* child_index + node_insert_child in one pass: lane i reads child i of p; the children after n
                 * move right one place from registers */
                const int32_t l = w.lane();
                int32_t cnt = nch[p];
                int32_t kid = l < MAXN ? (int32_t)z.KIDS(p * MAXN + (l & (MAXN - 1))) : -1;
                uint64_t m = w.ballot(l < cnt && kid == n);
                int32_t idx = (m ? W::ffs(m) : -1) + 1;
                w.sync();
                if (l >= idx && l < cnt) z.KIDS(p * MAXN + l + 1) = (IX)kid;
                if (l == 0) z.KIDS(p * MAXN + idx) = (IX)nn;
                w.sync();
                nch[p] = (int8_t)(cnt + 1);
                npar[nn] = (IX)p;
            } else {
                node_insert_child(p, child_index(p, n) + 1, nn);
            }
            if (nch[p] < MAXN) return first;
            n = p;
        }
    }
    /* Make room at child index j of leaf n; returns slot for the new row (after any split). */
    /* dup: the new slot starts as a copy of the row before it (j >= 1; a split's right part), made
     * by the same parallel shift instead of a separate row copy */
    MT_HD int32_t leaf_insert_slot(int32_t n, int32_t j, bool dup = false) {
        MT_PROF_SCOPE(PH_LEAFINS);
        int32_t c = nch[n];
        slab_shift_right(n, dup ? j - 1 : j, c);
        z.RID(n * MAXN + j) = -1; /* not a row yet (a leaf split must not re-home it): the caller assigns one */
        if constexpr (TILED)
            if (!dup) z.tl.xf[n * MAXN + j] = 0;
        nch[n] = (int8_t)(c + 1);
        if (c + 1 >= MAXN) {
            int32_t nn = split_node(n);
            if (nn < 0) return -1;
            if (j >= 4) return nn * MAXN + (j - 4);
        }
        return n * MAXN + j;
    }

    /* ---- text arena -------------------------------------------------------------------- */
    MT_HD uint16_t* arena_base(int32_t side) { return d.arena() + (int64_t)side * d.caps.acap; }
    /* reserve n units at the arena top; compacts into the other half when full */
    MT_HD int32_t arena_alloc(int32_t n) {
        if (h.arenaTop + n > d.caps.acap) {
            arena_gc();
            if (h.arenaTop + n > d.caps.acap) {
                fail(E_CAPACITY);
                return -1;
            }
        }
        int32_t off = h.arenaTop;
        h.arenaTop = off + n;
        return off;
    }
    /* copy n units (wave-parallel); returns the last unit copied (0 if n == 0) */
    MT_HD int32_t arena_copy(uint16_t* dst, const uint16_t* src, int32_t n) {
        int32_t last = 0;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            uint16_t v = i < n ? src[i] : 0;
            w.sync();
            if (i < n) dst[i] = v;
            if (b + W::N >= n) last = w.bcast(v, n - 1 - b);
        }
        w.sync();
        return last;
    }
    /* copy all live text rows into the other half, in document order. A row id is moved once
     * per GC even if its slot is transiently duplicated (scour compacts a slab in place). */
    MT_HD void arena_gc() {
        int32_t from = zh->arenaSide, to = from ^ 1;
        uint16_t* src = arena_base(from);
        uint16_t* dst = arena_base(to);
        int32_t ep = zh->gcEpoch % 255 + 1;
        zh->gcEpoch = ep;
        int32_t top = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t n = leaf_at(k), c = nch[n];
            for (int32_t j = 0; j < c; j++) {
                int32_t s = n * MAXN + j;
                if ((z.flags(s) & RF_NOTEXT) || cold(s).gc == ep) continue;
                int32_t L = z.len(s);
                arena_copy(dst + top, src + cold(s).toff, L);
                cold(s).toff = (uint32_t)top;
                cold(s).gc = (uint8_t)ep;
                top += L;
            }
        }
        zh->arenaSide = to;
        h.arenaTop = top;
        w.sync();
    }

    /* ---- splitAt (mergeTree.ts:523-567, textSegment.ts:103-111) ------------------------ */
    /* split_row on the GPU without delta events or local references, in two round trips: the leaf's rows (the
     * row being split and the ones the slab shift moves), its child count and the free row-id stack's top are
     * read in one pass, the row's cold record (one dword per lane) in a second; the shift, the new row and its
     * cold copy are then written from registers. Same result as the serial form below. */
    /* gapOut (an insert placed right after the left part, insert_row): when the leaf has room for both, the same
     * write pass also leaves an empty slot between the halves for the new row (rows after the split move two
     * slots), which *gapOut returns — the shift leaf_insert_slot would make with a second read of the leaf */
    MT_HD int32_t split_row_par(int32_t n, int32_t j, int32_t off, int32_t* rsOut, int32_t* gapOut = nullptr,
                                const HotRow* pre = nullptr, int32_t preC = -1, int32_t* ridOut = nullptr) {
        constexpr int CW = (int)(sizeof(typename HT::Cold) / 4);
        static_assert(W::N >= CW && W::N >= MAXN, "a lane per cold dword and per slot");
        const int32_t l = w.lane();
        int32_t s0 = n * MAXN + j;
        HotRow rr = pre ? *pre : load_row(n * MAXN + (l & (MAXN - 1)));
        int32_t c = pre ? preC : nch[n];
        int32_t nfr = zh->nfreeRid;
        int32_t frr = d.FRID(nfr > 0 ? nfr - 1 : 0);
        uint32_t fl0 = (uint32_t)w.bcast((int32_t)rr.flags, j);
        if (fl0 & RF_MARKER) return s0; /* Marker.createSplitSegmentAt -> undefined */
        int32_t rid0 = w.bcast((int32_t)rr.rid, j), len0 = w.bcast(rr.len, j);
        uint32_t ng0 = (uint32_t)w.bcast((int32_t)rr.ng, j), xf0 = (uint32_t)w.bcast((int32_t)rr.xf, j);
        typename HT::Cold* cd = d.cold();
        const int32_t* csrc = (const int32_t*)&cd[rid0];
        int32_t cv = l < CW ? csrc[l] : 0; /* the row's cold record: toff is dword 2, ovx the top of dword 3 */
        /* leaf_insert_slot(n, j + 1, dup): rows j..c-1 move right one slot; slot j + 1 starts as row j (with a gap:
         * two slots, slot j + 2 starts as row j and slot j + 1 is the new row's) */
        const int32_t g = gapOut && c + 2 < MAXN ? 1 : 0;
        bool willSplit = c + 1 >= MAXN;
        {
            MT_PROF_SCOPE(PH_LEAFINS);
            bool mv = l >= j && l < c && l < MAXN;
            w.sync();
            if (mv) store_row(n * MAXN + l + 1 + g, rr);
            w.sync();
            z.RID(n * MAXN + j + 1) = -1; /* not a row yet (a leaf split must not re-home it) */
            if (g) {
                if constexpr (TILED) z.tl.xf[n * MAXN + j + 1] = 0;
                *gapOut = n * MAXN + j + 1;
            }
            nch[n] = (int8_t)(c + 1 + g);
        }
        int32_t rs = n * MAXN + j + 1 + g;
        if constexpr (TILED) { /* a leaf split re-sums both leaves (split_node): the halves' lengths go first */
            if (willSplit && (xf0 & XF_STABLE)) {
                z.len(s0) = off < len0 ? off : len0;
                z.len(rs) = off < len0 ? len0 - off : 0;
            }
        }
        if (willSplit) {
            MT_PROF_SCOPE(PH_LEAFINS);
            int32_t nn = split_node(n);
            if (nn < 0) return -1;
            if (j + 1 >= 4) rs = nn * MAXN + (j + 1 - 4);
        }
        /* the left part stays at n*8+j unless the leaf split moved children 4..7 (then it sits just before the
         * new slot, in the new leaf) */
        int32_t ls = willSplit && j >= 4 ? rs - 1 : s0;
        int32_t rrid;
        if (zh->nfreeRid == nfr && nfr > 0) { /* alloc_rid, with the stack's top read above */
            zh->nfreeRid = nfr - 1;
            rrid = frr;
        } else {
            rrid = alloc_rid();
        }
        z.RID(rs) = (IX)rrid;
        z.RLEAF(rrid) = (IX)(rs / MAXN);
        /* splitAt copies every field (mergeTree.ts:523-567); the right part's text offset (or a PermutationSegment's
         * start + pos, unallocated staying 0) and its length differ */
        uint32_t toff0 = (uint32_t)w.bcast(cv, 2);
        uint32_t ovx0 = (uint32_t)w.bcast(cv, 3) >> 16;
        uint32_t rtoff;
        int32_t lenR;
        if (off < len0) {
            lenR = len0 - off;
            rtoff = ((fl0 & RF_PERM) && toff0 == 0) ? 0u : toff0 + (uint32_t)off;
        } else { /* a split at or past the end: the right part is an empty segment (textSegment.ts:103-111) */
            lenR = 0;
            rtoff = toff0 + (uint32_t)len0;
        }
        int32_t* cdst = (int32_t*)&cd[rrid];
        if (l < CW) cdst[l] = l == 2 ? (int32_t)rtoff : cv;
        /* a retired client byte: the right part's long ids (the retired-client table is by row id) */
        if constexpr (RECLAIM) {
            const uint32_t cb0 = (uint32_t)w.bcast((int32_t)rr.cli | ((int32_t)rr.rcli << 8), j);
            if ((cb0 & 0xFF) == RETIRED_CLIENT || (cb0 >> 8) == RETIRED_CLIENT) d.RCL(rrid) = d.RCL(rid0);
        }
        w.sync();
        if (ovx0) ovl_clone(rs, ls);
        z.len(rs) = lenR;
        if (off < len0) {
            z.len(ls) = off;
            z.flags(ls) = (uint8_t)(fl0 & ~(uint32_t)RF_NLK); /* the left part's last unit is not known any more */
        } else {
            z.flags(rs) = (uint8_t)((fl0 & ~(uint32_t)RF_NL) | RF_NLK);
        }
        h.nrows++;
        zh->sumW += 2;
        if constexpr (TILED) {
            if (xf0 & XF_W) win_add(rrid, rs);
            /* STABLE halves: in one leaf, its sum is unchanged; after a leaf split, split_node re-summed both
             * leaves with the halves' lengths written above */
        }
        if (ng0) split_groups(rid0, rrid, (int32_t)ng0); /* segmentGroups.copyTo */
        if (rsOut) *rsOut = rs;
        if (ridOut) *ridOut = rrid;
        return ls;
    }
    /* Split the row at lorder coordinate t at offset off (0 < off < len). Returns the slot of
     * the LEFT part afterwards (the right part is the next row in document order). */
    /* pre / preC (GPU): the leaf's rows (lane l: child l & 7) and child count as a search just read them */
    /* ridOut: the right part's row id (the caller need not read back what the split wrote) */
    MT_HD int32_t split_row(int32_t t, int32_t off, int32_t* rsOut = nullptr, int32_t* gapOut = nullptr,
                            const HotRow* pre = nullptr, int32_t preC = -1, int32_t* ridOut = nullptr) {
        MT_PROF_SCOPE(PH_SPLIT);
        int32_t n = leaf_at(t >> 3), j = t & 7;
        int32_t s0 = n * MAXN + j;
        if constexpr (W::N >= 64) {
            if (!dl_on() && !refs_on()) return split_row_par(n, j, off, rsOut, gapOut, pre, preC, ridOut);
        }
        if (z.flags(s0) & RF_MARKER) return s0; /* Marker.createSplitSegmentAt -> undefined */
        bool willSplit = nch[n] + 1 >= MAXN;
        int32_t rs = leaf_insert_slot(n, j + 1, true); /* rs starts as a copy of the row */
        if (rs < 0) return -1;
        /* the left part stays at n*8+j unless the leaf split moved children 4..7 (then it sits just
         * before the new slot, in the new leaf) */
        int32_t ls = n * MAXN + j;
        if (willSplit && j >= 4) ls = rs - 1;
        int32_t rrid = alloc_rid();
        z.RID(rs) = (IX)rrid;
        z.RLEAF(rrid) = (IX)(rs / MAXN);
        typename HT::Cold& cl = cold(ls);
        typename HT::Cold& cr = d.COLD(rrid);
        copy_cold(rs, ls); /* splitAt copies every field (mergeTree.ts:523-567) */
        if (RECLAIM && (z.cli(ls) == RETIRED_CLIENT || z.rcli(ls) == RETIRED_CLIENT)) d.RCL(rrid) = d.RCL(z.RID(ls));
        if (cl.ovx) ovl_clone(rs, ls);
        if (refs_on()) refs_split(z.RID(ls), rrid, off);
        int32_t lenL = z.len(ls);
        if (off < lenL) {
            z.len(rs) = lenL - off;
            /* the text offset, or PermutationSegment.createSplitSegmentAt's start + pos (unallocated stays) */
            cr.toff = ((z.flags(ls) & RF_PERM) && cl.toff == 0) ? 0u : cl.toff + (uint32_t)off;
            z.len(ls) = off;
            z.flags(ls) &= (uint8_t)~RF_NLK; /* the left part's last unit is not known any more */
        } else { /* a split at or past the end (a local reference past its segment's end): text.substring(off)
                    is "", so the right part is an empty segment and the left keeps its text
                    (textSegment.ts:103-111); insert_at_ref admits text rows only */
            z.len(rs) = 0;
            cr.toff = cl.toff + (uint32_t)lenL;
            z.flags(rs) = (uint8_t)((z.flags(rs) & ~RF_NL) | RF_NLK);
        }
        h.nrows++;
        zh->sumW += 2;
        if constexpr (TILED) {
            if (z.tl.xf[rs] & XF_W) win_add(z.RID(rs), rs);
            if (z.tl.xf[rs] & XF_STABLE) { /* the halves may sit in two leaves after a leaf split */
                int32_t two[2] = {ls / MAXN, rs / MAXN};
                leaves_restat(two, rs / MAXN != ls / MAXN ? 2 : 1);
            }
        }
        /* segmentGroups.copyTo (segmentGroupCollection.ts:37-39): the new segment joins the
         * same pending groups (in the row's FIFO order = log order), appended at the end of each
         * group's segment list */
        if (z.ng(ls)) split_groups(z.RID(ls), z.RID(rs), z.ng(ls));
        if (dl_on()) { /* MergeTreeMaintenanceType.SPLIT (mergeTree.ts:2264-2269): [segment, next] */
            dhead(MT_DELTA_SPLIT);
            dseg(-1, z.len(ls));
            dseg(-1, z.len(rs));
            dtail(2);
        }
        if (rsOut) *rsOut = rs;
        if (ridOut) *ridOut = rrid;
        return ls;
    }

    /* ---- segment groups ---------------------------------------------------------------- */
    /* an index of the pending-group ring in [0, 2 gcap) reduced to [0, gcap): gqHead stays reduced, so no integer
     * division (tens of instructions on the GPU) */
    MT_HD int32_t gq_wrap(int32_t x) const { return x >= d.caps.gcap ? x - d.caps.gcap : x; }
    /* segmentGroups.copyTo (segmentGroupCollection.ts:37-39) of a split: the right part (rrid) joins the same
     * pending groups as the left (lrid, in ng of them), in the row's FIFO order = log order, appended at the end
     * of each group's segment list */
    MT_HD void split_groups(int32_t lrid, int32_t rrid, int32_t ng) {
        if (zh->memN + ng > d.caps.mcap) mem_compact();
        int32_t head = zh->gqN ? d.GQ(zh->gqHead) : 0x7fffffff;
        int32_t m0 = zh->memN;
        for (int32_t b = 0; b < m0; b += W::N) {
            int32_t i = b + w.lane();
            int32_t g = i < m0 ? d.MGID(i) : -1;
            uint64_t m = w.ballot(i < m0 && d.MRID(i) == lrid && g >= head);
            while (m) {
                int32_t l = W::ffs(m);
                m &= m - 1;
                mem_append(w.bcast(g, l), rrid);
            }
        }
    }
    MT_HD void mem_append(int32_t gid, int32_t rid) {
        int32_t m = zh->memN;
        if (m >= d.caps.mcap) {
            mem_compact();
            m = zh->memN;
            if (m >= d.caps.mcap) {
                fail(E_CAPACITY);
                return;
            }
        }
        d.MGID(m) = gid;
        d.MRID(m) = rid;
        zh->memN = m + 1;
    }
    /* drop entries of groups already acked (gid < head gid): wave stream compaction */
    MT_HD void mem_compact() {
        int32_t head = zh->gqN ? d.GQ(zh->gqHead) : 0x7fffffff;
        int32_t n = zh->memN, wpos = 0;
        for (int32_t b = 0; b < n; b += W::N) {
            int32_t i = b + w.lane();
            int32_t g = i < n ? d.MGID(i) : -1;
            int32_t sd = i < n ? d.MRID(i) : 0;
            bool keep = i < n && g >= head;
            int32_t tot;
            int32_t off = w.excl_scan(keep ? 1 : 0, &tot);
            w.sync();
            if (keep) {
                d.MGID(wpos + off) = g;
                d.MRID(wpos + off) = sd;
            }
            w.sync();
            wpos += tot;
        }
        zh->memN = wpos;
    }
    /* SegmentGroupCollection.enqueue (segmentGroupCollection.ts:28-31) */
    MT_HD void row_enqueue_group(int32_t s, int32_t gid) {
        int32_t ng = z.ng(s);
        if (ng >= 255) {
            fail(E_CAPACITY);
            return;
        }
        z.ng(s) = (uint8_t)(ng + 1);
        mem_append(gid, z.RID(s));
    }
    /* addToPendingList (mergeTree.ts:1955-1962). Group ids come from a per-document counter, so they
     * increase along the pending queue (acks and compaction compare them with the head's); the ring
     * beside the queue keeps each group's SegmentGroup.localSeq (findReconnectionPostition uses it). */
    MT_HD void pending_add(int32_t s, int32_t localSeq, bool* created) {
        if (!*created) {
            if (zh->gqN >= d.caps.gcap) {
                fail(E_CAPACITY);
                return;
            }
            group_push(localSeq);
            *created = true;
        }
        row_enqueue_group(s, d.GQ(gq_wrap(zh->gqHead + zh->gqN - 1)));
    }
    /* pendingSegments.enqueue of a new group (the caller checked the ring's room) */
    MT_HD void group_push(int32_t localSeq) {
        int32_t gid = zh->gidNext;
        zh->gidNext = gid + 1;
        int32_t q = gq_wrap(zh->gqHead + zh->gqN);
        d.GQ(q) = gid;
        d.GQL(q) = localSeq;
        zh->gqN++;
    }

    /* ---- zamboni heap (collections.ts:212-264, LRUSegmentComparer mergeTree.ts:957-960) ---- */
    MT_HD void heap_swap(int32_t i, int32_t j) {
        IX tr = hrd[i];
        int32_t tq = hsq[i];
        uint8_t tg = hgn[i];
        hrd[i] = hrd[j];
        hsq[i] = hsq[j];
        hgn[i] = hgn[j];
        hrd[j] = tr;
        hsq[j] = tq;
        hgn[j] = tg;
    }
    /* Heap.add + fixup (collections.ts:221-225, 240-247). On the GPU the sift-up is one step: the
     * ancestors of the new leaf position are read in parallel (lane i: the (i+1)-th ancestor), the
     * ones it passes are exactly the leading run with maxSeq greater than it (ancestors are ordered
     * along a path), and they all move down one level at once. */
    /* gen: the row id's generation if the caller has read it (-1: read here) */
    MT_HD void heap_add(int32_t rid, int32_t seq, int32_t knownGen = -1) {
        MT_PROF_SCOPE(PH_HEAP);
        int32_t n = h.heapN;
        if (n >= HCAPR) {
            fail(E_CAPACITY);
            return;
        }
        MT_PROF_COUNT(PH_C_PUSH, 1);
        int32_t k = n + 1; /* L[k] (1-based) lives at index k-1 */
        h.heapN = n + 1;
        if (n + 1 > zh->hwHeap) zh->hwHeap = n + 1;
        uint8_t gen = knownGen >= 0 ? (uint8_t)knownGen : z.RGEN(rid);
        if (seq >= hmax) { /* every ancestor's maxSeq <= hmax <= seq: the fixup moves nothing (collections.ts:240-247) */
            hmax = seq;
            if (w.lane() == 0) {
                hrd[n] = (IX)rid;
                hsq[n] = seq;
                hgn[n] = gen;
            }
            w.sync();
            if (n == 0) zh->heapTop = seq;
            return;
        }
        if constexpr (W::N >= 32) {
            int32_t l = w.lane();
            int32_t a = l < 31 ? (k >> (l + 1)) : 0; /* ancestor l+1 (0 = none) */
            int32_t as = a >= 1 ? hsq[a - 1] : 0;
            uint64_t m = w.ballot(a >= 1 && as - seq > 0);
            int32_t up = __builtin_ctzll(~m); /* length of the leading run */
            IX ar = 0;
            uint8_t ag = 0;
            if (l < up) {
                ar = hrd[a - 1];
                ag = hgn[a - 1];
            }
            w.sync();
            if (l < up) { /* ancestor l+1 moves to ancestor l (ancestor 0 = position k) */
                int32_t dst = (k >> l) - 1;
                hrd[dst] = ar;
                hsq[dst] = as;
                hgn[dst] = ag;
            }
            int32_t fin = k >> up;
            if (l == 0) {
                hrd[fin - 1] = (IX)rid;
                hsq[fin - 1] = seq;
                hgn[fin - 1] = gen;
            }
            w.sync();
            if (fin == 1) zh->heapTop = seq;
        } else {
            hrd[k - 1] = (IX)rid;
            hsq[k - 1] = seq;
            hgn[k - 1] = gen;
            while (k > 1 && hsq[(k >> 1) - 1] - hsq[k - 1] > 0) {
                heap_swap((k >> 1) - 1, k - 1);
                k >>= 1;
            }
            zh->heapTop = hsq[0];
        }
    }
    /* Heap.get (collections.ts:227-233) + fixdown (249-263). On the GPU, for a heap of at most 256
     * entries, every entry is read in one pass (lane = index mod 64, one register per 64 entries and
     * field), the descent is taken on scalars, and the entries on the path move up one level in one
     * parallel pass whose values come from those registers (lane shuffles): one round trip per pop. */
    MT_HD void heap_pop(int32_t* rid, int32_t* seq, int32_t* gen) {
        MT_PROF_SCOPE(PH_HEAP);
        MT_PROF_COUNT(PH_C_POP, 1);
        int32_t cnt = h.heapN;
        if (W::N == 64 && (HT::H <= 256 || cnt <= 256)) {
            int32_t l = w.lane();
            int32_t c0 = l < cnt ? hsq[l] : 0;
            int32_t c1 = 64 + l < cnt ? hsq[64 + l] : 0;
            int32_t c2 = 128 + l < cnt ? hsq[128 + l] : 0;
            int32_t c3 = 192 + l < cnt ? hsq[192 + l] : 0;
            /* the image's heap (tiled profile): every field in this pass; an LDS heap re-reads the moved entries */
            constexpr bool PICK = TILED && !NARROW;
            int32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, g0 = 0, g1 = 0, g2 = 0, g3 = 0;
            if (PICK) {
                r0 = l < cnt ? (int32_t)hrd[l] : 0, g0 = l < cnt ? hgn[l] : 0;
                r1 = 64 + l < cnt ? (int32_t)hrd[64 + l] : 0, g1 = 64 + l < cnt ? hgn[64 + l] : 0;
                r2 = 128 + l < cnt ? (int32_t)hrd[128 + l] : 0, g2 = 128 + l < cnt ? hgn[128 + l] : 0;
                r3 = 192 + l < cnt ? (int32_t)hrd[192 + l] : 0, g3 = 192 + l < cnt ? hgn[192 + l] : 0;
            }
            int32_t last = cnt - 1; /* index of the entry that moves to the root */
            IX xr = hrd[last];
            uint8_t xg = hgn[last];
            *rid = hrd[0];
            *gen = hgn[0];
            auto L = [&](int32_t i) -> int32_t { /* maxSeq at 1-based position i (i >= 2) */
                int32_t x = i - 1, c = x >> 6;
                int32_t v = c == 0 ? c0 : c == 1 ? c1 : c == 2 ? c2 : c3;
                return w.bcast(v, x & 63);
            };
            *seq = w.bcast(c0, 0);
            int32_t xs = L(cnt >= 2 ? cnt : 2);
            if (cnt < 2) xs = *seq;
            cnt--;
            h.heapN = cnt;
            if (cnt == 0) return;
            /* lane t < d: the t-th entry of the descent (src) moves to its parent (dst), written into lane t as
             * the descent goes (no path array: a dynamically indexed one lives in scratch memory) */
            int32_t d = 0, k = 1;
            int32_t src = 1, dst = 1;
            while ((k << 1) <= cnt) {
                int32_t j = k << 1;
                int32_t sj = L(j);
                if (j < cnt) {
                    int32_t s2 = L(j + 1);
                    if (sj - s2 > 0) {
                        j++;
                        sj = s2;
                    }
                }
                if (xs - sj <= 0) break;
                src = w.writelane(j, d, src);
                dst = w.writelane(k, d, dst);
                d++;
                k = j;
            }
            /* its fields from the registers of the first pass (every lane active: the shuffles read other lanes) */
            int32_t sx = src - 1, sl = sx & 63, sc = sx >> 6;
            auto pick = [&](int32_t v0, int32_t v1, int32_t v2, int32_t v3) -> int32_t {
                int32_t a0 = w.shfl(v0, sl), a1 = w.shfl(v1, sl), a2 = w.shfl(v2, sl), a3 = w.shfl(v3, sl);
                return sc == 0 ? a0 : sc == 1 ? a1 : sc == 2 ? a2 : a3;
            };
            IX mr = 0;
            uint8_t mg = 0;
            int32_t ms = 0;
            if (PICK) {
                mr = (IX)pick(r0, r1, r2, r3);
                mg = (uint8_t)pick(g0, g1, g2, g3);
                ms = pick(c0, c1, c2, c3);
            } else if (l < d) {
                mr = hrd[src - 1];
                mg = hgn[src - 1];
                ms = hsq[src - 1];
            }
            w.sync();
            if (l < d) {
                hrd[dst - 1] = mr;
                hsq[dst - 1] = ms;
                hgn[dst - 1] = mg;
            }
            if (l == 0) {
                hrd[k - 1] = xr;
                hsq[k - 1] = xs;
                hgn[k - 1] = xg;
            }
            w.sync();
            zh->heapTop = d > 0 ? w.bcast(ms, 0) : xs;
        } else if constexpr (W::N == 64) {
            /* Larger heaps: the sift-down looks 5 levels ahead at a time. The 62 nodes of the 5-level
             * subtree below the current node are read in one pass (lane l: depth dd, offset off), the
             * descent through them is taken on scalars (lane broadcasts), then the next subtree; the
             * entries on the path move up one level in one parallel pass, as above. */
            int32_t l = w.lane();
            *rid = hrd[0];
            *gen = hgn[0];
            *seq = hsq[0];
            int32_t last = cnt - 1;
            IX xr = hrd[last];
            uint8_t xg = hgn[last];
            int32_t xs = hsq[last];
            cnt--;
            h.heapN = cnt;
            if (cnt == 0) return;
            int32_t dd = l < 2 ? 1 : l < 6 ? 2 : l < 14 ? 3 : l < 30 ? 4 : l < 62 ? 5 : 0;
            int32_t off = dd ? l - ((1 << dd) - 2) : 0;
            int32_t d = 0, k = 1, lastj = 1;
            int32_t src = 0, dst = 0; /* lane t < d: the t-th entry of the descent and its parent (as above) */
            bool done = false;
            while (!done) {
                int32_t node = dd ? (k << dd) + off : 0;
                int32_t sv = (dd && node <= cnt) ? hsq[node - 1] : 0;
                int32_t cur = 0; /* the current node is (k << t) + cur */
                for (int32_t t = 0; t < 5; t++) {
                    int32_t j = (k << (t + 1)) + 2 * cur; /* its left child (1-based) */
                    if (j > cnt) {
                        done = true;
                        break;
                    }
                    int32_t lj = (1 << (t + 1)) - 2 + 2 * cur; /* the lane holding it */
                    int32_t sj = w.bcast(sv, lj);
                    int32_t c2 = 2 * cur;
                    if (j < cnt) {
                        int32_t s2 = w.bcast(sv, lj + 1);
                        if (sj - s2 > 0) {
                            j++;
                            sj = s2;
                            c2++;
                        }
                    }
                    if (xs - sj <= 0) {
                        done = true;
                        break;
                    }
                    src = w.writelane(j, d, src);
                    dst = w.writelane(lastj, d, dst); /* the root (1) for the first */
                    lastj = j;
                    d++;
                    cur = c2;
                }
                if (!done) k = lastj;
            }
            int32_t fin = d > 0 ? lastj : 1;
            IX mr = 0;
            uint8_t mg = 0;
            int32_t ms = 0;
            if (l < d) {
                mr = hrd[src - 1];
                mg = hgn[src - 1];
                ms = hsq[src - 1];
            }
            w.sync();
            if (l < d) {
                hrd[dst - 1] = mr;
                hsq[dst - 1] = ms;
                hgn[dst - 1] = mg;
            }
            if (l == 0) {
                hrd[fin - 1] = xr;
                hsq[fin - 1] = xs;
                hgn[fin - 1] = xg;
            }
            w.sync();
            zh->heapTop = d > 0 ? w.bcast(ms, 0) : xs;
        } else {
            *rid = hrd[0];
            *seq = hsq[0];
            *gen = hgn[0];
            hrd[0] = hrd[cnt - 1];
            hsq[0] = hsq[cnt - 1];
            hgn[0] = hgn[cnt - 1];
            cnt--;
            h.heapN = cnt;
            int32_t k = 1;
            while ((k << 1) <= cnt) {
                int32_t j = k << 1;
                if (j < cnt && hsq[j - 1] - hsq[j] > 0) j++;
                if (hsq[k - 1] - hsq[j - 1] <= 0) break;
                heap_swap(k - 1, j - 1);
                k = j;
            }
            if (cnt > 0) zh->heapTop = hsq[0];
        }
    }
    /* addToLRUSet (mergeTree.ts:1306-1316) */
    MT_HD void add_lru(int32_t s, int32_t seq) {
        int32_t n = s / MAXN;
        if (nsc[n] != 1 && seq > h.currentSeq) {
            nsc[n] = 1;
            heap_add(z.RID(s), seq);
        }
    }
    /* add_lru of a row whose id, generation and leaf's needsScour the caller has read */
    MT_HD void add_lru_known(int32_t n, int32_t rid, int32_t gen, int32_t sc, int32_t seq) {
        if (sc != 1 && seq > h.currentSeq) {
            nsc[n] = 1;
            heap_add(rid, seq, gen);
        }
    }

    /* ---- properties (segmentPropertiesManager.ts:35-111) ---------------------------- */
    MT_HD int32_t key_slot(uint16_t key) {
        for (int32_t i = 0; i < zh->nkeys; i++)
            if (keys[i] == key) return i;
        if (zh->nkeys >= HT::K) {
            fail(E_CAPACITY); /* the profile's key slots: a larger profile holds more (capacity promotion) */
            return -1;
        }
        keys[zh->nkeys] = key;
        return zh->nkeys++;
    }
#ifndef MT_PROPS_PAR
#define MT_PROPS_PAR 1
#endif
#ifndef MT_ACKANN_PAR
#define MT_ACKANN_PAR 1
#endif
    /* add_props on the GPU: lane k holds key slot k (its key id, the row's value and pending-key count), lane j
     * the op's j-th key / value; everything is read in one pass, the fold runs on those registers in the
     * reference's order (rewrite deletions, then the op's keys in order, new key slots in first-appearance
     * order), and the row's property state is written back in one pass. Same result as the serial form. */
    /* knownFl >= 0: the row's flags as the caller holds them (a row just placed: its cold property state is not read) */
    MT_HD void add_props_par(int32_t s, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t seq, bool collaborating,
                             int32_t knownFl = -1) {
        static_assert(HT::K <= W::N, "a lane per key slot");
        const bool rewrite = comb == MT_COMBINE_REWRITE;
        typename HT::Cold& c = cold(s);
        const int32_t l = w.lane();
        const bool kl = l < HT::K;
        const int32_t kx = kl ? l : 0; /* K is 8 or 24: not a mask */
        uint32_t fl = knownFl >= 0 ? (uint32_t)knownFl : (uint32_t)z.flags(s);
        const bool fresh = !(fl & RF_PROPS);
        /* propertyManager / properties created: every slot absent, no pending counts */
        int32_t prw = 0, pv = 0, pk = 0;
        if (!fresh) {
            prw = c.prw;
            pv = kl ? (int32_t)c.pv[kx] : 0;
            pk = kl ? (int32_t)c.pk[kx] : 0;
        }
        int32_t key = kl ? (int32_t)keys[kx] : -1;
        int32_t nk = zh->nkeys;
        int32_t ok = l < nkv ? (int32_t)kv[l].key : -1, ov = l < nkv ? (int32_t)kv[l].value : 0;
        if (!(prw > 0 && seq != UNASSIGNED_SEQ && collaborating)) {
            if (rewrite) {
                if (collaborating && seq == UNASSIGNED_SEQ) prw++;
                bool inNew = false;
                for (int32_t j = 0; j < nkv; j++) {
                    int32_t vj = w.bcast(ov, j);
                    if (key == w.bcast(ok, j) && vj != 0 && !(vj & MT_VALUE_FALSY)) inNew = true;
                }
                bool modify = seq == UNASSIGNED_SEQ || pk == 0;
                if (l < nk && pv != 0 && !inNew && modify) pv = 0;
            }
            for (int32_t j = 0; j < nkv; j++) {
                int32_t kj = w.bcast(ok, j), vj = w.bcast(ov, j);
                uint64_t m = w.ballot(l < nk && key == kj);
                int32_t k;
                if (m) {
                    k = W::ffs(m);
                } else { /* a new key slot (key_slot) */
                    if (nk >= HT::K) {
                        fail(E_CAPACITY);
                        break;
                    }
                    k = nk++;
                    key = w.writelane(kj, k, key);
                    if (l == 0) keys[k] = (uint16_t)kj;
                }
                int32_t pkk = w.bcast(pk, k);
                if (collaborating) {
                    if (seq == UNASSIGNED_SEQ) {
                        if (pkk == 0xFF) {
                            fail(E_CAPACITY);
                            break;
                        }
                        pk = w.writelane(pkk + 1, k, pk);
                    } else if (pkk != 0 && comb < MT_COMBINE_INCR) {
                        continue;
                    }
                }
                if (comb >= MT_COMBINE_INCR) { /* Properties.combine (combine_value) */
                    vj = combine_value(comb, w.bcast(pv, k), seq);
                    if (vj < 0) break;
                }
                pv = w.writelane(vj, k, pv);
            }
            zh->nkeys = nk;
        }
        int32_t hsum = 0;
        if constexpr (TILED) hsum = w.sum(kl ? prop_mix(kx, pv) : 0); /* TileState::ph */
        w.sync();
        if (kl) {
            c.pv[kx] = (uint16_t)pv;
            c.pk[kx] = (uint8_t)pk;
        }
        if constexpr (TILED) {
            if (l == 0) z.tl.ph[s] = (uint16_t)hsum;
        }
        if (l == 0) c.prw = (uint8_t)prw;
        if (fresh && l == 0) z.flags(s) = (uint8_t)(fl | RF_PROPS);
        w.sync();
    }
    /* Properties.combine (properties.ts:26-59) as addProperties calls it (segmentPropertiesManager.ts:96-97): with
     * newValue still undefined, and no defaultValue / minValue (wire.py and the facade refuse
     * them). "incr": current + undefined — NaN from nothing, NaN, a number or a boolean; the string + "undefined"
     * from a string or a consensus object ("[object Object]undefined"; an interned object or array: refused, its
     * String() has no canonical base). "consensus":
     * a present value unchanged (cv.seq === -1 only for an object a local consensus made, which the engine refuses);
     * over nothing a {value: undefined, seq} object. Returns the key's new value id, or -1 (latched: an incr over a
     * value of undeclared kind, E_UNSUPPORTED; a full table of derived values, E_CAPACITY). */
    MT_HD int32_t combine_value(int32_t comb, int32_t cur, int32_t seq) {
        if (comb == MT_COMBINE_CONSENSUS) return cur != 0 ? cur : dv_intern(1, seq);
        if (cur == 0 || cur == MT_VALUE_NAN) return dv_nan();
        if (cur >= MT_VALUE_CONS0 && cur < MT_VALUE_NAN) return dv_intern(0, 1 << 16); /* "[object Object]undefined" */
        if (cur >= MT_VALUE_STRCAT0 && cur < MT_VALUE_CONS0) {
            int32_t x = z.dvs[cur - MT_VALUE_STRCAT0];
            if ((uint32_t)x >= 0x7FFF0000u) {
                fail(E_CAPACITY);
                return -1;
            }
            return dv_intern(0, x + (1 << 16));
        }
        const int32_t id = cur & ~MT_VALUE_FALSY;
        const int32_t kind = id < nvk ? (int32_t)vk[id] : MT_VKIND_UNKNOWN;
        if (kind == MT_VKIND_NUMERIC) return dv_nan();
        if (kind == MT_VKIND_STRING) return dv_intern(0, cur | (1 << 16));
        fail(E_UNSUPPORTED);
        return -1;
    }
    MT_HD int32_t dv_nan() {
        zh->ndv |= 1 << 16;
        return MT_VALUE_NAN;
    }
    /* the per-document entry holding a derived value (cons = 0: STRCAT x; 1: a consensus object of seq x), added if
     * new; its value id */
    MT_HD int32_t dv_intern(int32_t cons, int32_t x) {
        int32_t nd = zh->ndv;
        const int32_t n = cons ? (nd >> 8) & 0xFF : nd & 0xFF, cap = cons ? 127 : 128;
        int32_t* tab = cons ? z.dvc : z.dvs;
#pragma clang loop unroll(disable)
        for (int32_t i = 0; i < n; i++)
            if (tab[i] == x) return (cons ? MT_VALUE_CONS0 : MT_VALUE_STRCAT0) + i;
        if (n >= cap) {
            fail(E_CAPACITY);
            return -1;
        }
        w.sync();
        if (w.lane() == 0) tab[n] = x;
        w.sync();
        zh->ndv = nd + (cons ? 1 << 8 : 1);
        return (cons ? MT_VALUE_CONS0 : MT_VALUE_STRCAT0) + n;
    }
    /* some key value of 8 slots (4 dwords) is NaN or a consensus object: matchProperties never matches it */
    MT_HD static bool pv_unmatchable(const I4& v) {
        bool u = false;
        for (int q = 0; q < 4; q++) {
            uint32_t x = (uint32_t)v.x[q];
            u |= ((x >> 7) & 0x1FFu) == 0xFFu || ((x >> 23) & 0x1FFu) == 0xFFu;
        }
        return u;
    }
    /* one key slot's term of the property hash (0 for an absent value): the hash is the sum of the terms */
    MT_HD static int32_t prop_mix(int32_t k, int32_t v) {
        return v ? (int32_t)(((uint32_t)v * 0x9E3779B1u + (uint32_t)k * 0x85EBCA77u) >> 16) : 0;
    }
    MT_HD void prop_rehash(int32_t s) {
        if constexpr (TILED) {
            const typename HT::Cold& c = cold(s);
            int32_t hsum = 0;
            for (int32_t k = 0; k < HT::K; k++) hsum += prop_mix(k, c.pv[k]);
            z.tl.ph[s] = (uint16_t)hsum;
        }
    }
    MT_HD void add_props(int32_t s, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t seq, bool collaborating,
                         int32_t knownFl = -1) {
        if constexpr (W::N >= 32 && MT_PROPS_PAR) {
            if (nkv <= W::N) {
                add_props_par(s, kv, nkv, comb, seq, collaborating, knownFl);
                return;
            }
        }
        add_props_serial(s, kv, nkv, comb, seq, collaborating);
        prop_rehash(s);
    }
    MT_HD void add_props_serial(int32_t s, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t seq, bool collaborating) {
        const bool rewrite = comb == MT_COMBINE_REWRITE;
        typename HT::Cold& c = cold(s); /* the row id is read once, not after every store */
        if (!(z.flags(s) & RF_PROPS)) {
            c.prw = 0;
            z.flags(s) |= RF_PROPS;
            clear_props(s);
        }
        if (c.prw > 0 && seq != UNASSIGNED_SEQ && collaborating) return;
        if (rewrite) {
            if (collaborating && seq == UNASSIGNED_SEQ) c.prw++;
            for (int32_t k = 0; k < zh->nkeys; k++) {
                if (c.pv[k] == 0) continue;
                bool inNew = false;
                for (int32_t j = 0; j < nkv; j++)
                    if (kv[j].key == keys[k] && kv[j].value != 0 && !(kv[j].value & MT_VALUE_FALSY)) inNew = true;
                bool modify = seq == UNASSIGNED_SEQ || c.pk[k] == 0;
                if (!inNew && modify) c.pv[k] = 0;
            }
        }
        for (int32_t j = 0; j < nkv; j++) {
            int32_t k = key_slot(kv[j].key);
            if (k < 0) return;
            if (collaborating) {
                if (seq == UNASSIGNED_SEQ) {
                    if (c.pk[k] == 0xFF) {
                        fail(E_CAPACITY);
                        return;
                    }
                    c.pk[k]++;
                } else if (!(c.pk[k] == 0) && comb < MT_COMBINE_INCR) {
                    continue;
                }
            }
            if (comb >= MT_COMBINE_INCR) { /* Properties.combine (combine_value) */
                int32_t v = combine_value(comb, c.pv[k], seq);
                if (v < 0) return;
                c.pv[k] = (uint16_t)v;
                continue;
            }
            c.pv[k] = kv[j].value;
        }
    }
    /* ackPendingProperties (segmentPropertiesManager.ts:19-33) */
    MT_HD void ack_props(int32_t s, const mt_kv* kv, int32_t nkv, bool rewrite) {
        typename HT::Cold& c = cold(s);
        if (rewrite) c.prw--;
        for (int32_t j = 0; j < nkv; j++) {
            int32_t k = key_slot(kv[j].key);
            if (k < 0) return;
            if (c.pk[k]) c.pk[k]--;
        }
    }
    /* property values and pending-key counters of row s to "absent" (16 / 8 bytes per store) */
    MT_HD void clear_props(int32_t s) {
        typename HT::Cold& c = cold(s);
        I4 zero = {{0, 0, 0, 0}};
        for (int i = 0; i < HT::K / 8; i++) st4(&c.pv[8 * i], zero);
        if constexpr (TILED) z.tl.ph[s] = 0;
        for (int i = 0; i < HT::K / 8; i++) {
            uint64_t z8 = 0;
            __builtin_memcpy(__builtin_assume_aligned(&c.pk[8 * i], 8), &z8, 8);
        }
    }
    MT_HD bool match_props(int32_t a, int32_t b) { /* matchProperties (properties.ts:61-92) */
        MT_PROF_SCOPE(PH_CAND);
        bool pa = z.flags(a) & RF_PROPS, pb = z.flags(b) & RF_PROPS;
        if (pa != pb) return false;
        if (!pa) return true;
        const typename HT::Cold& ca = cold(a);
        const typename HT::Cold& cb = cold(b);
        const bool um = ((zh->ndv >> 8) & 0x1FF) != 0; /* NaN or consensus objects exist: never matched (pv_unmatchable) */
        for (int i = 0; i < HT::K / 8; i++) { /* 8 key slots per 16-byte compare */
            I4 va = ld4((const int32_t*)&ca.pv[8 * i]);
            if (!eq4(va, ld4((const int32_t*)&cb.pv[8 * i])) || (um && pv_unmatchable(va))) return false;
        }
        return true;
    }

    /* ---- zamboni: scourNode / pack / zamboniSegments (mergeTree.ts:1322-1511) ---------- */
    /* a SubSequence document (DV_RUN): read from the image header, only where a length test needs it */
    MT_HD bool run_doc() const { return (zh->ndv & DV_RUN) != 0; }
    /* the length half of canAppend for rows of lengths La, Lb: TextSegment's granularity (textSegment.ts:66-67,
     * TextSegmentGranularity 256), or in a SubSequence document MaxRun (sequence sharedSequence.ts:12, 57-60) */
    MT_HD bool gran_ok(int32_t La, int32_t Lb) const {
        const int32_t m = La < Lb ? La : Lb;
        return m <= MT_RUN_MAXRUN || (m <= GRANULARITY && !run_doc());
    }
    /* canAppend (textSegment.ts:63-68; SubSequence: sharedSequence.ts:57-60, no newline rule) */
    MT_HD bool can_append(int32_t a, int32_t b) {
        MT_PROF_SCOPE(PH_CAND);
        /* PermutationSegment.canAppend (permutationvector.ts:87-93): both unallocated, or b's handles follow a's */
        if ((z.flags(a) | z.flags(b)) & RF_PERM)
            return (z.flags(a) & z.flags(b) & RF_PERM) != 0 && perm_follows(a, b, z.len(a));
        if (z.flags(a) & RF_MARKER) return false;
        if (ends_nl(a, z.len(a))) return false;
        if (z.flags(b) & RF_MARKER) return false;
        return gran_ok(z.len(a), z.len(b));
    }
    /* PermutationSegment.canAppend's handle rule for rows a (current length La) and b */
    MT_HD bool perm_follows(int32_t a, int32_t b, int32_t La) {
        uint32_t sa = cold(a).toff, sb = cold(b).toff;
        return sa == 0 ? sb == 0 : sb == sa + (uint32_t)La;
    }
    /* the text of the row in slot a (current length La) ends with "\n" (textSegment.ts:64) */
    MT_HD bool ends_nl(int32_t a, int32_t La) {
        int32_t f = z.flags(a);
        if (f & RF_NLK) return (f & RF_NL) != 0;
        MT_PROF_SCOPE(PH_CAND);
        bool nl = La > 0 && !run_doc() && arena_base(zh->arenaSide)[cold(a).toff + La - 1] == '\n';
        z.flags(a) = (uint8_t)(f | RF_NLK | (nl ? RF_NL : 0));
        return nl;
    }
    /* TextSegment.append (textSegment.ts:74-85): the merged text is rebuilt at the arena top */
    MT_HD void append_text(int32_t a, int32_t b) {
        uint32_t xa = 0, xb = 0;
        if constexpr (TILED) {
            xa = z.tl.xf[a];
            xb = z.tl.xf[b];
        }
        append_rows(a, b, z.RID(a), z.RID(b), z.len(a), z.len(b), z.flags(a), z.flags(b), xa, xb);
    }
    /* append_text with the two rows' ids, lengths, flags and window flags as the caller read them (scour) */
    MT_HD void append_stat(int32_t a, int32_t Lb, uint32_t xa, uint32_t xb) {
        if constexpr (TILED) { /* b's length joins a's row: keep the leaf's STABLE sum exact */
            bool sa = xa & XF_STABLE, sb = xb & XF_STABLE;
            if (sa && !sb) lst_add(a / MAXN, Lb);
            if (!sa && sb) lst_add(a / MAXN, -Lb);
        }
    }
    MT_HD void append_rows(int32_t a, int32_t b, int32_t ra, int32_t rb, int32_t La, int32_t Lb, uint32_t fa,
                           uint32_t fb, uint32_t xa, uint32_t xb) {
        MT_PROF_SCOPE(PH_APPEND);
        append_stat(a, Lb, xa, xb);
        if (fa & RF_PERM) { /* PermutationSegment.append (permutationvector.ts:95-101) */
            z.len(a) = La + Lb;
            return;
        }
        typename HT::Cold* cd = d.cold();
        uint16_t* base = arena_base(zh->arenaSide);
        int32_t ta = (int32_t)cd[ra].toff, tb = (int32_t)cd[rb].toff; /* both reads in one round trip */
        if (ta + La == h.arenaTop && h.arenaTop + Lb <= d.caps.acap) {
            int32_t off = arena_alloc(Lb);
            arena_copy(base + off, base + tb, Lb);
        } else if (ta + La == tb) {
            /* already contiguous */
        } else {
            int32_t off = arena_alloc(La + Lb);
            if (off < 0) return;
            base = arena_base(zh->arenaSide); /* a GC may have switched halves (and moved both texts) */
            arena_copy(base + off, base + cd[ra].toff, La);
            arena_copy(base + off + La, base + cd[rb].toff, Lb);
            cd[ra].toff = (uint32_t)off;
        }
        z.len(a) = La + Lb;
        /* the merged text ends where b's did */
        z.flags(a) = (uint8_t)((fa & ~(uint32_t)(RF_NLK | RF_NL)) | (fb & (RF_NLK | RF_NL)));
    }
#ifndef MT_APPEND_BATCH
#define MT_APPEND_BATCH 1 /* scour's text appends planned on scalars during the walk, their copies made together after it */
#endif
    /* copy jobs of scour's append walk: lane j < nj holds job j (destination, source, units in the current arena
     * half); all of them in one wave-parallel copy, a lane per unit, every load of a block before its stores (the
     * sources are texts from before the walk, the destinations fresh space above them) */
    MT_HD void copy_jobs(int32_t jd, int32_t js, int32_t jn, int32_t nj) {
        uint16_t* base = arena_base(zh->arenaSide);
        int32_t tot;
        int32_t pre = w.excl_scan(w.lane() < nj ? jn : 0, &tot);
        for (int32_t b = 0; b < tot; b += W::N) {
            int32_t i = b + w.lane();
            int32_t jj = 0;
            for (int32_t t = 1; t < nj; t++)
                if (w.bcast(pre, t) <= i) jj = t;
            int32_t o = i - w.shfl(pre, jj);
            int32_t src = w.shfl(js, jj), dst = w.shfl(jd, jj);
            uint16_t v = i < tot ? base[src + o] : 0;
            w.sync();
            if (i < tot) base[dst + o] = v;
        }
        w.sync();
    }
    /* scourNode on leaf n: compacts the slab in place; returns the new child count. Rows are
     * merged into their predecessor or unlinked exactly as the reference decides. */
    MT_HD int32_t scour_leaf(int32_t n) {
        MT_PROF_SCOPE(PH_SCOUR);
        int32_t c = nch[n];
        int32_t wpos = 0;
        int32_t prev = -1; /* slot of prevSegment in the compacted slab */
        int32_t minSeq = h.minSeq;
        for (int32_t k = 0; k < c; k++) {
            int32_t s = n * MAXN + k;
            if (z.ng(s) == 0) {
                if (z.rseq(s) != NOREM) {
                    if (z.rseq(s) > minSeq) {
                        if (wpos != k) copy_row(n * MAXN + wpos, s);
                        wpos++;
                    } else {
                        if (dl_on()) { /* MergeTreeMaintenanceType.UNLINK (mergeTree.ts:1343-1348) */
                            dhead(MT_DELTA_UNLINK);
                            dseg(-1, z.len(s));
                            dtail(1);
                        }
                        if (ht_on() && (z.flags(s) & RF_PERM)) ht_unlinked(z.RID(s), z.len(s));
                        if (refs_on()) { /* the segment loses its parent: its references detach */
                            refs_move(z.RID(s), INT32_MIN, REF_DETACHED, 0);
                            coll_drop(z.RID(s));
                        }
                        free_rid(z.RID(s)); /* unlinked */
                    }
                    prev = -1;
                } else {
                    if (z.seq(s) <= minSeq) {
                        /* hot predicates first; the cold ones (props values, trailing newline) are
                         * only read for a candidate pair. Same conjunction as mergeTree.ts:1355-1360. */
                        bool ok = prev >= 0 && local_len(s) > 0 &&
                                  ((z.flags(prev) & z.flags(s) & RF_PERM) ||
                                   (!((z.flags(prev) | z.flags(s)) & RF_NOTEXT) && gran_ok(z.len(prev), z.len(s)))) &&
                                  ((z.flags(prev) ^ z.flags(s)) & RF_PROPS) == 0 && match_props(prev, s) &&
                                  can_append(prev, s);
                        if (ok) {
                            if (refs_on()) refs_append(z.RID(prev), z.RID(s), z.len(prev));
                            append_text(prev, s);
                            if (dl_on()) { /* APPEND (mergeTree.ts:1368-1373): [prevSegment, segment] */
                                dhead(MT_DELTA_APPEND);
                                dseg(-1, z.len(prev));
                                dseg(-1, z.len(s));
                                dtail(2);
                            }
                            free_rid(z.RID(s));
                        } else {
                            int32_t dst = n * MAXN + wpos;
                            if (wpos != k) copy_row(dst, s);
                            wpos++;
                            prev = local_len(dst) > 0 ? dst : -1;
                        }
                    } else {
                        if (wpos != k) copy_row(n * MAXN + wpos, s);
                        wpos++;
                        prev = -1;
                    }
                }
            } else {
                if (wpos != k) copy_row(n * MAXN + wpos, s);
                wpos++;
                prev = -1;
            }
        }
        h.nrows -= c - wpos;
        nch[n] = (int8_t)wpos;
        if (wpos < c) clear_slots(n * MAXN + wpos, c - wpos);
        return wpos;
    }

    /* scourNode (mergeTree.ts:1322-1398), wave-parallel form, over nl <= 8 leaves at once: lane q
     * holds child q & 7 of leaf q >> 3. Every row's hot fields are loaded in one pass; the keep /
     * unlink / append decisions are the reference's sequential walk, taken on scalar copies of those
     * fields (v_readlane), with cold data (props values, the trailing character) read only for a
     * candidate pair; the frees and the slab compaction are again one parallel pass. cnt[i] gets the
     * new child count of leaf i. Same result as scour_leaf on each leaf in turn. */
    /* pre (one leaf): lanes < 8 hold its rows and preC its child count, read by the caller */
    MT_HD void scour_par(const int32_t* leaves, int32_t nl, int32_t* cnt, const HotRow* pre = nullptr,
                         int32_t preC = 0) {
        MT_PROF_SCOPE(PH_SCOUR);
#if defined(MT_PROF) && defined(__HIP_DEVICE_COMPILE__)
        uint64_t _t0 = __builtin_amdgcn_s_memtime();
#endif
        int32_t q = w.lane();
        int32_t li = q >> 3, j = q & (MAXN - 1);
        int32_t n = -1;
        for (int32_t i = 0; i < MAXN; i++)
            if (i == li && i < nl) n = leaves[i];
        int32_t c = n >= 0 ? (pre ? preC : nch[n]) : 0;
        bool valid = j < c;
        HotRow r = {};
        if (valid) r = pre ? *pre : load_row(n * MAXN + j);
        int32_t minSeq = h.minSeq;
        /* 0: no row; 1: held, resets prevSegment; 2: unlinked, resets prevSegment; 3: merge candidate */
        int32_t code = 0;
        if (valid) {
            if (r.ng)
                code = 1;
            else if (r.rseq != NOREM)
                code = r.rseq > minSeq ? 1 : 2;
            else
                code = r.seq > minSeq ? 1 : 3;
        }
        int32_t nlen = r.len;
        uint64_t vmask = w.ballot(valid);
#if defined(MT_PROF) && defined(__HIP_DEVICE_COMPILE__)
        uint64_t _t1 = __builtin_amdgcn_s_memtime();
        if (prof) prof[PH_S1] += _t1 - _t0;
#endif
        /* Only a candidate whose predecessor in the same leaf is a candidate can be appended; every
         * other row is decided by its own code: held rows (1) are kept, unlinked rows (2) are
         * dropped, and a candidate after a non-candidate starts a run as prevSegment (kept). */
        uint64_t cand = w.ballot(code == 3);
        uint64_t pairs = cand & (cand << 1) & ~0x0101010101010101ull;
        uint64_t keep = w.ballot(code == 1) | (cand & ~pairs);
        int32_t fl = r.flags;
        /* Every test of an append that does not depend on the run's length, for all pairs at once (their cold
         * reads overlap): a run's head has the properties, type, handle chain and last text unit of the run's
         * last row (appends require equal properties, keep the head's start, and end with the appended
         * text), so "head + row k" is decided by rows k-1 and k. Lane k: the pair (k-1, k). */
        bool pairOk = false;
        int32_t tofP = 0, tofK = 0; /* a pair's text offsets (its left and right row), read with its tests */
        /* the shuffles read the predecessor lane, which may not be a pair's lane: outside the branch, where
         * every lane is active */
        int32_t lenP = w.shfl(r.len, q - 1), flP = w.shfl(fl, q - 1);
        int32_t ridP = w.shfl((int32_t)r.rid, q - 1); /* the pair's cold rows by the ids this pass read */
        int32_t phP = TILED ? w.shfl((int32_t)r.ph, q - 1) : 0;
        if ((pairs >> q) & 1) {
            bool permPair = (flP & fl & RF_PERM) != 0;
            /* localNetLength > 0 on both sides: a zero-length row (the empty right part of a split past a
             * segment's end) is held and leaves no prevSegment (mergeTree.ts:1355-1383) */
            pairOk = lenP > 0 && r.len > 0 && ((flP ^ fl) & RF_PROPS) == 0 &&
                     (permPair || !((flP | fl) & RF_NOTEXT));
            /* tiled: property hashes that differ decide matchProperties without the cold values */
            if (TILED && (fl & RF_PROPS) && phP != (int32_t)r.ph) pairOk = false;
        }
        if (pairOk) {
            const bool permPair = (flP & fl & RF_PERM) != 0;
            const typename HT::Cold& ca = d.COLD(ridP);
            const typename HT::Cold& cb = d.COLD((int32_t)r.rid);
            tofP = (int32_t)ca.toff;
            tofK = (int32_t)cb.toff;
            if (pairOk && (fl & RF_PROPS)) { /* matchProperties (properties.ts:61-92) */
                for (int i = 0; i < HT::K / 8; i++)
                    if (!eq4(ld4((const int32_t*)&ca.pv[8 * i]), ld4((const int32_t*)&cb.pv[8 * i]))) pairOk = false;
                if (pairOk && ((zh->ndv >> 8) & 0x1FF)) /* NaN and consensus objects never match (pv_unmatchable) */
                    for (int i = 0; i < HT::K / 8; i++)
                        if (pv_unmatchable(ld4((const int32_t*)&ca.pv[8 * i]))) pairOk = false;
            }
            if (pairOk && permPair) { /* PermutationSegment.canAppend: handles follow, or both unallocated */
                uint32_t sa = (uint32_t)tofP, sb = (uint32_t)tofK;
                pairOk = sa == 0 ? sb == 0 : sb == sa + (uint32_t)lenP;
            } else if (pairOk) { /* TextSegment.canAppend: the run does not end with "\n" (textSegment.ts:64) */
                bool nl = (flP & RF_NLK) ? (flP & RF_NL) != 0
                                         : !run_doc() && arena_base(zh->arenaSide)[tofP + lenP - 1] == '\n';
                pairOk = !nl;
            }
        }
        uint64_t okm = w.ballot(pairOk);
        int32_t prev = -1, prevLen = 0, prevFl = 0;
        int32_t alen = 0; /* an appended row's lane: its prevSegment's length right after the append */
        /* Only a pair that passed the tests above can append; every other pair is kept. The walk visits those
         * pairs in order: a pair whose left row was not appended starts from that row as prevSegment (it
         * opened a run, or was kept; either way it has absorbed nothing yet), otherwise the run goes on. */
        keep |= pairs & ~okm;
        uint64_t app = 0; /* rows appended so far */
        uint64_t m = pairs & okm;
#if MT_APPEND_BATCH
        /* TextSegment.append's arena work planned on the run head's text offset (prevT): copy jobs (lane j: job j)
         * and the heads whose text moved (lane: the new offset), applied after the walk; the same arena decisions
         * as append_rows. A walk that needs a GC applies what it planned and goes on through append_rows. */
        int32_t jd = 0, js = 0, jn = 0, nj = 0, ntof = 0, prevT = 0;
        uint64_t moved = 0;
        bool serial = false;
#endif
        while (m) {
            int32_t k = W::ffs(m);
            m &= m - 1;
            if (!((app >> (k - 1)) & 1)) {
                prev = k - 1;
                prevLen = w.bcast(r.len, prev);
                prevFl = w.bcast(fl, prev);
#if MT_APPEND_BATCH
                prevT = w.bcast(tofP, k);
#endif
            }
            int32_t lk = w.bcast(r.len, k);
            int32_t fk = w.bcast(fl, k);
            bool ok = true;
            /* the serial part: a text append needs either side <= TextSegment granularity (the run grows) */
            if (!(prevFl & fk & RF_PERM)) ok = gran_ok(prevLen, lk);
            if (ok) {
                int32_t sp = w.bcast(n, prev) * MAXN + (prev & (MAXN - 1));
                int32_t sk = w.bcast(n, k) * MAXN + (k & (MAXN - 1));
                int32_t rp = w.bcast((int32_t)r.rid, prev), rk = w.bcast((int32_t)r.rid, k);
                if (refs_on()) refs_append(rp, rk, prevLen);
                uint32_t xp = TILED ? (uint32_t)w.bcast((int32_t)r.xf, prev) : 0u, xk = TILED ? (uint32_t)w.bcast((int32_t)r.xf, k) : 0u;
#if MT_APPEND_BATCH
                if (!serial && (prevFl & RF_PERM)) {
                    append_stat(sp, lk, xp, xk); /* PermutationSegment.append: the length, written by the compaction */
                } else if (!serial) {
                    MT_PROF_SCOPE(PH_APPEND);
                    append_stat(sp, lk, xp, xk);
                    int32_t tb = w.bcast(tofK, k), top = h.arenaTop, cap = d.caps.acap;
                    if (prevT + prevLen == top && top + lk <= cap) { /* the head's text ends at the top: extend it */
                        jd = w.writelane(top, nj, jd);
                        js = w.writelane(tb, nj, js);
                        jn = w.writelane(lk, nj, jn);
                        nj++;
                        h.arenaTop = top + lk;
                    } else if (prevT + prevLen == tb) { /* already contiguous */
                    } else if (top + prevLen + lk <= cap) { /* both texts to the top */
                        jd = w.writelane(top, nj, jd);
                        js = w.writelane(prevT, nj, js);
                        jn = w.writelane(prevLen, nj, jn);
                        jd = w.writelane(top + prevLen, nj + 1, jd);
                        js = w.writelane(tb, nj + 1, js);
                        jn = w.writelane(lk, nj + 1, jn);
                        nj += 2;
                        prevT = top;
                        ntof = w.writelane(top, prev, ntof);
                        moved |= 1ull << prev;
                        h.arenaTop = top + prevLen + lk;
                    } else { /* a GC: the copies, the heads' lengths and moved offsets land first (it reads them) */
                        copy_jobs(jd, js, jn, nj);
                        nj = 0;
                        if (valid && nlen != r.len) z.len(n * MAXN + j) = nlen;
                        if ((moved >> q) & 1) d.COLD(r.rid).toff = (uint32_t)ntof;
                        moved = 0;
                        w.sync();
                        serial = true;
                        append_rows(sp, sk, rp, rk, prevLen, lk, (uint32_t)prevFl, (uint32_t)fk, 0u, 0u);
                    }
                    if (nj > W::N - 2) { /* room for the next append's two jobs */
                        copy_jobs(jd, js, jn, nj);
                        nj = 0;
                    }
                } else
#endif
                /* updates z.len(sp) (read by a GC inside it) and its NL bits */
                append_rows(sp, sk, rp, rk, prevLen, lk, (uint32_t)prevFl, (uint32_t)fk, xp, xk);
                prevLen += lk;
                prevFl = (prevFl & ~(RF_NLK | RF_NL)) | (fk & (RF_NLK | RF_NL));
                nlen = w.writelane(prevLen, prev, nlen);
                alen = w.writelane(prevLen, k, alen);
                fl = w.writelane(prevFl, prev, fl);
                app |= 1ull << k;
            } else {
                keep |= 1ull << k; /* kept: the next pair, if it tests ok, starts from this row */
            }
        }
#if MT_APPEND_BATCH
        if (nj) copy_jobs(jd, js, jn, nj);
        if ((moved >> q) & 1) d.COLD(r.rid).toff = (uint32_t)ntof;
#endif
#if defined(MT_PROF) && defined(__HIP_DEVICE_COMPILE__)
        uint64_t _t2 = __builtin_amdgcn_s_memtime();
        if (prof) prof[PH_S2] += _t2 - _t1;
#endif
        /* frees: every valid row not kept (unlinked or appended) */
        uint64_t drop = vmask & ~keep;
        if (refs_on()) { /* references on unlinked rows detach (their segment loses its parent) */
            uint64_t um = drop & w.ballot(code == 2);
            while (um) {
                int32_t l = W::ffs(um);
                um &= um - 1;
                int32_t ur = w.bcast((int32_t)r.rid, l);
                refs_move(ur, INT32_MIN, REF_DETACHED, 0);
                coll_drop(ur);
            }
        }
        if (dl_on() || ht_on()) { /* UNLINK / APPEND maintenance events in the reference's walk order (lane order) */
            uint64_t em = drop;
            const bool dlo = dl_on();
            while (em) {
                int32_t l = W::ffs(em);
                em &= em - 1;
                int32_t ln = w.bcast(r.len, l);
                if (w.bcast(code, l) == 2) {
                    if (dlo) {
                        dhead(MT_DELTA_UNLINK);
                        dseg(-1, ln);
                        dtail(1);
                    }
                    if (ht_on() && (w.bcast((int32_t)fl, l) & RF_PERM)) ht_unlinked(w.bcast((int32_t)r.rid, l), ln);
                } else if (!dlo) {
                } else {
                    dhead(MT_DELTA_APPEND);
                    dseg(-1, w.bcast(alen, l));
                    dseg(-1, ln);
                    dtail(2);
                }
            }
        }
        /* nothing dropped: nothing appended either (an appended row is dropped), so every row keeps its slot, length
         * and flags and the leaves their child counts; no writes */
        if (drop) {
            uint64_t below = q ? (~0ull >> (64 - q)) : 0ull;
            if ((drop >> q) & 1) {
                int32_t pos = zh->nfreeRid + __builtin_popcountll(drop & below);
                z.RGEN(r.rid)++;
                d.FRID(pos) = (IX)r.rid;
            }
            int32_t ndrop = __builtin_popcountll(drop);
            zh->nfreeRid += ndrop;
            h.nrows -= ndrop;
            /* compaction: kept rows move down within their leaf; vacated slots get length 0 */
            uint64_t lmask = n >= 0 ? (0xFFull << (8 * li)) : 0ull;
            int32_t newc = __builtin_popcountll(keep & lmask);
            w.sync();
            if ((keep >> q) & 1) {
                r.len = nlen;
                r.flags = (uint8_t)fl;
                store_row(n * MAXN + __builtin_popcountll(keep & lmask & below), r);
            }
            if (valid && j >= newc) z.len(n * MAXN + j) = 0; /* disjoint from every kept row's target */
            if (n >= 0 && j == 0) nch[n] = (int8_t)newc;
            w.sync();
        }
#pragma unroll
        for (int32_t i = 0; i < MAXN; i++) /* constant indices: the caller's array stays in registers */
            if (i < nl) cnt[i] = __builtin_popcountll(keep & (0xFFull << (8 * i)));
#if defined(MT_PROF) && defined(__HIP_DEVICE_COMPILE__)
        if (prof) prof[PH_S3] += __builtin_amdgcn_s_memtime() - _t2;
#endif
    }
    /* scourNode of one leaf: the parallel form on the GPU, the serial walk on the host */
    MT_HD int32_t scour_one(int32_t n) {
        if constexpr (W::N >= MAXN * MAXN) {
            int32_t cnt[1];
            scour_par(&n, 1, cnt);
            return cnt[0];
        } else {
            return scour_leaf(n);
        }
    }
    /* pack's leaf level on the GPU (mergeTree.ts:1401-1446): scour the pc sibling leaves under `parent`, then
     * redistribute their rows over cc = total / 4 leaves (the old node ids first, in order). The per-leaf values
     * are lane arrays (lane i: leaf i's node id / row count / first row), read by lane broadcasts: no locally
     * indexed array, which the compiler would keep in scratch memory. Same result as the serial form in pack(). */
    MT_HD bool pack_leaves(int32_t parent, int32_t pc) { /* false: out of nodes (pack stops, as the serial form) */
        const int32_t q = w.lane();
        {
            int32_t sib[MAXN], cnt[MAXN];
#pragma unroll
            for (int32_t i = 0; i < MAXN; i++) sib[i] = i < pc ? z.KIDS(parent * MAXN + i) : -1;
            scour_par(sib, pc, cnt);
        }
        MT_PROF_SCOPE(PH_P1);
        int32_t okv = q < pc ? (int32_t)z.KIDS(parent * MAXN + (q & (MAXN - 1))) : 0; /* lane i: old leaf i */
        int32_t ocv = q < pc ? (int32_t)nch[okv] : 0;                                 /* its rows after scour */
        int32_t total;
        int32_t oex = w.excl_scan(ocv, &total); /* lane i: leaf i's first row in the run of all rows */
        int32_t cc = total / (MAXN / 2);
        if (cc > MAXN - 1) cc = MAXN - 1;
        if (cc < 1) cc = 1;
        int32_t base = total / cc, extra = total % cc;
        int32_t firstPos = TILED ? 0 : (int32_t)lp[w.bcast(okv, 0)];
        /* new leaf ni: the old node id ni < pc, else a new node; ncv its row count, nex its first row */
        int32_t nkv = q < pc ? okv : 0;
        for (int32_t ni = pc; ni < cc; ni++) {
            int32_t nb = alloc_node(0);
            if (nb < 0) return false;
            nkv = w.writelane(nb, ni, nkv);
        }
        int32_t ncv = q < cc ? base + (q < extra ? 1 : 0) : 0;
        int32_t ntot;
        int32_t nex = w.excl_scan(ncv, &ntot);
        /* move the held rows (<= 49) from old positions to new ones: read all, then write */
        bool has = q < total;
        int32_t src = 0, dst = 0;
#pragma unroll
        for (int32_t t = 0; t < MAXN; t++) {
            int32_t os = w.bcast(oex, t), oc = w.bcast(ocv, t), ok = w.bcast(okv, t);
            if (t < pc && q >= os && q < os + oc) src = ok * MAXN + (q - os);
            int32_t ns = w.bcast(nex, t), nc = w.bcast(ncv, t), nk = w.bcast(nkv, t);
            if (t < cc && q >= ns && q < ns + nc) dst = nk * MAXN + (q - ns);
        }
        HotRow r;
        if (has) r = load_row(src);
        w.sync();
        if (has) {
            store_row(dst, r);
            z.RLEAF(r.rid) = (IX)(dst / MAXN);
        }
        w.sync();
        if (q < cc) { /* the new leaves' headers, a lane each */
            nch[nkv] = (int8_t)ncv;
            npar[nkv] = (IX)parent;
            nlev[nkv] = 0;
            nsc[nkv] = -1;
        }
        w.sync();
        for (int32_t ni = 0; ni < cc; ni++) {
            int32_t nc = w.bcast(ncv, ni);
            if (nc < MAXN) clear_slots(w.bcast(nkv, ni) * MAXN + nc, MAXN - nc);
        }
        int32_t nl = h.nleaf;
        int32_t delta = cc - pc;
        if constexpr (TILED) { /* the rope: extra leaves after the kept ones, surplus ones out */
            for (int32_t i = pc; i < cc; i++) rope_insert_after(w.bcast(nkv, i - 1), w.bcast(nkv, i));
            for (int32_t i = cc; i < pc; i++) rope_remove(w.bcast(okv, i));
            int32_t nk[MAXN];
#pragma unroll
            for (int32_t i = 0; i < MAXN; i++) nk[i] = w.bcast(nkv, i);
            leaves_restat(nk, cc);
        }
        for (int32_t i = cc; i < pc; i++) free_node(w.bcast(okv, i));
        if constexpr (!TILED) {
            /* lorder: [firstPos, firstPos+pc) becomes [firstPos, firstPos+cc) */
            lorder_shift(firstPos + pc, nl, delta);
            if (q >= pc && q < cc) {
                lo[firstPos + q] = (IX)nkv;
                lp[nkv] = (IX)(firstPos + q);
            }
            w.sync();
        }
        h.nleaf = nl + delta;
        if (delta > 0) note_leaves();
        if (q < cc) z.KIDS(parent * MAXN + q) = (IX)nkv;
        w.sync();
        nch[parent] = (int8_t)cc;
        return true;
    }
    /* pack (mergeTree.ts:1401-1453) of `block`'s parent */
    MT_HD void pack(int32_t block0) {
        MT_PROF_SCOPE(PH_PACK);
      int32_t block = block0;
      for (;;) { /* iterative: pack recurses upward while the parent underflows (1447-1452) */
        int32_t parent = npar[block];
        int32_t pc = nch[parent];
        int8_t lvl = nlev[block];
        if (lvl == 0) {
          if constexpr (W::N >= MAXN * MAXN) {
            if (!pack_leaves(parent, pc)) return;
          } else {
            /* scour every sibling leaf, then redistribute their rows over new leaves */
            int32_t total = 0;
            if constexpr (W::N >= MAXN * MAXN) {
                int32_t sib[MAXN], cnt[MAXN];
                for (int32_t i = 0; i < MAXN; i++) sib[i] = i < pc ? z.KIDS(parent * MAXN + i) : -1;
                scour_par(sib, pc, cnt);
                for (int32_t i = 0; i < pc; i++) total += cnt[i];
            } else {
                for (int32_t i = 0; i < pc; i++) total += scour_leaf(z.KIDS(parent * MAXN + i));
            }
            MT_PROF_SCOPE(PH_P1);
            int32_t cc = total / (MAXN / 2);
            if (cc > MAXN - 1) cc = MAXN - 1;
            if (cc < 1) cc = 1;
            int32_t base = total / cc, extra = total % cc;
            /* Packed blocks reuse the old leaf node ids in order (ids are not observable), so
             * pack never needs more nodes than it had; they are new blocks for needsScour. */
            int32_t oldk[MAXN];
            int32_t ocnt[MAXN];
            for (int32_t i = 0; i < pc; i++) {
                oldk[i] = z.KIDS(parent * MAXN + i);
                ocnt[i] = nch[oldk[i]];
            }
            int32_t firstPos = TILED ? 0 : lp[oldk[0]];
            int32_t newk[MAXN];
            int32_t ncnt[MAXN];
            for (int32_t ni = 0; ni < cc; ni++) {
                ncnt[ni] = base + (ni < extra ? 1 : 0);
                newk[ni] = ni < pc ? oldk[ni] : alloc_node(0);
                if (newk[ni] < 0) return;
            }
            /* move the held rows (<= 49) from old positions to new ones: read all, then write */
            if (W::N >= MAXN * MAXN) {
                int32_t q = w.lane();
                bool has = q < total;
                HotRow r;
                int32_t dst = 0;
                if (has) {
                    int32_t i = 0, acc = 0;
                    while (q >= acc + ocnt[i]) acc += ocnt[i++];
                    r = load_row(oldk[i] * MAXN + (q - acc));
                    int32_t ti = 0, tacc = 0;
                    while (q >= tacc + ncnt[ti]) tacc += ncnt[ti++];
                    dst = newk[ti] * MAXN + (q - tacc);
                }
                w.sync();
                if (has) {
                    store_row(dst, r);
                    z.RLEAF(r.rid) = (IX)(dst / MAXN);
                }
                w.sync();
            } else {
                HotRow tmp[MAXN * MAXN];
                int32_t q = 0;
                for (int32_t i = 0; i < pc; i++)
                    for (int32_t j = 0; j < ocnt[i]; j++) tmp[q++] = load_row(oldk[i] * MAXN + j);
                q = 0;
                for (int32_t i = 0; i < cc; i++)
                    for (int32_t j = 0; j < ncnt[i]; j++) {
                        store_row(newk[i] * MAXN + j, tmp[q]);
                        z.RLEAF(tmp[q++].rid) = (IX)newk[i];
                    }
            }
            for (int32_t ni = 0; ni < cc; ni++) {
                int32_t nb = newk[ni];
                nch[nb] = (int8_t)ncnt[ni];
                npar[nb] = (IX)parent;
                nlev[nb] = 0;
                nsc[nb] = -1;
                if (ncnt[ni] < MAXN) clear_slots(nb * MAXN + ncnt[ni], MAXN - ncnt[ni]);
            }
            int32_t nl = h.nleaf;
            int32_t delta = cc - pc;
            if constexpr (TILED) { /* the rope: extra leaves after the kept ones, surplus ones out */
                for (int32_t i = pc; i < cc; i++) rope_insert_after(newk[i - 1], newk[i]);
                for (int32_t i = cc; i < pc; i++) rope_remove(oldk[i]);
                leaves_restat(newk, cc);
            }
            for (int32_t i = cc; i < pc; i++) free_node(oldk[i]);
            if constexpr (!TILED) {
                /* lorder: [firstPos, firstPos+pc) becomes [firstPos, firstPos+cc) */
                lorder_shift(firstPos + pc, nl, delta);
                for (int32_t i = pc; i < cc; i++) {
                    lo[firstPos + i] = (IX)newk[i];
                    lp[newk[i]] = (IX)(firstPos + i);
                }
            }
            h.nleaf = nl + delta;
            if (delta > 0) note_leaves();
            for (int32_t i = 0; i < cc; i++) z.KIDS(parent * MAXN + i) = (IX)newk[i];
            nch[parent] = (int8_t)cc;
          }
        } else {
            MT_PROF_SCOPE(PH_P2);
            if constexpr (W::N >= MAXN * MAXN) {
                /* interior, wave-parallel: lane q reads grandchild q & 7 of child q >> 3 in one pass,
                 * its rank among all grandchildren places it in the regrouped nodes */
                int32_t q = w.lane();
                int32_t i = q >> 3, j = q & (MAXN - 1);
                int32_t cb = i < pc ? z.KIDS(parent * MAXN + i) : -1;
                int32_t cn = cb >= 0 ? nch[cb] : 0;
                bool has = j < cn;
                int32_t ch = has ? z.KIDS(cb * MAXN + j) : -1;
                uint64_t vm = w.ballot(has);
                int32_t total = __builtin_popcountll(vm);
                uint64_t below = q ? (~0ull >> (64 - q)) : 0ull;
                int32_t rank = __builtin_popcountll(vm & below);
                int32_t cc = total / (MAXN / 2);
                if (cc > MAXN - 1) cc = MAXN - 1;
                if (cc < 1) cc = 1;
                int32_t base = total / cc, extra = total % cc;
                /* the old children, then the new nodes: lane broadcasts and a lane array (lane ni: new node ni),
                 * not locally indexed arrays (scratch memory) */
                for (int32_t k = 0; k < pc; k++) free_node(w.bcast(cb, k * MAXN));
                int32_t nbv = 0;
                for (int32_t ni = 0; ni < cc; ni++) {
                    int32_t nb = alloc_node(lvl);
                    if (nb < 0) return;
                    nbv = w.writelane(nb, ni, nbv);
                }
                /* the first `extra` nodes take base + 1 children */
                int32_t big = extra * (base + 1);
                int32_t ni = rank < big ? rank / (base + 1) : extra + (rank - big) / base;
                int32_t slot = rank < big ? rank - ni * (base + 1) : rank - big - (ni - extra) * base;
                int32_t nb = w.shfl(nbv, ni >= 0 && ni < cc ? ni : 0); /* every lane active: a shuffle */
                w.sync();
                if (has) {
                    z.KIDS(nb * MAXN + slot) = (IX)ch;
                    npar[ch] = (IX)nb;
                }
                w.sync();
                if (q < cc) {
                    nch[nbv] = (int8_t)(base + (q < extra ? 1 : 0));
                    npar[nbv] = (IX)parent;
                    z.KIDS(parent * MAXN + q) = (IX)nbv;
                }
                w.sync();
                nch[parent] = (int8_t)cc;
            } else {
                IX hold[MAXN * MAXN];
                int32_t total = 0;
                int32_t oldk[MAXN];
                for (int32_t i = 0; i < pc; i++) {
                    int32_t cb = z.KIDS(parent * MAXN + i);
                    oldk[i] = cb;
                    for (int32_t q = 0; q < nch[cb]; q++) hold[total++] = z.KIDS(cb * MAXN + q);
                }
                int32_t cc = total / (MAXN / 2);
                if (cc > MAXN - 1) cc = MAXN - 1;
                if (cc < 1) cc = 1;
                int32_t base = total / cc, extra = total % cc;
                for (int32_t i = 0; i < pc; i++) free_node(oldk[i]);
                int32_t read = 0;
                for (int32_t ni = 0; ni < cc; ni++) {
                    int32_t cnt = base + (extra > 0 ? 1 : 0);
                    if (extra > 0) extra--;
                    int32_t nb = alloc_node(lvl);
                    if (nb < 0) return;
                    for (int32_t q = 0; q < cnt; q++) {
                        int32_t ch = hold[read++];
                        z.KIDS(nb * MAXN + q) = (IX)ch;
                        npar[ch] = (IX)nb;
                    }
                    nch[nb] = (int8_t)cnt;
                    npar[nb] = (IX)parent;
                    z.KIDS(parent * MAXN + ni) = (IX)nb;
                }
                nch[parent] = (int8_t)cc;
            }
        }
        if (!(nch[parent] < MAXN / 2 && npar[parent] >= 0)) return;
        block = parent;
      }
    }
    /* zamboniSegments (mergeTree.ts:1455-1511) */
    MT_HD void zamboni() {
        MT_PROF_SCOPE(PH_ZAMBONI);
        if (!h.collaborating) return;
        for (int i = 0; i < 2; i++) {
            if (h.heapN < 1) break;
            if (zh->heapTop > h.minSeq) break; /* peek (mergeTree.ts:1465-1468) */
            int32_t rid, mseq, gen;
            heap_pop(&rid, &mseq, &gen);
            int32_t n, before, after, par;
            if constexpr (W::N >= MAXN * MAXN) {
                /* slot_of, needsScour and scourNode's row reads in two round trips: the row's leaf, then
                 * everything about that leaf */
                int32_t g = z.RGEN(rid);
                n = z.RLEAF(rid);
                if (g != (uint8_t)gen) continue; /* unlinked since it was queued */
                int32_t j = w.lane();
                HotRow r = load_row(n * MAXN + (j & (MAXN - 1)));
                before = nch[n];
                int32_t sc = nsc[n];
                par = npar[n];
                if (!w.ballot(j < before && r.rid == (IX)rid)) continue; /* merged away since it was queued */
                if (sc == 0) continue;
                MT_PROF_COUNT(PH_C_SCOUR, 1);
                int32_t cnt1[1];
                scour_par(&n, 1, cnt1, &r, before);
                after = cnt1[0];
            } else {
                int32_t s = slot_of(rid, gen); /* -1: unlinked or merged away since it was queued */
                if (s < 0) continue;
                n = s / MAXN;
                if (nsc[n] == 0) continue;
                before = nch[n];
                MT_PROF_COUNT(PH_C_SCOUR, 1);
                after = scour_one(n);
                par = npar[n];
            }
            nsc[n] = 0;
            if (after < before) {
                MT_PROF_COUNT(PH_C_PACK, after < MAXN / 2 && par >= 0);
                if (after < MAXN / 2 && par >= 0) pack(n);
            }
        }
    }
    /* A zamboniSegments call the record makes (at the end of insertSegments / markRangeRemoved /
     * annotateRange / ackPendingSegment, and in setMinSeq): queued and run when the record is done
     * (run_zamboni), under the minSeq of the call. Nothing a record does after such a call reads what zamboni
     * changes, so the order of effects is the reference's; and zamboni is inlined once, not at every caller
     * (the replay kernel's code is several hundred KB: instruction-cache pressure). */
    MT_HD void zamboni_soon() {
        if (zq == 0) zms = h.minSeq;
        zq++;
    }
    MT_HD void run_zamboni() {
#pragma clang loop unroll(disable)
        for (int32_t i = 0; i < zq; i++) { /* at most 2: the op's or the ack's, then setMinSeq's */
            int32_t ms = h.minSeq;
            if (i == 0) h.minSeq = zms;
            zamboni();
            h.minSeq = ms;
        }
        zq = 0;
    }
    /* setMinSeq (mergeTree.ts:1751-1769) */
    MT_HD void set_min_seq(int32_t minSeq) {
        if (!(minSeq <= h.currentSeq)) fail(E_ASSERT);
        if (!(h.minSeq <= minSeq)) fail(E_ASSERT);
        if (minSeq > h.minSeq) {
            h.minSeq = minSeq;
            zamboni_soon();
        }
    }

    /* ---- insert (insertSegments 2001-2031, blockInsert 2174-2257) -------------------- */
    /* breakTie for a zero-length row (2281-2310) */
    MT_HD bool break_tie_of(const RowView& r, int32_t refSeq, int32_t client) const {
        int32_t rs = r.rseq;
        if (rs != NOREM && rs != 0 && rs <= refSeq && rs != UNASSIGNED_SEQ) return false;
        if (client == h.localShort) return true;
        return r.seq != UNASSIGNED_SEQ;
    }
    MT_HD bool break_tie(int32_t s, int32_t refSeq, int32_t client) const {
        return break_tie_of(row_view(s), refSeq, client);
    }
    /* continueFrom (2187-2194): first row after leaf lorder[k] with localNetLength > 0 is a
     * local-pending insert */
    MT_HD bool continue_from(int32_t k) {
        if constexpr (TILED) { /* walk the following leaves in order (the first visible row is near) */
            for (int32_t kk = knext(k); kvalid(kk); kk = knext(kk)) {
                int32_t n = leaf_at(kk), c = nch[n];
                int32_t fj = -1;
                if constexpr (W::N >= MAXN) {
                    int32_t j = w.lane();
                    bool hit = j < c && z.len(n * MAXN + (j & 7)) > 0 && z.rseq(n * MAXN + (j & 7)) == NOREM;
                    uint64_t m = w.ballot(hit);
                    if (m) fj = W::ffs(m);
                } else {
                    for (int32_t j = 0; j < c && fj < 0; j++)
                        if (z.len(n * MAXN + j) > 0 && z.rseq(n * MAXN + j) == NOREM) fj = j;
                }
                if (fj >= 0) return z.seq(n * MAXN + fj) == UNASSIGNED_SEQ;
            }
            return false;
        }
        int32_t T = h.nleaf * MAXN;
        for (int32_t b = (k + 1) * MAXN; b < T; b += 4 * W::N) {
            int32_t s0 = quad_slot(b + 4 * w.lane());
            int32_t fq = -1, fseq = 0;
            if (s0 >= 0) {
                I4 L = ld4(&z.len(s0));
                I4 R = ld4(&z.rseq(s0));
                I4 Q = ld4(&z.seq(s0));
                for (int q = 3; q >= 0; q--)
                    if (L.x[q] > 0 && R.x[q] == NOREM) {
                        fq = q;
                        fseq = Q.x[q];
                    }
            }
            uint64_t m = w.ballot(fq >= 0);
            if (m) return w.bcast(fseq, W::ffs(m)) == UNASSIGNED_SEQ;
        }
        return false;
    }
    /* ensureIntervalBoundary (2274-2278): split the row strictly containing pos */
    MT_HD void ensure_boundary(int32_t pos, int32_t refSeq, int32_t client) {
        int32_t P, s, v;
        int32_t t = find_reach(pos, refSeq, client, &P, &s, &v);
        if (t < 0) return;
        if (P + v > pos) split_row(t, pos - P);
    }
    /* returns the slot of the inserted row or -1 */
    /* Boundary split (ensureIntervalBoundary, 2274-2278) and insert placement (blockInsert,
     * 2174-2257) from ONE perspective scan: the row reaching pos (P < pos <= P + vis) is split
     * at pos if pos falls strictly inside it; placement then resumes right after its left part. */
    MT_HD int32_t insert_row(int32_t pos, int32_t refSeq, int32_t client, int32_t seq) {
        MT_PROF_SCOPE(PH_INSROW);
        MT_PROF_COUNT(PH_C_INS, 1);
        int32_t k, j;
        if (pos == 0) {
            k = 0;
            j = 0;
        } else {
            int32_t P, s, v;
            HotRow lr;
            int32_t lc = -1; /* the found leaf's rows and child count (tiled GPU search): the split reuses them */
            constexpr bool PRE = TILED && W::N >= 64;
            int32_t t = find_reach(pos, refSeq, client, &P, &s, &v, PRE ? &lr : nullptr, PRE ? &lc : nullptr);
            if (t < 0) return -1;
            int32_t fls = PRE && lc >= 0 ? w.bcast((int32_t)lr.flags, s & (MAXN - 1)) : z.flags(s);
            if (P + v > pos && !(fls & RF_MARKER)) {
                int32_t rs = -1, gap = -1;
                int32_t ls = split_row(t, pos - P, &rs, &gap, PRE && lc >= 0 ? &lr : nullptr, PRE ? lc : -1);
                if (ls < 0) return -1;
                /* the right part (visible: the row was) starts the run at pos and captures the insert, which goes
                 * right before it when no leaf boundary falls between the halves (Appendix C); no row read, and on
                 * the GPU the split's own write pass left the slot */
                if (gap >= 0) return gap;
                if (rs >= 0 && rs / MAXN == ls / MAXN) return leaf_insert_slot(ls / MAXN, (ls & (MAXN - 1)) + 1);
                k = kpos(ls / MAXN);
                j = (ls & (MAXN - 1)) + 1;
            } else {
                k = t >> 3;
                j = t & 7;
                /* pos strictly inside an unsplittable segment: insert before it */
                if (!(P + v > pos)) j++;
            }
        }
        for (;;) {
            int32_t n = leaf_at(k);
            int32_t c = nch[n];
            for (; j < c; j++) {
                int32_t s = n * MAXN + j;
                RowView r = row_view(s);
                if (vis_of(s, r, refSeq, client) > 0 || break_tie_of(r, refSeq, client)) return leaf_insert_slot(n, j);
            }
            if (seq != UNASSIGNED_SEQ && kvalid(knext(k)) && continue_from(k)) {
                k = knext(k);
                j = 0;
                continue;
            }
            return leaf_insert_slot(n, c);
        }
    }
    /* a segment record's length (mt_oplog.h): text_len, or pos2 for snapshot-load records */
    MT_HD static int32_t seg_len(const mt_op_rec& op) {
        if (op.seg_kind == MT_SEG_MARKER) return 1;
        return (op.kind & MT_OP_KIND_MASK) >= MT_OP_RELOAD ? op.pos2 : op.text_len;
    }
    /* insertSegments (mergeTree.ts:2001-2040) of one segment; preRseq > 0: the segment arrives
     * already removed (a loaded segment's merge info, snapshotLoader.ts:101-106) */
    MT_HD void insert_segments(const mt_op_rec& op, const Pools& p, int32_t refSeq, int32_t client, int32_t seq,
                               int32_t preRseq = 0, uint8_t preRcli = 0, int32_t atT = -1) {
        int32_t pos = op.pos1;
        bool hasL = seq == UNASSIGNED_SEQ;
        int32_t localSeq = hasL ? ++zh->localSeq : 0;
        bool marker = op.seg_kind == MT_SEG_MARKER;
        bool perm = op.seg_kind == MT_SEG_PERM; /* PermutationSegment(length) (permutationvector.ts:47-51) */
        /* new SubSequence(items) (sharedSequence.ts:116-125): its items are the record's units (item ids); the document
         * becomes a SubSequence document (the host keeps TextSegment inserts out of it, mt_engine_submit) */
        const bool run = op.seg_kind == MT_SEG_RUN;
        if (run) zh->ndv |= DV_RUN;
        int32_t L = seg_len(op);
        if (L <= 0) ensure_boundary(pos, refSeq, client); /* the split still happens (2004) */
        if (L > 0) {
            /* tiled profile: read ahead of the position search, the free row-id stack's top and (a text of at
             * most a wave's length) the op's text, one unit per lane (config 4 +2.2 %; at config 3's 8 waves per
             * SIMD the live registers cost more than the round trips: -2.8 %, r04r) */
            constexpr bool RA = TILED && W::N >= 64;
            const bool text = !marker && !perm;
            int32_t nfr = RA ? zh->nfreeRid : 0;
            int32_t frr = RA ? (int32_t)d.FRID(nfr > 0 ? nfr - 1 : 0) : 0;
            /* and the entry under it (its line): a split of the row at pos takes the top for its right part */
            int32_t frr2 = RA ? (int32_t)d.FRID(nfr > 1 ? nfr - 2 : 0) : 0;
            /* the props record of a segment with properties (the shared pool: a cache hit), for the row set-up */
            const bool pa = RA && op.props;
            int32_t prOff = 0, prN = 0, prComb = 0;
            if (pa) {
                const mt_props_rec& pr0 = p.props[op.props - 1];
                prOff = (int32_t)pr0.kv_off;
                prN = pr0.nkv;
                prComb = pr0.combining;
            }
            const bool tpreOk = RA && text && L <= W::N;
            int32_t tpre = tpreOk && w.lane() < L ? p.text[op.text_off + w.lane()] : 0;
            int32_t off = 0;
            if (!marker && !perm) {
                MT_PROF_SCOPE(PH_TEXT);
                off = arena_alloc(L);
                if (off < 0) return;
            }
            /* atT >= 0: right before the row at document coordinate atT (insertAtReferencePosition) */
            int32_t s = atT >= 0 ? leaf_insert_slot(leaf_at(atT >> 3), atT & (MAXN - 1)) : insert_row(pos, refSeq, client, seq);
            if (s < 0) {
                fail(E_INSERT_FAILED);
                return;
            }
            MT_PROF_SCOPE(PH_PLACE);
            /* flat GPU profile: the set-up's independent reads issued together once the search is done (no register
             * lives across it, which at 8 waves per SIMD costs more than it saves, r04r): the free row-id stack's top,
             * the text (up to a wave's length), the props record; then the row id's generation with the property
             * reads */
            constexpr bool FP = !TILED && W::N >= 64;
            int32_t fnfr = 0, ffrr = 0, ftp = 0, fpOff = 0, fpN = 0, fpComb = 0;
            const bool ftpOk = FP && text && L <= W::N;
            const bool fpa = FP && op.props;
            if constexpr (FP) {
                fnfr = zh->nfreeRid;
                ffrr = (int32_t)d.FRID(fnfr > 0 ? fnfr - 1 : 0);
                ftp = ftpOk && w.lane() < L ? p.text[op.text_off + w.lane()] : 0;
                if (fpa) {
                    const mt_props_rec& pr0 = p.props[op.props - 1];
                    fpOff = (int32_t)pr0.kv_off;
                    fpN = pr0.nkv;
                    fpComb = pr0.combining;
                }
            }
            int32_t rid;
            if (RA && zh->nfreeRid == nfr && nfr > 0) { /* alloc_rid, with the stack's top read above */
                zh->nfreeRid = nfr - 1;
                rid = frr;
            } else if (RA && zh->nfreeRid == nfr - 1 && nfr > 1) { /* a split took the top */
                zh->nfreeRid = nfr - 2;
                rid = frr2;
            } else if (FP && fnfr > 0) {
                zh->nfreeRid = fnfr - 1;
                rid = ffrr;
            } else {
                rid = alloc_rid();
            }
            const int32_t fgen = FP ? (int32_t)z.RGEN(rid) : 0; /* for the LRU entry */
            int32_t gen = 0, sc = 0;
            if (RA) { /* for the window set and the LRU entry: one round trip */
                gen = z.RGEN(rid);
                sc = nsc[s / MAXN];
            }
            z.RID(s) = (IX)rid;
            typename HT::Cold& c = d.COLD(rid); /* row id kept in a register, not re-read per field */
            z.len(s) = L;
            z.seq(s) = seq;
            z.rseq(s) = preRseq > 0 ? preRseq : NOREM;
            int32_t fl = (marker ? RF_MARKER : 0) | (perm ? RF_PERM : 0) | (hasL ? RF_LSEQ : 0);
            /* the cold row's first 16 bytes in one store: lseq, lrseq = 0, toff (text offset / a marker's refType
             * / an unallocated PermutationSegment start), prw = gc = ovx = 0; then the inline overlap list. pv / pk
             * are set up by add_props with RF_PROPS. */
            I4 c0;
            c0.x[0] = localSeq;
            c0.x[1] = 0;
            /* a PermutationSegment's start: unallocated, except a loaded body segment's (APPEND records carry it) */
            c0.x[2] = marker ? op.pos2 : perm ? ((op.kind & MT_OP_KIND_MASK) == MT_OP_APPEND ? (int32_t)op.text_off : 0) : off;
            c0.x[3] = 0;
            st4(&c, c0);
            c.ovl = 0;
            z.RLEAF(rid) = (IX)(s / MAXN);
            h.nrows++;
            zh->sumW++;
            if (preRseq <= 0) h.localLen += L;
            if (text) {
                MT_PROF_SCOPE(PH_TEXT);
                int32_t last;
                if (tpreOk || ftpOk) {
                    const int32_t tv = tpreOk ? tpre : ftp;
                    if (w.lane() < L) arena_base(zh->arenaSide)[off + w.lane()] = (uint16_t)tv;
                    last = w.bcast(tv, L - 1);
                    w.sync();
                } else {
                    last = arena_copy(arena_base(zh->arenaSide) + off, p.text + op.text_off, L);
                }
                fl |= RF_NLK | (last == '\n' && !run ? RF_NL : 0);
            }
            /* {cli, rcli, flags, ng = 0} in one store */
            st_bytes4(s, (uint32_t)(uint8_t)(client < 0 ? LOCAL_CLIENT : client) |
                             ((uint32_t)(preRseq > 0 ? preRcli : 0) << 8) | ((uint32_t)(uint8_t)fl << 16));
            if (pa || fpa) { /* TextSegment.make(text, props): the new row's flags are known (no RF_PROPS), so nothing of
                              * it is read; its kv reads go out with the set-up's (one round trip) */
                const int32_t ko = pa ? prOff : fpOff, kn = pa ? prN : fpN, kc = pa ? prComb : fpComb;
                add_props(s, p.kv + ko, kn, kc == MT_COMBINE_REWRITE ? MT_COMBINE_REWRITE : MT_COMBINE_NONE, 0, false, fl);
            }
            if constexpr (RA)
                row_enter_known(s, rid, gen, seq, preRseq > 0 ? preRseq : NOREM, L);
            else if constexpr (TILED)
                row_enter(s);
            if (op.props && !pa && !fpa) { /* TextSegment.make(text, props): addProperties without collab */
                const mt_props_rec& pr = p.props[op.props - 1];
                add_props(s, p.kv + pr.kv_off, pr.nkv, pr.combining == MT_COMBINE_REWRITE ? MT_COMBINE_REWRITE : MT_COMBINE_NONE,
                          0, false);
            }
            if (h.collaborating) { /* saveIfLocal (2197-2212) */
                if (seq == UNASSIGNED_SEQ && client == h.localShort) {
                    bool created = false;
                    pending_add(s, localSeq, &created);
                } else if (seq > h.minSeq) {
                    if (RA)
                        add_lru_known(s / MAXN, rid, gen, sc, seq);
                    else if (FP)
                        add_lru_known(s / MAXN, rid, fgen, nsc[s / MAXN], seq);
                    else
                        add_lru(s, seq);
                }
            }
            if (dl_on()) { /* INSERT delta (mergeTree.ts:2014-2021), after blockInsert */
                int32_t pp = local_pos(s);
                dhead(MT_DELTA_INSERT);
                dseg(pp, L);
                dtail(1);
            }
        }
        if (h.collaborating && seq != UNASSIGNED_SEQ) zamboni_soon();
    }

    /* ---- range ops: markRangeRemoved (2640-2752) / annotateRange (2598-2638) ----------- */
    /* Boundaries and visit of a range op in ONE perspective scan. The reference splits at start
     * (ensureIntervalBoundary, mergeTree.ts:2274-2278), then at end, then visits the rows with
     * length > 0 in [start, end) (nodeMap, 2936-2998). The rows it visits are exactly the rows with
     * vis > 0 overlapping [start, end) before the splits — a contiguous run in document order — with
     * the first replaced by its right part if start falls inside it and the last cut at end. So one
     * scan finds the first and the last overlapping row, the two splits are made in the reference's
     * order, and the visit walks document order from the first row to the last. */
    /* Visit, in document order, the rows with vis > 0 from slot sa to slot sb: leaf(s, pos). With dl,
     * pos is the row's local-view position once the visit is done (Client.getPosition at the delta
     * callback, client.ts:291): the local length before sa plus, for each row passed, its local length
     * after its own visit (a REMOVE drops a visited row's; an ANNOTATE changes none). */
    template <class F>
    MT_HD void visit_run(int32_t sa, int32_t sb, int32_t refSeq, int32_t client, F& leaf, bool dl) {
        MT_PROF_SCOPE(PH_VISIT);
        int32_t run = dl ? local_pos(sa) : 0;
        int32_t ka = kpos(sa / MAXN), kb = kpos(sb / MAXN);
        for (int32_t k = ka;; k = knext(k)) {
            int32_t n = leaf_at(k), c = nch[n];
            int32_t j0 = k == ka ? (sa & (MAXN - 1)) : 0;
            int32_t j1 = k == kb ? (sb & (MAXN - 1)) : c - 1;
            for (int32_t j = j0; j <= j1; j++) {
                if (vis(n * MAXN + j, refSeq, client) > 0) leaf(n * MAXN + j, run);
                if (dl) run += local_len(n * MAXN + j);
            }
            if (k == kb || !kvalid(knext(k))) break;
        }
    }
    template <class F>
    MT_HD void range_op(int32_t start, int32_t end, int32_t refSeq, int32_t client, F&& leaf, bool dl = false) {
        MT_PROF_SCOPE(PH_MAP);
        MT_PROF_COUNT(PH_C_RANGE, 1);
        if constexpr (TILED) {
            range_op_tiled(start, end, refSeq, client, leaf, dl);
            return;
        }
        int32_t run = 0;
        int32_t T = h.nleaf * MAXN;
        int32_t tf = -1, Pf = 0, vf = 0, tg = -1, Pg = 0, vg = 0, sf = -1, sg = -1;
        {
            MT_PROF_SCOPE(PH_FIND);
            const bool loc = is_local(client);
            constexpr int NB = W::N >= 64 ? MT_SCAN_NB : 1; /* wave blocks whose loads are issued together */
            bool done = false;
            for (int32_t b0 = 0; b0 < T && !done; b0 += NB * 4 * W::N) {
                int32_t s0[NB];
                QuadRows x[NB];
#pragma unroll
                for (int q = 0; q < NB; q++) s0[q] = quad_slot(b0 + q * 4 * W::N + 4 * w.lane());
#pragma unroll
                for (int q = 0; q < NB; q++) x[q] = quad_load(s0[q], loc);
#pragma unroll
                for (int bq = 0; bq < NB; bq++) {
                    int32_t b = b0 + bq * 4 * W::N;
                    if (b >= T) {
                        done = true;
                        break;
                    }
                    int32_t v[4];
                    quad_vis_of(s0[bq], x[bq], refSeq, client, v);
                    int32_t tot;
                    int32_t p = run + w.excl_scan(v[0] + v[1] + v[2] + v[3], &tot);
                    int32_t hf = -1, pf = 0, lf = 0, hl = -1, pl = 0, ll = 0;
                    for (int q = 0; q < 4; q++) {
                        if (v[q] > 0 && p < end && p + v[q] > start) {
                            if (hf < 0) {
                                hf = q;
                                pf = p;
                                lf = v[q];
                            }
                            hl = q;
                            pl = p;
                            ll = v[q];
                        }
                        p += v[q];
                    }
                    uint64_t m = w.ballot(hf >= 0);
                    if (m) {
                        if (tf < 0) {
                            int32_t l = W::ffs(m);
                            tf = b + 4 * l + w.bcast(hf, l);
                            sf = w.bcast(s0[bq] + hf, l);
                            Pf = w.bcast(pf, l);
                            vf = w.bcast(lf, l);
                        }
                        int32_t l2 = 63 - __builtin_clzll(m);
                        tg = b + 4 * l2 + w.bcast(hl, l2);
                        sg = w.bcast(s0[bq] + hl, l2);
                        Pg = w.bcast(pl, l2);
                        vg = w.bcast(ll, l2);
                    }
                    run += tot;
                    if (run >= end) {
                        done = true;
                        break;
                    }
                }
            }
        }
        if (tf < 0) return;
        int32_t sa = sf, sb = sg; /* no split: the rows stay where the scan found them */
        if (Pf < start || Pg + vg > end) {
            int32_t ridLast = z.RID(sg);
            int32_t ridFirst = z.RID(sf);
            int32_t sl = sg; /* the last row's slot, while nothing has moved it */
            if (Pf < start) { /* start falls inside the first row: split it; its right part is first */
                int32_t rs = -1, rr = -1;
                if (split_row(tf, start - Pf, &rs, nullptr, nullptr, -1, &rr) < 0 || rs < 0) return;
                sl = -1;
                if (tf == tg) {
                    ridLast = rr;
                    sl = rs;
                    vg = Pf + vf - start;
                    Pg = start;
                }
                ridFirst = rr;
            }
            if (Pg + vg > end) { /* end falls inside the last row: split it; its left part keeps the id */
                if (sl < 0) sl = slot_of(ridLast, -1);
                if (sl < 0) {
                    fail(E_ASSERT);
                    return;
                }
                if (split_row(kpos(sl / MAXN) * MAXN + (sl & (MAXN - 1)), end - Pg) < 0) return;
            }
            slot_of2(ridFirst, ridLast, &sa, &sb);
            if (sa < 0 || sb < 0) {
                fail(E_ASSERT);
                return;
            }
        }
        if (runOnly) {
            runA = sa;
            runB = sb;
            return;
        }
        if (dl) { /* delta events need each visited row's position: the serial visit */
            visit_run(sa, sb, refSeq, client, leaf, true);
            return;
        }
        int32_t ta = kpos(sa / MAXN) * MAXN + (sa & (MAXN - 1));
        int32_t tb = kpos(sb / MAXN) * MAXN + (sb & (MAXN - 1));
        for (int32_t b = ta & ~3; b <= tb; b += 4 * W::N) {
            int32_t t0 = b + 4 * w.lane();
            int32_t s0 = quad_slot(t0);
            int32_t v[4];
            quad_vis(s0, refSeq, client, v);
            int32_t hm = 0;
            for (int q = 0; q < 4; q++)
                if (v[q] > 0 && t0 + q >= ta && t0 + q <= tb) hm |= 1 << q;
            uint64_t m = w.ballot(hm != 0);
            while (m) {
                int32_t l = W::ffs(m);
                m &= m - 1;
                int32_t bits = w.bcast(hm, l);
                int32_t sbase = w.bcast(s0, l);
                while (bits) {
                    int32_t q = __builtin_ctz((unsigned)bits);
                    bits &= bits - 1;
                    leaf(sbase + q, 0);
                }
            }
        }
    }
    /* range_op for the tiled profile: the first and last rows overlapping [start, end) are the rows
     * reaching start + 1 and min(end, length) (one window pass, two summary searches); the same
     * two splits; then the rows with length > 0 between them are visited leaf by leaf. */
    template <class F>
    MT_HD void range_op_tiled(int32_t start, int32_t end, int32_t refSeq, int32_t client, F& leaf, bool dl) {
        int32_t tf, Pf, tg, Pg, sf = -1, vf = 0, sg = -1, vg = 0;
        HotRow fr;
        int32_t fc = -1; /* the first row's leaf as the search read it (lanes 0-7), for its split */
        if (tiles_cover(refSeq, client)) {
            int32_t total = win_pass(refSeq, client) + stable_total();
            if (start >= total || end <= start) {
                win_clear();
                return;
            }
            int32_t last = end < total ? end : total;
            int32_t P1 = 0, P2 = 0;
            int32_t n1 = 0, n2 = 0, k1, k2;
#if MT_FIND2
            if constexpr (W::N >= 64) {
                tile_find2(start + 1, last, &k1, &P1, &n1, &k2, &P2, &n2);
            } else
#endif
            {
                k1 = tile_find(start + 1, refSeq, client, &P1, &n1);
                k2 = tile_find(last, refSeq, client, &P2, &n2);
            }
            win_clear();
            if (k1 < 0 || k2 < 0) {
                fail(E_ASSERT);
                return;
            }
#if MT_FIND2
            if constexpr (W::N >= 64) {
                leaf_find2(k1, n1, P1, start + 1, k2, n2, P2, last, refSeq, client, &tf, &Pf, &sf, &vf, &tg, &Pg, &sg,
                           &vg, &fr, &fc);
            } else
#endif
            {
                tf = leaf_find(k1, n1, P1, start + 1, refSeq, client, &Pf, &sf, &vf);
                tg = leaf_find(k2, n2, P2, last, refSeq, client, &Pg, &sg, &vg);
            }
        } else {
            int32_t total = length_tiled(refSeq, client);
            if (start >= total || end <= start) return;
            tf = find_reach_walk(start + 1, refSeq, client, &Pf, &sf, &vf);
            tg = find_reach_walk(end < total ? end : total, refSeq, client, &Pg, &sg, &vg);
        }
        if (tf < 0 || tg < 0) return;
        if (Pf >= start && Pg + vg <= end) { /* no split: the rows stay where the searches found them */
            if (runOnly) {
                runA = sf;
                runB = sg;
                return;
            }
            visit_run(sf, sg, refSeq, client, leaf, dl);
            return;
        }
        int32_t ridLast = z.RID(sg);
        int32_t ridFirst = z.RID(sf);
        int32_t sl = sg; /* the last row's slot, while nothing has moved it */
        if (Pf < start) {
            int32_t rs = -1, rr = -1;
            if (split_row(tf, start - Pf, &rs, nullptr, fc >= 0 ? &fr : nullptr, fc, &rr) < 0 || rs < 0) return;
            sl = -1;
            if (tf == tg) {
                ridLast = rr;
                sl = rs;
                vg = Pf + vf - start;
                Pg = start;
            }
            ridFirst = rr;
        }
        if (Pg + vg > end) {
            if (sl < 0) sl = slot_of(ridLast, -1);
            if (sl < 0) {
                fail(E_ASSERT);
                return;
            }
            if (split_row(kpos(sl / MAXN) * MAXN + (sl & (MAXN - 1)), end - Pg) < 0) return;
        }
        int32_t sa, sb;
        slot_of2(ridFirst, ridLast, &sa, &sb);
        if (sa < 0 || sb < 0) {
            fail(E_ASSERT);
            return;
        }
        if (runOnly) {
            runA = sa;
            runB = sb;
            return;
        }
        visit_run(sa, sb, refSeq, client, leaf, dl);
    }
    /* markRangeRemoved's per-segment step (mergeTree.ts:2660-2700, the range_edit callback below) on the rows with
     * vis > 0 from slot sa to slot sb, a leaf at a time with one lane per row (tiled profile, no delta events, no
     * local references): every row's fields are read in one pass and the row updates are made in parallel; the
     * steps whose order is observable — overlap-list pushes, window-set appends, the leaf's LRU entry (added by
     * its first such row), pending-group entries — are taken in row order. Same result as the serial visit.
     * Both profiles (the window set and STABLE summaries are the tiled profile's). */
    MT_HD void remove_run(int32_t sa, int32_t sb, int32_t refSeq, int32_t client, int32_t seq, int32_t localSeq,
                          bool hasL, uint32_t rcl, bool collab, bool* created) {
        MT_PROF_SCOPE(PH_VISIT);
        static_assert(W::N >= MAXN * MAXN, "one lane per row of a leaf");
        auto& t = z.tl;
        const int32_t j = w.lane();
        const uint64_t below = j ? (~0ull >> (64 - j)) : 0ull;
        int32_t ka = kpos(sa / MAXN), kb = kpos(sb / MAXN);
        for (int32_t k = ka;; k = knext(k)) {
            int32_t n = leaf_at(k);
            int32_t s = n * MAXN + (j & (MAXN - 1));
            RowView r = row_view(s); /* the row, its window flags and id, the leaf's child count: one round trip */
            uint8_t x = 0;
            int32_t lch0 = 0, lix0 = 0, lst0 = 0; /* tiled: the leaf's chunk, index and STABLE sum, for its update */
            if constexpr (TILED) {
                x = t.xf[s];
                lch0 = t.lch[n];
                lix0 = t.lix[n];
                lst0 = t.lst[n];
            }
            int32_t sc0 = nsc[n]; /* the leaf's needsScour, for its LRU entry */
            int32_t rid = z.RID(s);
            int32_t c = nch[n];
            int32_t j0 = k == ka ? (sa & (MAXN - 1)) : 0;
            int32_t j1 = k == kb ? (sb & (MAXN - 1)) : c - 1;
            bool sel = j < MAXN && j >= j0 && j <= j1 && vis_of(s, r, refSeq, client) > 0;
            int32_t rs = r.rseq, L = r.len;
            uint32_t b4 = r.b4, fl = (b4 >> 16) & 0xFF;
            bool fresh = sel && rs == NOREM, unas = sel && rs == UNASSIGNED_SEQ;
            const int32_t rgn = sel ? (int32_t)z.RGEN(rid) : 0; /* for the leaf's LRU entry (its read overlaps the updates) */
            int32_t nrs = fresh || unas ? seq : rs; /* rs after the update */
            uint64_t sm = w.ballot(sel);
            zh->sumW += __builtin_popcountll(sm);
            h.localLen -= w.sum(fresh ? L : 0); /* the rows leave the local view */
            if (fresh) {
                z.rseq(s) = seq;
                d.COLD(rid).lrseq = localSeq;
                uint32_t f2 = hasL ? (fl | RF_LRSEQ) : (fl & ~(uint32_t)RF_LRSEQ);
                st_bytes4(s, (b4 & 0xFF0000FFu) | (rcl << 8) | (f2 << 16));
            } else if (unas) {
                z.rseq(s) = seq;
                st_bytes4(s, (b4 & 0xFF0000FFu) | (rcl << 8) | ((fl & ~(uint32_t)RF_LRSEQ) << 16));
            }
            uint64_t om = sm & ~w.ballot(fresh || unas);
            while (om) { /* removed already by another client: removedClientOverlap (rare) */
                int32_t l = W::ffs(om);
                om &= om - 1;
                int32_t sl = w.bcast(s, l);
                uint32_t bl = (uint32_t)w.bcast((int32_t)b4, l);
                ovl_push(sl, client);
                st_bytes4(sl, (bl & 0xFF00FFFFu) | ((((bl >> 16) & 0xFF) | RF_OVL) << 16));
            }
            if constexpr (TILED) {
            /* row_removed: out of the STABLE summaries; into the window set unless the removal is settled */
            bool stable = sel && (x & XF_STABLE);
            int32_t lsd = w.sum(stable ? L : 0);
            uint8_t x2 = stable ? 0 : x;
            bool st = r.seq != UNASSIGNED_SEQ && r.seq <= h.minSeq &&
                      (nrs == NOREM || (nrs != UNASSIGNED_SEQ && nrs <= h.minSeq));
            bool wadd = sel && !(x2 & XF_W) && !st;
            if (wadd) x2 = XF_W;
            uint8_t g = wadd ? z.RGEN(rid) : 0;
            if (sel) t.xf[s] = x2;
            if (lsd) lst_add_known(n, lch0, lix0, lst0, -lsd);
            uint64_t wm = w.ballot(wadd);
            if (wm) {
                int32_t wn = t.wN, cnt = __builtin_popcountll(wm);
                if (wn + cnt > WCAPR) {
                    fail(E_CAPACITY);
                    return;
                }
                if (wadd) {
                    int32_t o = wn + __builtin_popcountll(wm & below);
                    twrid[o] = rid;
                    twgen[o] = g;
                    twslot[o] = s;
                }
                w.sync();
                t.wN = wn + cnt;
            }
            }
            if (collab) {
                bool pend = (fresh || unas) && seq == UNASSIGNED_SEQ && client == h.localShort;
                uint64_t pm = w.ballot(pend);
                while (pm) {
                    int32_t l = W::ffs(pm);
                    pm &= pm - 1;
                    pending_add(w.bcast(s, l), localSeq, created);
                }
                uint64_t lm = sm & ~w.ballot(pend);
                if (lm && sc0 != 1 && seq > h.currentSeq) { /* add_lru of the leaf's first such row (it marks the leaf) */
                    nsc[n] = 1;
                    heap_add(w.bcast(rid, W::ffs(lm)), seq, w.bcast(rgn, W::ffs(lm)));
                }
            }
            if (k == kb || !kvalid(knext(k))) break;
        }
    }

    /* markRangeRemoved (2640-2752) and annotateRange (2598-2638) share one range walk (range_op is inlined once
     * for both: the replay kernel's code size is what its instruction cache sees) */
    MT_HD void mark_range_removed(int32_t start, int32_t end, int32_t refSeq, int32_t client, int32_t seq) {
        range_edit(true, start, end, nullptr, 0, MT_COMBINE_NONE, refSeq, client, seq);
    }
    MT_HD void annotate_range(int32_t start, int32_t end, const mt_kv* kv, int32_t nkv, int32_t comb, int32_t refSeq,
                              int32_t client, int32_t seq) {
        range_edit(false, start, end, kv, nkv, comb, refSeq, client, seq);
    }
    MT_HD void range_edit(bool remove, int32_t start, int32_t end, const mt_kv* kv, int32_t nkv, int32_t comb,
                          int32_t refSeq, int32_t client, int32_t seq) {
        bool hasL = seq == UNASSIGNED_SEQ;
        int32_t localSeq = hasL ? ++zh->localSeq : 0;
        bool created = false;
        const bool collab = h.collaborating;
        const uint32_t rcl = (uint8_t)(client < 0 ? LOCAL_CLIENT : client);
        const bool dl = dl_on();
        bool dh = false; /* the event's head goes out after the boundary splits' SPLIT events */
        int32_t dn = 0;
        const bool rf = refs_on();
        bool saved = false;
        const int32_t dop = remove ? MT_DELTA_REMOVE : MT_DELTA_ANNOTATE;
        if constexpr (W::N >= MAXN * MAXN) {
            if (remove && !dl && !rf) { /* find and split, then the lane-parallel visit */
                auto none = [](int32_t, int32_t) {};
                runOnly = true;
                runA = -1;
                range_op(start, end, refSeq, client, none, false);
                runOnly = false;
                if (runA >= 0 && !h.err) remove_run(runA, runB, refSeq, client, seq, localSeq, hasL, rcl, collab, &created);
                if (h.collaborating && seq != UNASSIGNED_SEQ) zamboni_soon();
                return;
            }
        }
        range_op(start, end, refSeq, client, [&](int32_t s, int32_t dpos) {
            if (dl && !dh) {
                dhead(dop);
                dh = true;
            }
            zh->sumW++;
            if (!remove) { /* annotateRange's annotateSegment (2606-2621) */
                if (dl) { /* deltaSegments.push({segment, propertyDeltas}) (mergeTree.ts:2608-2609) */
                    dput(dpos);
                    dput(z.len(s));
                    prop_deltas(s, kv, nkv, comb, seq, collab);
                    dn++;
                }
                if (z.flags(s) & RF_MARKER) marker_keys_annotated(s, kv, nkv, comb == MT_COMBINE_REWRITE);
                add_props(s, kv, nkv, comb, seq, collab);
                if (collab) {
                    if (hasL)
                        pending_add(s, localSeq, &created);
                    else
                        add_lru(s, seq);
                }
                return;
            }
            int32_t rs = z.rseq(s), L = z.len(s);
            uint32_t b4 = ld_bytes4(s); /* {cli, rcli, flags, ng}: one read, one write */
            uint32_t fl = (b4 >> 16) & 0xFF;
            if (rs != NOREM) {
                if (rs == UNASSIGNED_SEQ) {
                    z.rseq(s) = rs = seq;
                    st_bytes4(s, (b4 & 0xFF0000FFu) | (rcl << 8) | ((fl & ~(uint32_t)RF_LRSEQ) << 16));
                } else {
                    ovl_push(s, client);
                    st_bytes4(s, (b4 & 0xFF00FFFFu) | ((fl | RF_OVL) << 16));
                }
            } else {
                h.localLen -= L; /* the row leaves the local view */
                z.rseq(s) = rs = seq;
                cold(s).lrseq = localSeq;
                fl = hasL ? (fl | RF_LRSEQ) : (fl & ~(uint32_t)RF_LRSEQ);
                st_bytes4(s, (b4 & 0xFF0000FFu) | (rcl << 8) | (fl << 16));
                if (dl) { /* removedSegments: only rows this op removes (mergeTree.ts:2669-2672) */
                    dseg(dpos, L);
                    dn++;
                }
                if (rf) { /* savedLocalRefs; segment.localRefs = undefined (mergeTree.ts:2673-2676) */
                    if (refs_move(z.RID(s), INT32_MIN, REF_SAVED, 0)) saved = true;
                    coll_drop(z.RID(s));
                }
            }
            if constexpr (TILED) row_removed(s);
            if (collab) {
                if (rs == UNASSIGNED_SEQ && client == h.localShort)
                    pending_add(s, localSeq, &created);
                else
                    add_lru(s, seq);
            }
        }, dl);
        if (saved) refs_slide(start, refSeq, client);
        if (dl) {
            if (!dh) dhead(dop);
            dtail(dn);
        }
        if (h.collaborating && seq != UNASSIGNED_SEQ) zamboni_soon();
    }

    /* ---- relative positions: MergeTree.posFromRelativePos (mergeTree.ts:1976-1999) ---------- */
    /* The reference's idToSegment map is written when a marker is inserted (mergeTree.ts:1218-1221) and
     * never follows a later annotate of its markerId; the engine finds markers by their current property
     * values. An annotate (or a rewrite) that changes a key slot on a marker records the slot in mkMask,
     * and a lookup by a key slot in that mask is refused (E_UNSUPPORTED) instead of answering by the new
     * value. */
    MT_HD void marker_keys_annotated(int32_t s, const mt_kv* kv, int32_t nkv, bool rewrite) {
        int32_t m = zh->mkMask;
        if (rewrite && (z.flags(s) & RF_PROPS)) {
            typename HT::Cold& c = cold(s);
            for (int32_t k = 0; k < zh->nkeys; k++)
                if (c.pv[k] != 0) m |= 1 << k;
        }
        for (int32_t j = 0; j < nkv; j++) {
            int32_t k = key_slot(kv[j].key);
            if (k >= 0) m |= 1 << k;
        }
        zh->mkMask = m;
    }
    /* The row of the marker whose property `kid` (the marker-id key) holds value `vid` (getMarkerFromId,
     * 1965-1967: the reference's idToSegment map, filled when a marker with an id is inserted): -1 none,
     * -2 more than one (the reference keeps the last one it registered; not modelled) */
    MT_HD int32_t marker_by_id(int32_t kid, int32_t vid) {
        int32_t slot = -1;
        for (int32_t k = 0; k < zh->nkeys; k++)
            if (keys[k] == kid) slot = k;
        if (slot < 0 || (vid & ~MT_VALUE_FALSY) == 0) return -1;
        if (zh->mkMask & (1 << slot)) return -2; /* the id key was annotated on a marker: not modelled */
        int32_t found = -1, n = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t lf = leaf_at(k), c = nch[lf];
            for (int32_t j0 = 0; j0 < c; j0 += W::N) {
                int32_t j = j0 + w.lane();
                bool hit = false;
                if (j < c) {
                    int32_t q = lf * MAXN + j;
                    uint8_t fl = z.flags(q);
                    hit = (fl & RF_MARKER) && (fl & RF_PROPS) &&
                          ((cold(q).pv[slot] ^ vid) & ~MT_VALUE_FALSY) == 0;
                }
                uint64_t m = w.ballot(hit);
                if (m) {
                    n += __builtin_popcountll(m);
                    found = lf * MAXN + j0 + W::ffs(m);
                }
            }
        }
        return n > 1 ? -2 : found;
    }
    /* one relative position (spec units {vid, bits, off lo, off hi}) under (refSeq, client); false if the
     * engine cannot resolve it as the reference would (no marker, or several) */
    MT_HD bool rel_pos(int32_t kid, const uint16_t* u, int32_t refSeq, int32_t client, int32_t* pos) {
        int32_t s = marker_by_id(kid, u[0]);
        if (s < 0) return false;
        int32_t off = (int32_t)((uint32_t)u[2] | ((uint32_t)u[3] << 16));
        int32_t P = position_of(s, refSeq, client);
        if (!(u[1] & 1)) {
            P += z.len(s); /* after the marker: + cachedLength (+ offset) */
            if (u[1] & 2) P += off;
        } else if (u[1] & 2) {
            P -= off;
        }
        *pos = P;
        return true;
    }
    /* getValidOpRange's relative positions of a sequenced record (mt_oplog.h MT_SEG_RELPOS): the record
     * with them resolved, or false */
    MT_HD bool resolve_rel(const mt_op_rec& op, const Pools& p, int32_t client, mt_op_rec* out) {
        const uint16_t* u = p.text + op.text_off + op.text_len;
        *out = op;
        out->seg_kind = (uint8_t)(op.seg_kind & 0x7F);
        if ((u[1] & 1) && !rel_pos(u[0], u + 2, op.ref_seq, client, &out->pos1)) return false;
        if ((u[1] & 2) && !rel_pos(u[0], u + 6, op.ref_seq, client, &out->pos2)) return false;
        return true;
    }

    /* ---- reconnect: Client.regeneratePendingOp (client.ts:706-762, 855-893) -------------- */
    /* findReconnectionPostition (client.ts:675-705): the lengths of the rows before slot s that are
     * inserted (no pending localSeq, or one <= lseq) and not removed (or removed by a local op after lseq) */
    MT_HD int32_t recon_pos(int32_t s, int32_t lseq) {
        int32_t ks = kpos(s / MAXN), js = s & (MAXN - 1), total = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t n = leaf_at(k), c = k == ks ? js : nch[n];
            int32_t v = 0;
            int32_t j = w.lane();
            if (j < c && j < MAXN) {
                int32_t q = n * MAXN + j;
                uint8_t fl = z.flags(q);
                bool ins = !(fl & RF_LSEQ) || cold(q).lseq <= lseq;
                bool live = z.rseq(q) == NOREM || ((fl & RF_LRSEQ) && cold(q).lrseq > lseq);
                if (ins && live) v = z.len(q);
            }
            if constexpr (W::N < MAXN) {
                for (int32_t jj = 1; jj < c; jj++) {
                    int32_t q = n * MAXN + jj;
                    uint8_t fl = z.flags(q);
                    bool ins = !(fl & RF_LSEQ) || cold(q).lseq <= lseq;
                    bool live = z.rseq(q) == NOREM || ((fl & RF_LRSEQ) && cold(q).lrseq > lseq);
                    if (ins && live) v += z.len(q);
                }
            }
            total += w.sum(v);
            if (k == ks) break;
        }
        return total;
    }
    /* resetPendingDeltaToOps (client.ts:708-762) for the head pending group (an op of `kind`): its segments in
     * document order (sorted by ordinal) each get a fresh single-segment group at the tail of the queue with
     * the op's localSeq, and a regenerated op at findReconnectionPostition — except a remove whose removal a
     * remote remove has taken over (localRemovedSeq undefined). With delta events on, the regenerated ops are
     * logged as one MT_DELTA_REGEN event.
     * The group's membership entries are marked in place with their row's document coordinate t
     * (mgid = -(t + 2)) and taken smallest first; a processed entry becomes -1, which the closing compaction
     * drops. Any number of segments; room for their new entries is made before the group leaves the head
     * (a compaction after that would drop its entries). */
    MT_HD void regen(int32_t kind) {
        if (zh->gqN <= 0) {
            fail(E_ASSERT); /* "Segment group not at head of merge tree pending queue" */
            return;
        }
        int32_t hq = zh->gqHead;
        int32_t g0 = d.GQ(hq), lseq0 = d.GQL(hq);
        int32_t mn = zh->memN, cnt = 0;
        for (int32_t b = 0; b < mn; b += W::N) {
            int32_t i = b + w.lane();
            cnt += w.sum(i < mn && d.MGID(i) == g0 ? 1 : 0);
        }
        if (zh->memN + cnt > d.caps.mcap) {
            mem_compact();
            if (zh->memN + cnt > d.caps.mcap) {
                fail(E_CAPACITY);
                return;
            }
        }
        zh->gqHead = gq_wrap(zh->gqHead + 1);
        zh->gqN--;
        mn = zh->memN;
        for (int32_t b = 0; b < mn; b += W::N) { /* mark: each member's coordinate (per lane: its leaf's 8 slots) */
            int32_t i = b + w.lane();
            if (i < mn && d.MGID(i) == g0) {
                int32_t rd = d.MRID(i), lf = z.RLEAF(rd), t = -1;
                for (int32_t j = 0; j < MAXN; j++)
                    if (j < nch[lf] && z.RID(lf * MAXN + j) == rd) t = kpos(lf) * MAXN + j;
                d.MGID(i) = t >= 0 ? -(t + 2) : -1;
                if (t < 0) fail(E_ASSERT);
            }
        }
        w.sync();
        const bool dl = dl_on();
        int32_t nops = 0;
        if (dl) dhead(MT_DELTA_REGEN);
        for (int32_t r = 0; r < cnt && !h.err; r++) {
            int32_t best = -1, bi = -1; /* the marked entry with the smallest coordinate (largest mark) */
            for (int32_t b = 0; b < mn; b += W::N) {
                int32_t i = b + w.lane();
                int32_t v = i < mn ? d.MGID(i) : 0;
                int32_t m = w.max(v <= -2 ? v : INT32_MIN);
                if (m != INT32_MIN && (bi < 0 || m > best)) {
                    best = m;
                    bi = b + W::ffs(w.ballot(v == m));
                }
            }
            if (bi < 0) {
                fail(E_ASSERT);
                break;
            }
            d.MGID(bi) = -1;
            w.sync();
            int32_t s = slot_at(-(best + 2));
            if (s < 0) {
                fail(E_ASSERT);
                break;
            }
            int32_t ng = z.ng(s); /* segment.segmentGroups.dequeue() */
            if (ng < 1) fail(E_ASSERT);
            if (ng > 0) z.ng(s) = (uint8_t)(ng - 1);
            bool op = true;
            if (kind == MT_OP_REMOVE) op = (z.flags(s) & RF_LRSEQ) != 0;
            else if (kind == MT_OP_INSERT && z.seq(s) != UNASSIGNED_SEQ) fail(E_ASSERT);
            else if (kind == MT_OP_ANNOTATE && !(z.flags(s) & RF_PROPS)) fail(E_ASSERT);
            if (!op) continue;
            int32_t pos = recon_pos(s, lseq0);
            if (zh->gqN >= d.caps.gcap) {
                fail(E_CAPACITY);
                break;
            }
            group_push(lseq0); /* { segments: [], localSeq: segmentGroup.localSeq } (client.ts:755-758) */
            row_enqueue_group(s, d.GQ(gq_wrap(zh->gqHead + zh->gqN - 1)));
            if (dl) {
                dput(pos);
                dput(z.len(s));
                dput(kind);
            }
            nops++;
        }
        if (dl) dtail(nops);
        mem_compact();
    }

    /* ---- ack (mergeTree.ts:1926-1953, BaseSegment.ack 486-521) ------------------------ */
    /* ackPendingSegment's per-segment step (mergeTree.ts:1140-1193) for an insert or remove group, one lane per
     * member row (mem: this lane holds a member, rd its row id): the slot lookup, the checks and the row updates
     * in parallel, the LRU entries (addToLRUSet) in member order. Same result as the serial loop in ack(). */
    MT_HD void ack_rows(int32_t kind, int32_t rd, bool mem, int32_t seq, const mt_kv* kv = nullptr, int32_t nkv = 0,
                        bool rewrite = false) {
        int32_t leaf = mem ? (int32_t)z.RLEAF(rd) : 0;
        int32_t gen = mem ? (int32_t)z.RGEN(rd) : 0; /* with the leaf id: the LRU entries need no more reads */
        int32_t c = nch[leaf];
        int32_t s = -1;
        /* an annotate's keys: their slots (the doc's key ids, a lane each, read with the rows) */
        const int32_t l = w.lane();
        int32_t key = kind == MT_OP_ANNOTATE && l < HT::K ? (int32_t)keys[l < HT::K ? l : 0] : -1;
#pragma unroll
        for (int32_t j = 0; j < MAXN; j++) /* the leaf's row ids: one round trip */
            if (mem && j < c && z.RID(leaf * MAXN + j) == (IX)rd) s = leaf * MAXN + j;
        bool bad = mem && s < 0;
        bool ok = mem && s >= 0;
        if (kind == MT_OP_ANNOTATE) { /* ackPendingProperties (segmentPropertiesManager.ts:19-33), a lane per row */
            if (ok && !(z.flags(s) & RF_PROPS)) bad = true;
            typename HT::Cold& cr = d.COLD(ok ? rd : 0);
            if (ok) {
                int32_t ng = z.ng(s);
                if (ng < 1) bad = true;
                if (ng > 0) z.ng(s) = (uint8_t)(ng - 1);
                if (rewrite) cr.prw = (uint8_t)(cr.prw - 1);
            }
            for (int32_t j = 0; j < nkv; j++) {
                int32_t kj = kv[j].key;
                uint64_t m = w.ballot(l < zh->nkeys && key == kj);
                int32_t k = m ? W::ffs(m) : key_slot((uint16_t)kj);
                if (k < 0) return;
                if (!m) key = w.writelane(kj, k, key);
                if (ok && cr.pk[k]) cr.pk[k] = (uint8_t)(cr.pk[k] - 1);
            }
            if (w.ballot(bad)) fail(E_ASSERT);
            w.sync();
            uint64_t om = w.ballot(ok);
            while (om) {
                int32_t q = W::ffs(om);
                om &= om - 1;
                int32_t sq = w.bcast(s, q);
                add_lru_known(sq / MAXN, w.bcast(rd, q), w.bcast(gen, q), nsc[sq / MAXN], seq);
            }
            return;
        }
        if (ok) {
            int32_t ng = z.ng(s);
            if (ng < 1) bad = true;
            if (ng > 0) z.ng(s) = (uint8_t)(ng - 1);
            if (kind == MT_OP_INSERT) {
                if (z.seq(s) != UNASSIGNED_SEQ) bad = true;
                z.seq(s) = seq;
                z.flags(s) &= (uint8_t)~RF_LSEQ;
            } else {
                int32_t rs = z.rseq(s);
                if (rs == NOREM || rs == 0) bad = true;
                z.flags(s) &= (uint8_t)~RF_LRSEQ;
                if (rs == UNASSIGNED_SEQ) z.rseq(s) = seq;
            }
        }
        if (w.ballot(bad)) fail(E_ASSERT);
        w.sync();
        uint64_t om = w.ballot(ok);
        while (om) {
            int32_t l = W::ffs(om);
            om &= om - 1;
            int32_t sl = w.bcast(s, l);
            add_lru_known(sl / MAXN, w.bcast(rd, l), w.bcast(gen, l), nsc[sl / MAXN], seq);
        }
    }
    MT_HD void ack(int32_t kind, const mt_kv* kv, int32_t nkv, bool rewrite, int32_t seq) {
        if (zh->gqN > 0) {
            MT_PROF_SCOPE(PH_ACK);
            int32_t gid = d.GQ(zh->gqHead);
            zh->gqHead = gq_wrap(zh->gqHead + 1);
            zh->gqN--;
            int32_t mn = zh->memN;
            for (int32_t b = 0; b < mn; b += W::N) {
                int32_t i = b + w.lane();
                int32_t rd = i < mn ? d.MRID(i) : 0;
                uint64_t msk = w.ballot(i < mn && d.MGID(i) == gid);
                if constexpr (W::N >= 64) {
                    if (kind == MT_OP_INSERT || kind == MT_OP_REMOVE || (MT_ACKANN_PAR && kind == MT_OP_ANNOTATE)) {
                        /* a lane per member row; LRU entries in member order */
                        if (msk) ack_rows(kind, rd, (msk >> w.lane()) & 1, seq, kv, nkv, rewrite);
                        continue;
                    }
                }
                while (msk) {
                    int32_t l = W::ffs(msk);
                    msk &= msk - 1;
                    int32_t s = slot_of(w.bcast(rd, l), -1);
                    if (s < 0) {
                        fail(E_ASSERT);
                        continue;
                    }
                    /* dequeue the row's head group (groups are acked in FIFO order: this one) */
                    int32_t ng = z.ng(s);
                    if (ng < 1) fail(E_ASSERT);
                    if (ng > 0) z.ng(s) = (uint8_t)(ng - 1);
                    if (kind == MT_OP_ANNOTATE) {
                        if (!(z.flags(s) & RF_PROPS)) fail(E_ASSERT);
                        ack_props(s, kv, nkv, rewrite);
                    } else if (kind == MT_OP_INSERT) {
                        if (z.seq(s) != UNASSIGNED_SEQ) fail(E_ASSERT);
                        z.seq(s) = seq;
                        z.flags(s) &= (uint8_t)~RF_LSEQ;
                    } else if (kind == MT_OP_REMOVE) {
                        if (z.rseq(s) == NOREM || z.rseq(s) == 0) fail(E_ASSERT);
                        z.flags(s) &= (uint8_t)~RF_LRSEQ;
                        if (z.rseq(s) == UNASSIGNED_SEQ) z.rseq(s) = seq;
                    } else {
                        fail(E_ASSERT);
                    }
                    add_lru(s, seq);
                }
            }
            /* drop the acked group's membership entries */
            mem_compact();
        }
        zamboni_soon();
    }

    /* ---- Client.applyMsg (client.ts:797-819) / local edits ---------------------------- */
    MT_HD void apply(const mt_op_rec& op, const Pools& p) {
        MT_PROF_SCOPE(PH_APPLY);
        if (h.err) return;
        int32_t at = h.opsDone;
        MT_PROF_COUNT(PH_C_HEAPN, h.heapN);
        apply_record(op, p);
        run_zamboni();
        if (h.err) zh->errOp = at;
    }
    /* One record. Every path that edits the tree ends in the one call site of insert_segments /
     * mark_range_removed / annotate_range below (each is inlined once). */
    MT_HD void apply_record(const mt_op_rec& op, const Pools& p) {
        int32_t kind = op.kind & MT_OP_KIND_MASK;
        if constexpr (DL) {
            if (Doc<HT>::has_fx(d.caps)) { /* delta events: this record's seq; none while a snapshot loads */
                DState* st = d.dstate();
                st->seq = (op.kind & MT_OPF_LOCAL) ? UNASSIGNED_SEQ : op.seq;
                st->on = (op.kind & MT_OPF_LOCAL) || kind < MT_OP_RELOAD;
            }
        }
        const mt_kv* kv = 0;
        int32_t nkv = 0;
        bool rw = false;
        int32_t comb = MT_COMBINE_NONE;
        if (op.props && kind == MT_OP_ANNOTATE) {
            const mt_props_rec& pr = p.props[op.props - 1];
            kv = p.kv + pr.kv_off;
            nkv = pr.nkv;
            comb = pr.combining;
            rw = comb == MT_COMBINE_REWRITE;
        }
        if ((op.seg_kind & MT_SEG_RELPOS) && (op.kind & (MT_OPF_LOCAL | MT_OPF_TREE) || kind > MT_OP_ANNOTATE)) {
            fail(E_UNSUPPORTED); /* relative positions: sequenced op records only (mt_oplog.h) */
            h.opsDone++;
            return;
        }
        if (kind == MT_OP_REF) { /* a local reference (mt_oplog.h): the client-feature build keeps them */
            if constexpr (DL) {
                if ((op.kind & MT_OPF_LOCAL) && op.seg_kind == MT_REF_REMOVE)
                    remove_ref(op.pos1);
                else if (op.kind & MT_OPF_LOCAL)
                    add_ref(op.pos1, op.pos2);
            } else {
                fail(E_UNSUPPORTED);
            }
            h.opsDone++;
            return;
        }
        /* the sender's short id of a sequenced or MergeTree-level record: in the recycling profiles registered at
         * one call site (its slot allocation and recycling, get_or_add_short, is inlined once); the small profiles
         * keep the call at each use, which their register allocation prefers (A/B) */
        const bool tree = (op.kind & MT_OPF_TREE) != 0;
        const bool seqd = !(op.kind & MT_OPF_LOCAL) && (tree || kind < MT_OP_RELOAD);
        const int32_t sc =
            RECLAIM && seqd && !(tree && op.client == MT_CLIENT_LOCAL) ? get_or_add_short(op.client) : -1;
        /* the edit the record makes, if any */
        mt_op_rec o = op;
        bool edit = false, remote = false, grouped = false;
        int32_t eref = 0, ecli = 0, eseq = 0, epre = 0, eat = -1;
        uint8_t eprc = 0;
        if (kind >= MT_OP_RELOAD && !(op.kind & MT_OPF_LOCAL) && !(op.kind & MT_OPF_TREE)) {
            if constexpr (LOAD)
                edit = apply_load(op, p, &o, &ecli, &epre, &eprc); /* snapshot load (mt_oplog.h) */
            else
                fail(E_UNSUPPORTED); /* the engine routes such batches to the full build */
            eref = UNIVERSAL_SEQ;
            eseq = op.seq;
        } else if (op.kind & MT_OPF_TREE) { /* MergeTree-level call with explicit (refSeq, clientId, seq) */
            ecli = RECLAIM ? sc : op.client == MT_CLIENT_LOCAL ? -1 : get_or_add_short(op.client);
            if (op.client == MT_CLIENT_NONCOLLAB || (op.kind & MT_OPF_LOCAL) || kind > MT_OP_ANNOTATE ||
                (kind == MT_OP_INSERT && op.seg_kind != MT_SEG_MARKER && op.text_len == 0)) {
                fail(E_UNSUPPORTED);
            } else {
                edit = true;
                eref = op.ref_seq;
                eseq = op.seq;
            }
        } else if (op.kind & MT_OPF_LOCAL) {
            ecli = h.collaborating ? h.localShort : -1;
            eref = h.currentSeq;
            eseq = h.collaborating ? UNASSIGNED_SEQ : UNIVERSAL_SEQ;
            /* getValidOpRange (client.ts:486-548) */
            int32_t length = length_local();
            int32_t start = op.pos1, end = op.pos2;
            bool bad = start < 0 || start > length || (start == length && kind != MT_OP_INSERT);
            if (kind != MT_OP_INSERT && end <= start) bad = true;
            if (kind == MT_OP_NOOP) { /* PermutationVector.getAllocatedHandle(pos1), or walkSegments' split (mt_oplog.h) */
                if constexpr (DL) {
                    if (op.seg_kind == MT_NOOP_SPLIT)
                        split_range(op.pos1, op.pos2);
                    else if (op.seg_kind == MT_NOOP_HTLOAD)
                        ht_load(op, p);
                    else
                        alloc_handle(op.pos1);
                } else {
                    fail(E_UNSUPPORTED);
                }
            } else if (kind == MT_OP_INSERT && (op.kind & MT_OPF_ATREF)) { /* pos1 is a reference, not a position */
                if constexpr (DL) {
                    edit = insert_at_ref(op, &eat);
                    ecli = h.localShort;
                    eseq = UNASSIGNED_SEQ;
                } else {
                    fail(E_UNSUPPORTED); /* the client-feature build (caps.rcap > 0) replays these */
                }
            } else if (op.kind & MT_OPF_REGEN) { /* regeneratePendingOp of the head pending op (mt_oplog.h) */
                if constexpr (DL)
                    regen(kind);
                else
                    fail(E_UNSUPPORTED);
            } else if (bad) { /* rejected: no effect (the reference logs InvalidOpRange and returns undefined) */
            } else if (kind == MT_OP_INSERT && op.seg_kind != MT_SEG_MARKER && op.text_len == 0) {
                return; /* insertSegmentLocal of an empty segment */
            } else {
                edit = kind <= MT_OP_ANNOTATE;
                /* a local consensus annotate: its ack calls updateConsensusProperty, which needs the marker-relative
                 * position and the pending-consensus callback of annotateMarkerNotifyConsensus (client.ts:982-989,
                 * 248-274); neither is modelled, and a plain one throws there in the reference */
                if (comb == MT_COMBINE_CONSENSUS) fail(E_UNSUPPORTED);
            }
        } else {
            remote = true;
            if constexpr (!RECLAIM) get_or_add_short(op.client);
            grouped = (op.kind & MT_OPF_GROUPED) != 0; /* a group member before the last (mt_oplog.h) */
            if (!grouped) zh->seqOps++; /* one sequenced message per group */
            if (grouped) {
            } else if constexpr (TILED) /* BASELINE.md tile formula (round 6: HBM-resident bytes only), in 16-byte
                                    units: 32 B per window row, 640 B for the target chunk's leaves + leaf line; the
                                    chunk summaries and the window set's entries are LDS-resident during a replay */
                zh->sumR += (32 * z.tl.wN + 640) / 16;
            else
                zh->sumR += h.nrows;
            if (kind != MT_OP_NOOP) {
                if ((int32_t)op.client == h.localLong) {
                    ack(kind, kv, nkv, rw, op.seq);
                } else {
                    ecli = RECLAIM ? sc : get_or_add_short(op.client);
                    eref = op.ref_seq;
                    eseq = op.seq;
                    edit = true;
                    if (op.seg_kind & MT_SEG_RELPOS) { /* relative positions (mt_oplog.h) */
                        if constexpr (DL)
                            edit = resolve_rel(op, p, ecli, &o);
                        else
                            edit = false;
                        if (!edit) fail(E_UNSUPPORTED);
                    }
                }
            }
        }
        if (edit) {
            if (kind == MT_OP_REMOVE || kind == MT_OP_ANNOTATE)
                range_edit(kind == MT_OP_REMOVE, o.pos1, o.pos2, kv, nkv, comb, eref, ecli, eseq);
            else
                insert_segments(o, p, eref, ecli, eseq, epre, eprc, eat);
            if (remote) {
                if (!(h.currentSeq < op.seq)) fail(E_ASSERT);
                if (!(h.minSeq <= op.min_seq)) fail(E_ASSERT);
            }
        }
        if (remote && !grouped) { /* a group's seq update waits for its last member (client.ts:782-790) */
            /* updateSeqNumbers (client.ts:821-828) */
            if (!(h.currentSeq <= op.seq)) fail(E_ASSERT);
            h.currentSeq = op.seq;
            if (!(op.min_seq <= op.seq)) fail(E_ASSERT);
            set_min_seq(op.min_seq);
        }
        h.opsDone++;
    }
    /* high-water mark of row slots in use (stats), noted whenever the leaf count grows */
    MT_HD void note_leaves() {
        if (h.nleaf * MAXN > zh->hwSlots) zh->hwSlots = h.nleaf * MAXN;
    }
    /* ---- snapshot load (SnapshotLoader, snapshotLoader.ts:86-228; records in mt_oplog.h) ------- */
    /* the fields of a loaded segment (SnapshotLoader.specToSegment, snapshotLoader.ts:96-126) on an
     * already placed row s whose text / props the insert path has set */
    MT_HD int32_t loader_client(uint16_t longId) {
        return longId == MT_CLIENT_NONCOLLAB ? -1 : get_or_add_short(longId); /* NonCollab: never a real client */
    }
    /* reloadFromSegments (mergeTree.ts:1229-1284) of records [cur, cur + n): leaf blocks of 7 rows in
     * order, then interior levels of 7 blocks, bottom-up (the single block of a level is the root) */
    MT_HD void reload(const Pools& p, int32_t n) {
        if (h.collaborating || h.nrows != 0 || h.nleaf != 1 || cur + n > p.nops) {
            fail(E_ASSERT); /* assert(!collaborating) (1231), on an empty replica, whole header at hand */
            return;
        }
        constexpr int32_t K = MAXN - 1;
        int32_t leaf = leaf_at(0), prevLeaf = -1;
        for (int32_t i = 0; i < n; i++) {
            const mt_op_rec op = p.ops[cur + i];
            if ((op.kind & MT_OP_KIND_MASK) != MT_OP_RELOAD) {
                fail(E_ASSERT);
                return;
            }
            int32_t j = i % K;
            if (j == 0 && i > 0) {
                prevLeaf = leaf;
                leaf = alloc_node(0);
                if (leaf < 0) return;
                lorder_insert_after(prevLeaf, leaf);
            }
            if (!place_loaded(op, p, leaf * MAXN + j)) return;
            nch[leaf] = (int8_t)(j + 1);
        }
        if constexpr (TILED)
            for (int32_t k = 0; kvalid(k); k = knext(k)) leaf_restat(leaf_at(k));
        /* interior levels; the previous level's nodes in order go through the (empty) heap arrays */
        int32_t cnt = 0;
        IX* hrd = z.hrid; /* the image's own heap array (N + 64 entries): an LDS heap may be smaller */
        for (int32_t k = 0; kvalid(k); k = knext(k)) hrd[cnt++] = (IX)leaf_at(k);
        int8_t lvl = 1;
        while (cnt > 1) {
            int32_t m = (cnt + K - 1) / K;
            for (int32_t bi = 0; bi < m; bi++) {
                int32_t nb = alloc_node(lvl);
                if (nb < 0) return;
                int32_t c = 0;
                for (int32_t i = bi * K; i < cnt && c < K; i++, c++) {
                    int32_t ch = hrd[i];
                    z.KIDS(nb * MAXN + c) = (IX)ch;
                    npar[ch] = (IX)nb;
                }
                nch[nb] = (int8_t)c;
                hrd[bi] = (IX)nb; /* bi <= i: written after its block's children were read */
            }
            cnt = m;
            lvl++;
        }
        zh->root = hrd[0];
        npar[zh->root] = -1;
    }
    /* one loaded segment into slot s (a fresh row): text / marker / permutation, props, merge info */
    MT_HD bool place_loaded(const mt_op_rec& op, const Pools& p, int32_t s) {
        bool marker = op.seg_kind == MT_SEG_MARKER, perm = op.seg_kind == MT_SEG_PERM;
        const bool run = op.seg_kind == MT_SEG_RUN; /* a loaded SubSequence ({items} spec) */
        if (run) zh->ndv |= DV_RUN;
        int32_t L = seg_len(op);
        if (L <= 0) {
            fail(E_UNSUPPORTED); /* a snapshot holds no empty segments */
            return false;
        }
        int32_t off = 0;
        if (!marker && !perm) {
            off = arena_alloc(L);
            if (off < 0) return false;
        }
        z.RID(s) = (IX)alloc_rid();
        cold(s).gc = 0;
        z.len(s) = L;
        z.seq(s) = op.seq;
        int32_t cl = loader_client(op.client);
        z.cli(s) = (uint8_t)(cl < 0 ? LOCAL_CLIENT : cl);
        z.rseq(s) = NOREM;
        z.rcli(s) = 0;
        if (op.ref_seq > 0) { /* removed above the snapshot's MSN */
            int32_t rc = loader_client((uint16_t)op.min_seq);
            z.rseq(s) = op.ref_seq;
            z.rcli(s) = (uint8_t)(rc < 0 ? LOCAL_CLIENT : rc);
        }
        z.ng(s) = 0;
        cold(s).lseq = 0;
        cold(s).lrseq = 0;
        cold(s).ovl = 0;
        cold(s).ovx = 0;
        z.RLEAF(z.RID(s)) = (IX)(s / MAXN);
        int32_t fl = (marker ? RF_MARKER : 0) | (perm ? RF_PERM : 0);
        if (marker) {
            cold(s).toff = (uint32_t)op.pos2;
        } else if (perm) {
            cold(s).toff = op.text_off; /* a loaded PermutationSegment's start ([length, start] spec): 0 = unallocated */
        } else {
            cold(s).toff = (uint32_t)off;
            int32_t last = arena_copy(arena_base(zh->arenaSide) + off, p.text + op.text_off, L);
            fl |= RF_NLK | (last == '\n' && !run ? RF_NL : 0);
        }
        z.flags(s) = (uint8_t)fl;
        if (op.props) {
            const mt_props_rec& pr = p.props[op.props - 1];
            add_props(s, p.kv + pr.kv_off, pr.nkv, pr.combining == MT_COMBINE_REWRITE ? MT_COMBINE_REWRITE : MT_COMBINE_NONE, 0,
                      false);
        }
        if constexpr (TILED) z.tl.xf[s] = 0;
        h.nrows++;
        if (z.rseq(s) == NOREM) h.localLen += L;
        if constexpr (TILED) row_enter(s);
        return true;
    }
    /* a snapshot-load record; true if it is a body segment to insert (the caller's insert: *ins at the position
     * loadBody computes, client *cl, removedSeq *pre by client *prc) */
    MT_HD bool apply_load(const mt_op_rec& op, const Pools& p, mt_op_rec* ins, int32_t* cl, int32_t* pre,
                          uint8_t* prc) {
        int32_t kind = op.kind & MT_OP_KIND_MASK;
        if (kind == MT_OP_RELOAD) {
            if (h.nrows == 0 && !h.collaborating) reload(p, op.pos1); /* the first of the header's records */
        } else if (kind == MT_OP_COLLAB) {
            start_collab(op.client, op.min_seq, op.seq);
        } else { /* MT_OP_APPEND: loadBody's insertSegments(root.cachedLength, segs, 0, client, seq) */
            /* a batch of segments (one insertSegments call, blockInsert 2226-2256) starts at the local
             * length; its later members (GROUPED) go at the previous position + the previous
             * segment's whole length, removed or not */
            *ins = op;
            ins->pos1 = (op.kind & MT_OPF_GROUPED) ? zh->loadPos : h.localLen;
            zh->loadPos = ins->pos1 + seg_len(op);
            *cl = loader_client(op.client);
            int32_t rc = op.ref_seq > 0 ? loader_client((uint16_t)op.min_seq) : 0;
            if (h.err) return false;
            *pre = op.ref_seq > 0 ? op.ref_seq : 0;
            *prc = (uint8_t)(rc < 0 ? LOCAL_CLIENT : rc);
            return true;
        }
        return false;
    }

    /* Client.getLength(): the local view's length, kept incrementally like root.cachedLength */
    MT_HD int32_t length_local() const { return h.localLen; }

    /* ---- reads: text (MergeTreeTextHelper.getText, textSegment.ts:154-275) ------------ */
    /* getText(refSeq, clientId, placeholder, start, end): mapRange over [start, end) (getValidRange 174-186:
     * start undefined = 0, end undefined = getLength; pass TEXT_RANGE_DEFAULT) visits every row with a
     * non-zero perspective length v at position p where start < p + v and end > p (nodeMap). gatherText
     * (188-271): a text row adds text.substring(start - p, end - p) with JavaScript's substring rules (the
     * whole text when start <= p and end >= p + v); any other row adds `placeholder` v times when the
     * placeholder is non-empty ("*", which prints Marker.toString(), is rejected by the callers). Writes at
     * most cap units; returns the text length. */
    static constexpr int32_t TEXT_RANGE_DEFAULT = INT32_MIN;
    MT_HD static void text_piece(int32_t v, int32_t rs, int32_t re, int32_t* a, int32_t* b) {
        if (rs <= 0 && re >= v) {
            *a = 0, *b = v;
            return;
        }
        int32_t x = rs < 0 ? 0 : rs, y = re >= v ? v : re; /* substring(x, y): clamp to [0, v], then order */
        x = x < 0 ? 0 : (x > v ? v : x);
        y = y < 0 ? 0 : (y > v ? v : y);
        *a = x < y ? x : y, *b = x < y ? y : x;
    }
    static constexpr int64_t PH_RUN_MAX = 1 << 24;
    MT_HD int64_t get_text(int32_t refSeq, int32_t client, uint16_t* out, int64_t cap) {
        return get_text_range(refSeq, client, 0, INT32_MAX, nullptr, 0, out, cap);
    }
    MT_HD int64_t get_text_range(int32_t refSeq, int32_t client, int32_t start, int32_t end, const uint16_t* ph,
                                 int32_t pl, uint16_t* out, int64_t cap) {
        if (start == TEXT_RANGE_DEFAULT) start = 0;
        if (end == TEXT_RANGE_DEFAULT) end = length(refSeq, client);
        if (start < 0) start = 0; /* the same rows and pieces as 0 (positions are >= 0); no overflow below */
        if (end < -1) end = -1;   /* the same as -1: no row */
        int64_t n = 0;
        int32_t P = 0; /* position of the pass's first row */
        const uint16_t* base = arena_base(zh->arenaSide);
        const bool runD = run_doc(); /* SubSequence rows are not TextSegments: gatherText gives their placeholders */
        if constexpr (W::N >= MAXN * MAXN) {
            /* 8 leaves x 8 slots per pass of the wave: each lane's row length under the perspective, one
             * scan for the positions and one for the output offsets, and every lane copies its own piece */
            int32_t k = 0;
            bool more = kvalid(0);
            while (more) {
                int32_t q = w.lane(), li = q >> 3, j = q & (MAXN - 1), leaf = -1;
                for (int32_t i = 0; i < MAXN && more; i++) {
                    int32_t lf = leaf_at(k);
                    if (i == li) leaf = lf;
                    k = knext(k);
                    more = kvalid(k);
                }
                int32_t v = 0, s = -1;
                if (leaf >= 0 && j < nch[leaf]) {
                    s = leaf * MAXN + j;
                    v = vis(s, refSeq, client);
                }
                int32_t vtot;
                int32_t p = P + w.excl_scan(v, &vtot);
                bool hit = v > 0 && start < p + v && end > p;
                bool text = s >= 0 && !(z.flags(s) & RF_NOTEXT) && !runD;
                int32_t a = 0, b = 0;
                if (hit && text) text_piece(v, start - p, end - p, &a, &b);
                /* a placeholder run longer than 2^24 units (a merged PermutationSegment of millions of rows
                 * at a long placeholder) is rejected rather than overflowing the int32 output scan */
                if (w.ballot(hit && !text && (int64_t)pl * v > PH_RUN_MAX)) return -E_UNSUPPORTED;
                int32_t ol = !hit ? 0 : text ? b - a : pl * v;
                int32_t tot;
                int64_t o = n + w.excl_scan(ol, &tot);
                if (out && ol > 0 && o < cap) {
                    int64_t m = ol < cap - o ? ol : cap - o;
                    if (text) {
                        const uint16_t* src = base + cold(s).toff + a;
                        for (int64_t u = 0; u < m; u++) out[o + u] = src[u];
                    } else {
                        for (int64_t u = 0; u < m; u++) out[o + u] = ph[u % pl];
                    }
                }
                n += tot;
                P += vtot;
            }
            w.sync();
            return n;
        }
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
            int32_t lf = leaf_at(k), c = nch[lf];
            for (int32_t j = 0; j < c; j++) {
                int32_t s = lf * MAXN + j;
                int32_t v = vis(s, refSeq, client), p = P;
                P += v;
                if (v <= 0 || !(start < p + v && end > p)) continue;
                if ((z.flags(s) & RF_NOTEXT) || runD) {
                    if ((int64_t)pl * v > PH_RUN_MAX) return -E_UNSUPPORTED;
                    for (int32_t u = 0; u < pl * v; u++, n++)
                        if (out && n < cap) out[n] = ph[u % pl];
                    continue;
                }
                int32_t a, b;
                text_piece(v, start - p, end - p, &a, &b);
                if (out) {
                    int64_t m = b - a;
                    if (n + m > cap) m = cap - n > 0 ? cap - n : 0;
                    arena_copy(out + n, base + cold(s).toff + a, (int32_t)m);
                }
                n += b - a;
            }
        }
        return n;
    }

    /* SharedSequence.getItems(start, end) (sequence sharedSequence.ts:150-183) in the local view: walkSegments(start,
     * end) visits the rows of positive length intersecting [start, end) and pushes every item of each SubSequence row
     * (markers and permutation rows push none); then the items before `start` in the first such row are spliced off
     * (start - getPosition(first)) and the array cut to end - start (end = MT_TEXT_DEFAULT: undefined, no cut; end <=
     * start: none). So a marker inside the range shifts the cut as it does in the reference. Item ids (the units) into
     * out (cap), the count returned. */
    MT_HD int64_t get_items(int32_t start, int32_t end, uint16_t* out, int64_t cap) {
        const bool noEnd = end == TEXT_RANGE_DEFAULT;
        if ((!noEnd && end <= start) || !run_doc()) return 0; /* TextSegments are no SubSequence: none pushed */
        const int32_t refSeq = h.currentSeq, client = h.localShort;
        const int32_t e = noEnd ? INT32_MAX : end;
        const uint16_t* base = arena_base(zh->arenaSide);
        int64_t lo = -1, hi = INT64_MAX, n = 0; /* the kept window of the pushed items, once the first row is known */
        int64_t I = 0;                          /* items pushed before the pass's first row */
        int32_t P = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) { /* rolled: a read, not a replay path */
            int32_t lf = leaf_at(k), c = nch[lf];
            for (int32_t j = 0; j < c; j++) {
                int32_t s = lf * MAXN + j;
                int32_t v = vis(s, refSeq, client), p = P;
                P += v;
                if (v <= 0 || !(start < p + v && e > p) || (z.flags(s) & RF_NOTEXT)) continue;
                if (lo < 0) { /* the first SubSequence row: splice(0, start - getPosition(it)) */
                    lo = start - p > 0 ? start - p : 0;
                    if (!noEnd) hi = lo + (int64_t)(end - start);
                }
                const uint16_t* src = base + cold(s).toff;
                for (int32_t u = 0; u < v; u++, I++)
                    if (I >= lo && I < hi) {
                        if (out && n < cap) out[n] = src[u];
                        n++;
                    }
            }
        }
        w.sync();
        return n;
    }

    /* ---- reads: getContainingSegment / getPosition (mergeTree.ts:1656-1667, 1619-1636) ---- */
    /* The row holding position pos under the perspective (searchBlock descends to the first child
     * with pos < length: the first row with P <= pos < P + vis); *off = pos - P. -1 if none. */
    MT_HD int32_t containing(int32_t pos, int32_t refSeq, int32_t client, int32_t* off) {
        if (pos < 0) return -1;
        int32_t P = 0, s = -1;
        int32_t t = find_reach(pos + 1, refSeq, client, &P, &s);
        if (t < 0) return -1;
        *off = pos - P;
        return s;
    }
    /* getPosition: the summed perspective lengths of every row before slot s in document order */
    /* the index of slot s in walkAllSegments order (the canonical dump's record index): every row before it */
    MT_HD int32_t ordinal_of(int32_t s) {
        int32_t ks = kpos(s / MAXN), total = s & (MAXN - 1);
        for (int32_t k = 0; kvalid(k) && k != ks; k = knext(k)) total += nch[leaf_at(k)];
        return total;
    }
    MT_HD int32_t position_of(int32_t s, int32_t refSeq, int32_t client) {
        int32_t k0 = kpos(s / MAXN), j0 = s & (MAXN - 1);
        int32_t total = 0;
        if constexpr (TILED) {
            if (tiles_cover(refSeq, client)) { /* chunks before, leaves before in the chunk, rows before */
                auto& t = z.tl;
                win_pass(refSeq, client);
                int32_t cp = k0 >> 6, li = k0 & 63, c = tcord[cp];
                for (int32_t b = 0; b < cp; b += W::N) {
                    int32_t p = b + w.lane();
                    total += w.sum(p < cp ? tcst[p] + cdel[p] : 0);
                }
                for (int32_t b = 0; b < li; b += W::N) {
                    int32_t l = b + w.lane();
                    total += w.sum(l < li ? t.cls[c][l] : 0);
                }
                int32_t nw = t.wN;
                for (int32_t b = 0; b < nw; b += W::N) {
                    int32_t i = b + w.lane();
                    total += w.sum(i < nw && wcp[i] == cp && wlx[i] < li ? wvs[i] : 0);
                }
                win_clear();
                int32_t n = leaf_at(k0);
                for (int32_t j = 0; j < j0; j++) total += vis(n * MAXN + j, refSeq, client);
                return total;
            }
        }
        if constexpr (TILED) { /* a remote perspective below minSeq: walk every leaf */
            for (int32_t k = 0; kvalid(k); k = knext(k)) {
                int32_t n = leaf_at(k), c = nch[n];
                for (int32_t j = 0; j < c; j++) {
                    if (k == k0 && j == j0) return total;
                    total += vis(n * MAXN + j, refSeq, client);
                }
            }
            return total;
        }
        /* flat profiles: the perspective scan over the slots before s (a quad per lane) */
        int32_t t0 = k0 * MAXN + j0;
        for (int32_t b = 0; b < t0; b += 4 * W::N) {
            int32_t tq = b + 4 * w.lane();
            int32_t v[4];
            quad_vis(quad_slot(tq), refSeq, client, v);
            int32_t x = 0;
            for (int q = 0; q < 4; q++)
                if (tq + q < t0) x += v[q];
            total += w.sum(x);
        }
        return total;
    }

    /* ---- canonical dump (include/mt_oplog.h) ------------------------------------------- */
    /* byte sink: writes into a buffer (if any) and/or folds FNV-1a-64 */
    struct Sink {
        uint8_t* out;
        int64_t cap, n;
        uint64_t h;
        bool hash;
    };
    MT_HD static void put_bytes(Sink* k, const void* src, int64_t len) {
        const uint8_t* p = (const uint8_t*)src;
        if (k->out && k->n + len <= k->cap)
            for (int64_t i = 0; i < len; i++) k->out[k->n + i] = p[i];
        if (k->hash)
            for (int64_t i = 0; i < len; i++) {
                k->h ^= p[i];
                k->h *= MT_FNV_PRIME;
            }
        k->n += len;
    }
    MT_HD int32_t long_of(uint8_t sh) const { return sh == LOCAL_CLIENT ? -1 : (int32_t)s2l[sh]; }
    /* the long ids of the client / removedClient of the row in slot s (a retired byte: the retired-client table) */
    MT_HD int32_t long_of_cli(int32_t s) const {
        uint8_t b = z.cli(s);
        return b == RETIRED_CLIENT ? (int32_t)(d.RCL(z.RID(s)) & 0xFFFF) : long_of(b);
    }
    MT_HD int32_t long_of_rcli(int32_t s) const {
        uint8_t b = z.rcli(s);
        return b == RETIRED_CLIENT ? (int32_t)(d.RCL(z.RID(s)) >> 16) : long_of(b);
    }
    /* Serial dump (only lane 0 writes the buffer); returns the byte count. */
    MT_HD int64_t dump(uint8_t* out, int64_t cap) {
        Sink k = {w.lane() == 0 ? out : 0, cap, 0, MT_FNV_OFFSET, false};
        dump_to(&k);
        return k.n;
    }
    MT_HD uint64_t digest() {
        Sink k = {0, 0, 0, MT_FNV_OFFSET, true};
        dump_to(&k);
        return k.h;
    }
    MT_HD void dump_to(Sink* o) {
        int32_t nsegs = 0;
        for (int32_t k = 0; kvalid(k); k = knext(k)) nsegs += nch[leaf_at(k)];
        int32_t hdr[6] = {h.currentSeq, h.minSeq, zh->localSeq, length_local(), nsegs, h.nleaf};
        put_bytes(o, hdr, sizeof(hdr));
        const uint16_t* base = arena_base(zh->arenaSide);
        const bool runD = run_doc(); /* text-bearing rows are SubSequence rows (kind MT_SEG_RUN) */
        int32_t ordinal = -1;
        for (int32_t k = 0; kvalid(k); k = knext(k)) {
          ordinal++;
          int32_t lfn = leaf_at(k), lc = nch[lfn];
          for (int32_t jj = 0; jj < lc; jj++) {
            int32_t s = lfn * MAXN + jj;
            uint8_t fl = z.flags(s);
            bool rem = z.rseq(s) != NOREM;
            int nov = ovl_count(s);
            int np = 0;
            if (fl & RF_PROPS)
                for (int k = 0; k < HT::K; k++)
                    if (cold(s).pv[k]) np++;
            bool hnd = (fl & RF_PERM) && cold(s).toff != 0; /* an allocated PermutationSegment start */
            uint8_t b4[4] = {(uint8_t)((fl & RF_MARKER) ? MT_SEG_MARKER : (fl & RF_PERM) ? MT_SEG_PERM : runD ? MT_SEG_RUN : MT_SEG_TEXT),
                             (uint8_t)(((fl & RF_PROPS) ? MT_DF_HAS_PROPS : 0) | (rem ? MT_DF_REMOVED : 0) |
                                       ((fl & RF_LSEQ) ? MT_DF_LSEQ : 0) | ((fl & RF_LRSEQ) ? MT_DF_LRSEQ : 0) |
                                       (hnd ? MT_DF_HANDLE : 0)),
                             (uint8_t)nov, z.ng(s)};
            put_bytes(o, b4, 4);
            int32_t f[8] = {z.len(s),
                            z.seq(s),
                            long_of_cli(s),
                            rem ? z.rseq(s) : 0,
                            rem ? long_of_rcli(s) : 0,
                            (fl & RF_LSEQ) ? cold(s).lseq : 0,
                            (fl & RF_LRSEQ) ? cold(s).lrseq : 0,
                            ordinal};
            put_bytes(o, f, sizeof(f));
            for (int k = 0; k < nov; k++) {
                int32_t lo = long_of((uint8_t)ovl_at(s, k));
                put_bytes(o, &lo, 4);
            }
            uint16_t h2[2] = {(uint16_t)np, (uint16_t)((fl & RF_MARKER) ? cold(s).toff : 0)};
            put_bytes(o, h2, 4);
            /* props sorted by global key id */
            int32_t last = -1;
            for (int q = 0; q < np; q++) {
                int32_t best = -1, bk = 0x7fffffff;
                for (int k = 0; k < HT::K; k++) {
                    int32_t key = keys[k];
                    if (cold(s).pv[k] && key > last && key < bk) {
                        bk = key;
                        best = k;
                    }
                }
                uint16_t v = cold(s).pv[best];
                if (v >= MT_VALUE_DERIVED && v < MT_VALUE_NAN) v = v < MT_VALUE_CONS0 ? MT_VALUE_STRCAT0 : MT_VALUE_CONS0;
                uint16_t kv2[2] = {(uint16_t)bk, v};
                put_bytes(o, kv2, 4);
                last = bk;
            }
            if (zh->ndv & 0xFFFF) { /* derived values' contents, in pair order (mt_oplog.h) */
                last = -1;
                for (int q = 0; q < np; q++) {
                    int32_t best = -1, bk = 0x7fffffff;
                    for (int k = 0; k < HT::K; k++) {
                        int32_t key = keys[k];
                        if (cold(s).pv[k] && key > last && key < bk) {
                            bk = key;
                            best = k;
                        }
                    }
                    last = bk;
                    int32_t v = cold(s).pv[best];
                    if (v < MT_VALUE_DERIVED || v >= MT_VALUE_NAN) continue;
                    int32_t ab[2];
                    if (v < MT_VALUE_CONS0) {
                        int32_t x = z.dvs[v - MT_VALUE_STRCAT0];
                        ab[0] = x & 0xFFFF, ab[1] = (int32_t)((uint32_t)x >> 16);
                    } else {
                        ab[0] = z.dvc[v - MT_VALUE_CONS0], ab[1] = 0;
                    }
                    put_bytes(o, ab, 8);
                }
            }
            if (hnd) {
                int32_t st = (int32_t)cold(s).toff;
                put_bytes(o, &st, 4);
            }
            if (!(fl & RF_NOTEXT)) put_bytes(o, base + cold(s).toff, 2 * (int64_t)z.len(s));
          }
        }
    }
    MT_HD static uint64_t fnv(const uint8_t* p, int64_t n) {
        uint64_t h = MT_FNV_OFFSET;
        for (int64_t i = 0; i < n; i++) {
            h ^= p[i];
            h *= MT_FNV_PRIME;
        }
        return h;
    }

    /* Apply a whole event stream, one record at a time. */
    MT_HD void replay(const Pools& p) {
        static_assert(sizeof(mt_op_rec) == 32, "op record is 8 dwords");
        vk = p.vkind;
        nvk = p.nvk;
        hmax = INT32_MIN; /* the heap's largest maxSeq */
        for (int32_t b = 0; b < h.heapN; b += W::N) {
            int32_t i = b + w.lane();
            int32_t m = w.max(i < h.heapN ? hsq[i] : INT32_MIN);
            if (m > hmax) hmax = m;
        }
        /* One record per event, read uniformly when its turn comes: nothing is held across apply(). (Reading a
         * wave's worth of records at once and broadcasting them kept 8 registers live through every event,
         * which the config-3 kernel spilled to scratch: 333.97 -> 344.63M ops/s without it, r04zr.) */
        for (int64_t i = 0; i < p.nops; i++) {
            const int32_t* src = (const int32_t*)&p.ops[i];
            I4 a0 = ld4(src), a1 = ld4(src + 4);
            int32_t u[8];
            for (int q = 0; q < 4; q++) {
                u[q] = w.uniform(a0.x[q]);
                u[4 + q] = w.uniform(a1.x[q]);
            }
            mt_op_rec op;
            __builtin_memcpy(&op, u, sizeof(op));
            cur = i;
            if constexpr (TILED)
                if (pfcur) *(volatile int32_t*)pfcur = (int32_t)cur; /* the prefetch helpers run ahead of it */
            apply(op, p);
            if (h.err) return;
        }
    }
};

} /* namespace mt */
