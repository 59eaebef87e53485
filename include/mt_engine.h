/*
 * mt_engine.h — C ABI of the MI355X merge-tree replay engine (libmtreplay.so).
 *
 * The reference has no FFI for this path: its boundary is the TypeScript module
 * @fluidframework/merge-tree (packages/dds/merge-tree/src/index.ts:6-22), whose `Client` is
 * called by SharedSegmentSequence (packages/dds/sequence/src/sequence.ts:579-616) and
 * SharedMatrix/PermutationVector (packages/dds/matrix/src/matrix.ts:568-578). The entry points
 * below are what a Node-API addon binding that module's hot path would call;
 * each cites the reference member it replaces. One engine = a batch of documents resident in
 * one GPU's HBM, one replica per document. All calls are synchronous unless noted; errors
 * are returned as MT_E_* status codes (no exceptions cross the ABI) and per-document replay
 * errors are latched and reported by mt_engine_errors (the reference throws synchronously).
 */
#ifndef MT_ENGINE_H
#define MT_ENGINE_H
#include <stdint.h>

#include "mt_oplog.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mt_engine mt_engine;

/* Per-document capacities (device memory is sized from these). */
typedef struct mt_caps {
    int32_t ncap; /* B-tree nodes per doc; row slots = 8 * ncap                        */
    int32_t hcap; /* zamboni LRU heap entries (collections.ts:212-264)                 */
    int32_t acap; /* text arena half size, UTF-16 units                                 */
    int32_t mcap; /* pending segment-group membership log entries                       */
    int32_t gcap; /* pending local ops (segment groups) in flight                       */
    int32_t ccap; /* distinct clients per doc (<= 254)                                  */
    int32_t dcap; /* delta event log words per doc; 0 = no delta events (mt_oplog.h)   */
    int32_t rcap; /* local references per doc (MT_OP_REF records); 0 = none           */
    int32_t pcap; /* PermutationVector handles per doc (getAllocatedHandle records); 0 = none */
} mt_caps;

/* status codes */
enum {
    MT_OK = 0,
    MT_E_INSERT_FAILED = 1, /* per doc: mergeTree.ts:2243-2249 "MergeTree insert failed"       */
    MT_E_ASSERT = 2,        /* per doc: a reference `assert` would have thrown                 */
    MT_E_INVALID_RANGE = 3, /* reserved (a local op getValidOpRange rejects is a no-op, client.ts:486) */
    MT_E_UNSUPPORTED = 4,   /* per doc: a path the engine does not model (mt_oplog.h)          */
    MT_E_CAPACITY = 5,      /* per doc: a capacity was exceeded even after promotion (mt_engine_sync) */
    MT_E_ARG = 16,          /* engine: bad argument                                            */
    MT_E_HIP = 17,          /* engine: HIP runtime error (mt_engine_last_error has the text)  */
    MT_E_NOMEM = 18,        /* engine: device allocation failed                                */
};

/* Create an engine with `ndocs` empty, non-collaborating replicas on HIP device `device`
 * (new Client() + MergeTree constructor, client.ts:75-84, mergeTree.ts:1143-1146). */
int32_t mt_engine_create(int32_t device, int64_t ndocs, const mt_caps* caps, mt_engine** out);
void mt_engine_destroy(mt_engine* e);
const char* mt_engine_last_error(const mt_engine* e);

/* Client.startOrUpdateCollaboration(longClientId, minSeq, currentSeq) for every doc
 * (client.ts:1053-1073); local_long_ids[d] is doc d's own long-client index. */
int32_t mt_engine_start_collab(mt_engine* e, const int32_t* local_long_ids, int32_t min_seq, int32_t cur_seq);
/* The same with each document's own minSeq and currentSeq (client.ts:1053-1073 per replica): a
 * batch of documents that join collaboration at different points of their streams (e.g. loaded from
 * summaries taken at different sequence numbers). Reset returns every document to these. */
int32_t mt_engine_start_collab_docs(mt_engine* e, const int32_t* local_long_ids, const int32_t* min_seqs,
                                    const int32_t* cur_seqs);

/* Stage a batch of per-doc event streams (host memory; copied to HBM). Doc d's events are
 * ops[op_off[d] .. op_off[d+1]), its pools start at text+text_off[d], props+props_off[d],
 * kv+kv_off[d] (pools may be shared between docs). Replaces the previous staged batch. */
int32_t mt_engine_submit(mt_engine* e, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                         int64_t text_units, const int64_t* text_off, const mt_props_rec* props, int64_t nprops,
                         const int64_t* props_off, const mt_kv* kv, int64_t nkv, const int64_t* kv_off);

/* mt_engine_submit + mt_engine_run with the hand-off overlapped: the documents go in chunks (an eighth of the batch, at
 * least the documents the GPU holds at once), and chunk k's records replay while chunk k+1's are checked on the host
 * and copied (from pinned memory directly, from pageable memory through the engine's pinned staging buffers). The
 * same results as submit + run; returns once every record has been copied (the caller's buffers are free again), with
 * the replay running (mt_engine_sync waits). On MT_E_ARG (a record out of bounds) the chunks before the bad one have
 * been replayed and nothing stays staged. */
int32_t mt_engine_submit_run(mt_engine* e, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                             int64_t text_units, const int64_t* text_off, const mt_props_rec* props, int64_t nprops,
                             const int64_t* props_off, const mt_kv* kv, int64_t nkv, const int64_t* kv_off);
/* Stage records for some documents only: docs[0..m) (increasing ids) and, for docs[k], the records
 * ops[op_off[k] .. op_off[k+1]) with pools at text+text_off[k], props+props_off[k], kv+kv_off[k]. The next
 * mt_engine_run replays those documents alone (one small launch); the others keep their state. What an interactive
 * host (the JS facade's reads) stages after a few edits; the reference applies each op as it arrives. */
int32_t mt_engine_submit_docs(mt_engine* e, int64_t m, const int64_t* docs, const mt_op_rec* ops, const int64_t* op_off,
                              const uint16_t* text, int64_t text_units, const int64_t* text_off,
                              const mt_props_rec* props, int64_t nprops, const int64_t* props_off, const mt_kv* kv,
                              int64_t nkv, const int64_t* kv_off);
/* The kind of each property value id (MT_VKIND_*, kinds[id & ~MT_VALUE_FALSY], n entries): what an "incr" combining
 * annotate makes of a key holding it (properties.ts:26-59: current + undefined). Without it an incr over a present
 * interned value latches MT_E_UNSUPPORTED. Takes effect at the next run. */
int32_t mt_engine_set_value_kinds(mt_engine* e, const uint8_t* kinds, int32_t n);
/* Pinned (page-locked) host memory for op logs a caller builds in place: the hand-off then copies by DMA alone. */
int32_t mt_host_alloc(int64_t bytes, void** out);
void mt_host_free(void* p);

/* Apply every staged event to its doc: Client.applyMsg for sequenced messages (client.ts:797),
 * insertSegmentLocal / removeRangeLocal / annotateRangeLocal for local edits (202/189/164).
 * Asynchronous on the engine's HIP stream; mt_engine_sync waits. */
int32_t mt_engine_run(mt_engine* e);
/* Wait for the replay. Capacity promotion (on unless MT_NO_PROMOTE=1): documents whose replay latched
 * MT_E_CAPACITY (nodes / row slots, heap, property key slots, text arena, membership log, pending
 * groups) replay again from their staged logs in an engine of the next profile (small -> 2,048 nodes and
 * 24 key slots -> 16,384 -> 262,144 tiled, 4x the arena, membership and pending-group capacities), as
 * often as needed; every per-document call below then answers for them from there. */
int32_t mt_engine_sync(mt_engine* e);
/* The documents the last mt_engine_sync promoted (writes up to cap ids); returns their count. */
int64_t mt_engine_promoted(const mt_engine* e, int64_t* docs_out, int64_t cap);
/* Device time of the last mt_engine_run's replay kernel (HIP events on the engine stream). */
float mt_engine_last_run_ms(const mt_engine* e);
/* The engine's hipStream_t (as void*), for callers that time or order work around it. */
void* mt_engine_stream(const mt_engine* e);

/* Return every doc to the state right after create/start_collab (same local ids), keeping the
 * staged batch, so a replay can be repeated (bench steps). Asynchronous. */
int32_t mt_engine_reset(mt_engine* e);
/* Per-doc work counters for roofline accounting: out3[3d..3d+2] = (sequenced messages applied,
 * sum over them of rows in the table before the message, rows written). */
int32_t mt_engine_work(mt_engine* e, int64_t* out3);
/* Per document, when the last replay's workgroup for it started and finished: out2[2d], out2[2d + 1] in ticks of
 * the GPU's constant 100 MHz clock (s_memrealtime; comparable across documents of one device): the per-document
 * time spread and the launch's tail. Promoted documents report their replay in the larger profile. */
int32_t mt_engine_doc_times(mt_engine* e, int64_t* out2);
/* Dispatch order of the replay kernel: workgroup b replays document order[b] (a permutation of [0, ndocs); NULL
 * restores document order). The GPU dispatches workgroups in index order as slots free up, so the documents in
 * decreasing order of expected cost make a longest-first list schedule. No effect on results. */
int32_t mt_engine_set_order(mt_engine* e, const int32_t* order);
/* Kernel build selection (no effect on results; no reference counterpart — the reference has one code path):
 *   MT_VAR_SMALL_WAVES (1 | 4 | 8): build of the config-2/3 replay kernel: 1 = the hot image in LDS (three documents
 *     per CU), 4 or 8 = HBM-resident at 4 or 8 waves per SIMD (default: 1 when the batch's documents fit three per
 *     CU, 4 when they fit 4 per SIMD, else 8; the MT_SMALL_WAVES environment variable sets it at create);
 *   MT_VAR_TILED_WIDE (0 | 1): the config-4 (tiled) kernel with the zamboni heap in HBM and the full window set
 *     (default 0: the narrow LDS-heap build, which promotes documents it cannot hold to the wide one).
 *   MT_VAR_CHUNK_DOCS (>= 0): documents per chunk of mt_engine_submit_run (0: automatic).
 * Takes effect at the next mt_engine_run / mt_engine_submit_run. */
enum { MT_VAR_SMALL_WAVES = 1, MT_VAR_TILED_WIDE = 2, MT_VAR_CHUNK_DOCS = 3 };
int32_t mt_engine_set_variant(mt_engine* e, int32_t key, int32_t value);

/* Per-doc latched error code (MT_E_*) and index of the event that raised it (-1 if none). */
int32_t mt_engine_errors(mt_engine* e, int32_t* err, int32_t* err_op);
/* The same for one document (an 8-byte read). */
int32_t mt_engine_doc_error(mt_engine* e, int64_t doc, int32_t* err, int32_t* err_op);
/* Per-doc FNV-1a-64 digest of the canonical segment dump (mt_oplog.h), computed on device. */
int32_t mt_engine_digests(mt_engine* e, uint64_t* out);
/* Canonical dump of one doc; returns bytes needed (writes if cap suffices), <0 on error. */
int64_t mt_engine_dump(mt_engine* e, int64_t doc, uint8_t* out, int64_t cap);
/* MergeTree.getLength(refSeq, clientId) (mergeTree.ts:1610); long_client < 0 = local view
 * (Client.getLength, client.ts:1051). */
int32_t mt_engine_get_length(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, int32_t* out);
/* MergeTreeTextHelper.getText(refSeq, clientId) (textSegment.ts:154-172); long_client < 0 =
 * local view. Returns the length in UTF-16 units (writes at most cap), <0 on error. */
int64_t mt_engine_get_text(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out,
                           int64_t cap);
/* MergeTreeTextHelper.getText(refSeq, clientId, placeholder, start, end) (textSegment.ts:154-186): the text
 * of [start, end) under the perspective (getValidRange: MT_TEXT_DEFAULT start = 0, end = getLength), every
 * visited non-text segment (marker, permutation segment) adding `placeholder` cachedLength times
 * (gatherText 188-271; placeholder_len 0 = ""). JavaScript substring rules apply to a text segment's
 * piece (an end before the start swaps them). The placeholder "*" (Marker.toString()) returns
 * -MT_E_UNSUPPORTED. Returns the length in UTF-16 units (writes at most cap), <0 on error. */
#define MT_TEXT_DEFAULT INT32_MIN
int64_t mt_engine_get_text_range(mt_engine* e, int64_t doc, int32_t ref_seq, int32_t long_client,
                                 const uint16_t* placeholder, int32_t placeholder_len, int32_t start, int32_t end,
                                 uint16_t* out, int64_t cap);
/* SharedSequence.getItems(start, end) (sequence sharedSequence.ts:150-183; SharedObjectSequence /
 * SharedNumberSequence.getRange) of a SubSequence document (mt_oplog.h MT_SEG_RUN) in the local view: the item ids
 * (the host's item interner) of every visited SubSequence segment of [start, end), the ones before `start` in the
 * first of them spliced off and the result cut to end - start (end = MT_TEXT_DEFAULT: undefined, no cut; end <= start:
 * none). Returns the item count (writes at most cap), <0 on error. In such a document getText sees no TextSegment:
 * every visited segment gives the placeholder. */
int64_t mt_engine_get_items(mt_engine* e, int64_t doc, int32_t start, int32_t end, uint16_t* out, int64_t cap);
/* A segment handle (the reference returns live ISegment objects, mergeTree.ts:87-117): the row's
 * stable id and its generation. A handle stops resolving once zamboni merges the row into its
 * neighbour or unlinks it (mergeTree.ts:1322-1398), as a detached reference segment would. */
typedef struct mt_seg_ref {
    int32_t rid;    /* row id, -1: no segment at the position (the reference's `segment: undefined`) */
    int32_t gen;    /* row-id generation */
    int32_t offset; /* position - the segment's start */
    int32_t length; /* cachedLength */
    int32_t seq;    /* the segment's seq (-1: local, unacked) */
    int32_t client; /* long client index of its inserter, -1 = LocalClientId */
    int32_t removed_seq;    /* removedSeq: MT_NOT_REMOVED (the reference's undefined), -1 = a pending local remove */
    int32_t removed_client; /* long client index of the remover (0 when not removed), -1 = LocalClientId */
    int32_t ordinal;        /* the segment's index in walkAllSegments order (its canonical dump record) */
} mt_seg_ref;
#define MT_NOT_REMOVED INT32_MIN
/* MergeTree.getContainingSegment(pos, refSeq, clientId) (mergeTree.ts:1656-1667); long_client < 0 =
 * Client.getContainingSegment, the local view (client.ts:1006-1008). */
int32_t mt_engine_get_containing_segment(mt_engine* e, int64_t doc, int32_t pos, int32_t ref_seq, int32_t long_client,
                                         mt_seg_ref* out);
/* MergeTree.getPosition(segment, refSeq, clientId) (mergeTree.ts:1619-1636) of a handle;
 * MT_E_ARG if the handle no longer resolves. long_client < 0 = Client.getPosition (client.ts:291). */
int32_t mt_engine_get_position(mt_engine* e, int64_t doc, int32_t rid, int32_t gen, int32_t ref_seq,
                               int32_t long_client, int32_t* out);
/* MergeTree.posFromRelativePos(relativePos, refSeq, clientId) (mergeTree.ts:1976-1999; Client.posFromRelativePos
 * client.ts:308, SharedString.insertTextRelative / insertMarkerRelative): the position of the marker whose
 * property id_key (the interned "markerId" key) holds id_value, after it (+ cachedLength + offset) or before
 * it (- offset); *out = -1 if no marker holds the id; MT_E_UNSUPPORTED if several do. long_client < 0 = the
 * local view. */
int32_t mt_engine_pos_from_relative_pos(mt_engine* e, int64_t doc, int32_t id_key, int32_t id_value, int32_t before,
                                        int32_t has_offset, int32_t offset, int32_t ref_seq, int32_t long_client,
                                        int32_t* out);
/* MergeTree.resolveRemoteClientPosition(pos, refSeq, clientId) (mergeTree.ts:2140-2160; SharedSegmentSequence,
 * sequence.ts:314): the local position of what a remote client saw at `pos` under its (refSeq, client):
 * getPosition(segment) + offset in the local view, the local length when pos is that client's length, else
 * *out = -1 (undefined). A perspective persp_refused names (include note at mt_engine_get_length) returns
 * MT_E_UNSUPPORTED. */
int32_t mt_engine_resolve_remote_client_position(mt_engine* e, int64_t doc, int32_t pos, int32_t ref_seq,
                                                 int32_t long_client, int32_t* out);
/* PermutationVector.adjustPosition(pos, fromSeq, clientId) (permutationvector.ts:185-196; SharedMatrix.processCore,
 * matrix.ts:597-605): as resolveRemoteClientPosition for a segment that exists and is not removed, else -1. */
int32_t mt_engine_adjust_position(mt_engine* e, int64_t doc, int32_t pos, int32_t from_seq, int32_t long_client,
                                  int32_t* out);
/* PermutationVector.handleToPosition(handle, localSeq) (permutationvector.ts:198-253; matrix.ts:532-533): the
 * segment whose allocated handles hold `handle` (walkAllSegments order), at findReconnectionPostition(segment,
 * localSeq) + offset (client.ts:675-705). MT_E_ARG if no segment holds it or local_seq is past the replica's
 * collabWindow.localSeq (the reference's asserts, permutationvector.ts:199, client.ts:676). */
int32_t mt_engine_handle_to_position(mt_engine* e, int64_t doc, int32_t handle, int32_t local_seq, int32_t* out);
/* Client.getMarkerFromId / MergeTree.getMarkerFromId (client.ts:312, mergeTree.ts:1965-1967): the marker whose
 * property id_key holds id_value (the engine's lookup, with mt_engine_pos_from_relative_pos's limits: several
 * markers, or an id an annotate changed, return MT_E_UNSUPPORTED); out->rid = -1 if none. */
int32_t mt_engine_get_marker_from_id(mt_engine* e, int64_t doc, int32_t id_key, int32_t id_value, mt_seg_ref* out);
/* Every segment's handle in walkAllSegments order (mergeTree.ts:3002-3016), i.e. aligned with the canonical
 * dump's records: out[2i] = rid, out[2i+1] = gen for at most cap segments; returns the segment count (<0 on
 * error). With the dump this is what Client.walkSegments / getPropertiesAtPosition / findTile read. */
int64_t mt_engine_segment_ids(mt_engine* e, int64_t doc, int32_t* out, int64_t cap);
/* Delta events (mt_oplog.h MT_DELTA_*; engines created with caps.dcap > 0): the stream a
 * SharedString "sequenceDelta" + "maintenance" listener would see (sequence.ts:136-150), batched.
 * mt_engine_delta_state: per doc the words emitted since create/reset (n_out, may exceed dcap) and
 * their FNV-1a-64 (hash_out). mt_engine_deltas: one doc's logged words, the first min(n, dcap); writes
 * at most cap of them and returns how many are logged (<0 on error). */
int32_t mt_engine_delta_state(mt_engine* e, int64_t* n_out, uint64_t* hash_out);
int64_t mt_engine_deltas(mt_engine* e, int64_t doc, int32_t* out, int64_t cap);
/* Local references (MT_OP_REF records; engines created with caps.rcap > 0): per doc the number of
 * references (nref_out[d]) and, for reference i, LocalReference.toPosition() (localReference.ts:62-68:
 * Client.getPosition(segment) + getOffset(), -1 when detached) at pos_out[d * rcap + i]. References
 * follow their segment through splits and zamboni appends, and a remove slides SlideOnRemove ones to
 * the next (or last) segment and detaches the rest (mergeTree.ts:2703-2732, localReference.ts:
 * 251-342). -2: the reference's Client.addLocalReference threw for this reference (its offset holds
 * only slid references, so refsByOffset[offset].at is undefined, localReference.ts:195-201); the
 * reference keeps no such reference, and the engine leaves the tree untouched for it. */
int32_t mt_engine_ref_positions(mt_engine* e, int32_t* nref_out, int32_t* pos_out);
/* PermutationVector (engines created with caps.pcap > 0): the document's HandleTable.snapshot()
 * (handletable.ts:80-82: handles[0] = the free-list head, then 0 for an allocated handle or the next free one),
 * `len` entries; writes min(len, cap) and returns len (<0 on error). */
int64_t mt_engine_handle_table(mt_engine* e, int64_t doc, int32_t* out, int64_t cap);
/* PermutationVector.getMaybeHandle(pos) (permutationvector.ts:157-161, HandleCache.getHandle): the handle of
 * local position pos (segment start + offset; INT32_MIN = Handle.unallocated when the segment has none). */
int32_t mt_engine_get_handle(mt_engine* e, int64_t doc, int32_t pos, int32_t* out);
/* caps.rcap of the engine (the row length of mt_engine_ref_positions' pos_out) */
int32_t mt_engine_ref_capacity(const mt_engine* e);
/* Per-doc counters: nleaf, high-water row slots, high-water heap, events applied. */
int32_t mt_engine_stats(mt_engine* e, int32_t* out4_per_doc);
int64_t mt_engine_ndocs(const mt_engine* e);

#ifdef __cplusplus
}
#endif
#endif
