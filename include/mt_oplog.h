/*
 * mt_oplog.h — packed op-log and canonical-dump formats shared by the HIP replay
 * engine (libmtreplay.so), the host facades and the test oracle.
 *
 * One record = one event in ONE replica's arrival-ordered stream, i.e. exactly what
 * the reference `Client` sees:
 *   - a sequenced message  -> Client.applyMsg      (packages/dds/merge-tree/src/client.ts:797-819)
 *       * from another client      -> applyRemoteOp  (client.ts:768-795)
 *       * from this replica itself -> ackPendingSegment (client.ts:589-626, mergeTree.ts:1926-1953)
 *       * a non-op message (NOOP)  -> only updateSeqNumbers (client.ts:818-828)
 *   - a local edit (MT_OPF_LOCAL) -> insertSegmentLocal / removeRangeLocal / annotateRangeLocal
 *                                    (client.ts:202, 189, 164)
 *
 * Wire-level mapping (reference ops.ts:29-102, protocol.ts:132-172):
 *   kind       <- IMergeTreeOp.type (INSERT=0, REMOVE=1, ANNOTATE=2), NOOP = non-op message
 *   client     <- msg.clientId, as an index into the document's long-client-id table
 *   seq/ref/min<- sequenceNumber / referenceSequenceNumber / minimumSequenceNumber
 *   pos1/pos2  <- op.pos1 / op.pos2           (positions in UTF-16 code units)
 *   text       <- op.seg (string or {text, props}) as UTF-16 code units in the doc text pool
 *   props      <- op.props / op.seg.props     (1-based index into the doc props table)
 *
 * All integers little-endian; records are 32 bytes, naturally aligned.
 */
#ifndef MT_OPLOG_H
#define MT_OPLOG_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* op kinds (low 3 bits of mt_op_rec.kind); values follow MergeTreeDeltaType (ops.ts:29-34) */
enum {
    MT_OP_INSERT = 0,
    MT_OP_REMOVE = 1,
    MT_OP_ANNOTATE = 2,
    /* Local reference (with MT_OPF_LOCAL; localReference.ts:20-117): what `new LocalReference(client,
     * segment, offset, refType)` + Client.addLocalReference (client.ts:295) does for the segment and
     * offset Client.getContainingSegment(pos1) returns in the local view (client.ts:1006); pos2 =
     * refType (ReferenceType, ops.ts; SlideOnRemove = 0x40). The document's references are numbered in
     * creation order; a position past the end makes a detached reference. */
    MT_OP_REF = 3, /* with seg_kind = MT_REF_REMOVE: Client.removeLocalReference of reference pos1 */
    MT_OP_NOOP = 4, /* sequenced message that is not a merge-tree op: advances currentSeq/MSN only. With
                     * MT_OPF_LOCAL: PermutationVector.getAllocatedHandle(pos1) (permutationvector.ts:
                     * 157-183) in the local view: the PermutationSegment at pos1 keeps its handle if it has
                     * one, else a one-row segment is split out at pos1 and gets HandleTable.allocate()
                     * (handletable.ts:35-40); zamboni's unlinks free handles (onMaintenance, 338-363).
                     * Client-feature build with caps.pcap > 0 (others latch MT_E_UNSUPPORTED). */
    /* Snapshot load (SnapshotLoader, snapshotLoader.ts:86-228), on an empty non-collaborating replica:
     *   RELOAD: one header segment; pos1 counts down n..1 over the header's n records, and the whole
     *           header becomes the tree at once (reloadFromSegments, mergeTree.ts:1229-1284: blocks of
     *           MaxNodesInBlock-1 = 7 children built bottom-up);
     *   COLLAB: startOrUpdateCollaboration(client, minSeq = min_seq, currentSeq = seq) (1053-1073);
     *   APPEND: one body segment (loadBody, 160-227): insertSegments(localLength, [seg], refSeq 0, client,
 *           seq); consecutive segments without seq/client go in one batch insertSegments call whose
 *           members after the first are flagged MT_OPF_GROUPED (placed at the previous member's
 *           position + its length, blockInsert mergeTree.ts:2226-2256).
     * Segment fields of RELOAD / APPEND: seg_kind, text_off (a PERM segment: its start handle, 0 = unallocated),
     * props; pos2 = the segment's length in
     * UTF-16 units (TEXT) or rows (PERM), a marker's refType (MARKER) — a loaded segment may exceed
     * text_len's 16 bits; seq (0 = UniversalSequenceNumber); client = the spec's long client,
     * MT_CLIENT_NONCOLLAB if absent; ref_seq = removedSeq (> 0) or 0 if not removed; min_seq = the
     * removing long client. */
    MT_OP_RELOAD = 5,
    MT_OP_COLLAB = 6,
    MT_OP_APPEND = 7,
};
#define MT_CLIENT_NONCOLLAB 0xFFFF /* NonCollabClient (constants.ts:15) */
#define MT_OP_KIND_MASK 0x07
#define MT_OPF_LOCAL 0x80 /* unsequenced local edit made by this replica */
/* seg_kind of an MT_OP_REF | MT_OPF_LOCAL record that removes reference pos1 (creation order) from its
 * segment's LocalReferenceCollection (Client.removeLocalReference, client.ts:299-301 ->
 * LocalReferenceCollection.removeLocalRef, localReference.ts:225-264); 0 creates one */
#define MT_REF_REMOVE 1
/* seg_kind of an MT_OP_NOOP | MT_OPF_LOCAL record that is the splitRange of Client.walkSegments(..., pos1, pos2,
 * accum, splitRange = true) (client.ts:276-285 -> MergeTree.mapRange, mergeTree.ts:2830-2838): ensureIntervalBoundary
 * at pos1, then at pos2, each only when non-zero, in the local view (client-feature build); 0 is
 * PermutationVector.getAllocatedHandle(pos1) */
#define MT_NOOP_SPLIT 1
/* seg_kind of an MT_OP_NOOP | MT_OPF_LOCAL record that loads PermutationVector's HandleTable from a summary
 * (PermutationVector.load -> HandleTable.load, permutationvector.ts:270-275, handletable.ts:84-86): entries
 * [pos1, pos1 + text_len / 2) of the `handles` array, each as two text-pool units (low, high), pos2 = the array's
 * length. A loaded PermutationSegment's start ([length, start] spec) rides in its RELOAD / APPEND record's
 * text_off (0 = unallocated). Client-feature build with caps.pcap >= length - 1. */
#define MT_NOOP_HTLOAD 2
/* A group op (MergeTreeDeltaType.GROUP, ops.ts:33, 100; e.g. SharedString.replaceRange,
 * sequence.ts:464) is one sequenced message carrying several member ops: it is sent as its member
 * records in order, all with the message's client/seq/ref_seq/min_seq, every member but the last
 * flagged MT_OPF_GROUPED. Members apply (or, for this replica's own message, ack) one after another
 * under the one seq (client.ts:782-790, 615-622); the message's updateSeqNumbers runs after the last. */
#define MT_OPF_GROUPED 0x40
/* A local insert (MT_OP_INSERT | MT_OPF_LOCAL) with MT_OPF_ATREF is Client.insertAtReferencePositionLocal
 * (client.ts:217-245, MergeTree.insertAtReferencePosition mergeTree.ts:2033-2130): pos1 is the index of
 * one of the document's local references (MT_OP_REF); nothing happens if it is detached. */
#define MT_OPF_ATREF 0x08
/* A local record with MT_OPF_REGEN (kind = the pending op's kind) is Client.regeneratePendingOp for the
 * head pending op (client.ts:706-762, 855-893; SharedSegmentSequence.reSubmitCore on reconnect): each of
 * its segments, in document order, gets a new single-segment pending group at the tail of the queue and a
 * regenerated op at findReconnectionPostition (675-705). The ack of the resubmitted message is then one
 * member record per regenerated op (a NOOP if there are none). REF, ATREF and REGEN records need the
 * client-feature build (caps.rcap or caps.dcap > 0); other engines latch MT_E_UNSUPPORTED. */
#define MT_OPF_REGEN 0x10
/* A record with MT_OPF_TREE (kind INSERT / REMOVE / ANNOTATE, without MT_OPF_LOCAL) is a MergeTree-level
 * call with explicit (refSeq, clientId, seq): MergeTree.insertSegments (mergeTree.ts:2001-2031),
 * markRangeRemoved (2640-2738, overwrite = false) or annotateRange (2598-2638) of the one segment / range
 * the record holds — client = MT_CLIENT_LOCAL for LocalClientId (constants.ts:14), seq = -1
 * (UnassignedSequenceNumber) for a local pending op. No ack, no getValidOpRange, no updateSeqNumbers: the
 * caller owns the collaboration window, as the reference's Client does around these calls. */
#define MT_OPF_TREE 0x20
#define MT_CLIENT_LOCAL 0xFFFE /* LocalClientId (constants.ts:14) in an MT_OPF_TREE record */

/* segment kinds */
enum {
    MT_SEG_TEXT = 0,   /* TextSegment   (textSegment.ts:16-112)            */
    MT_SEG_MARKER = 1, /* Marker, length 1 (mergeTree.ts:668-832)          */
    MT_SEG_PERM = 2,   /* PermutationSegment (matrix permutationvector.ts:36-122): length =
                          text_len, no text, handle unallocated; any two such rows can append */
    MT_SEG_RUN = 3,    /* SubSequence<T> (sequence sharedSequence.ts:18-101: SharedObjectSequence /
                          SharedNumberSequence items): the text units are item ids (the host's item interner);
                          canAppend = both SubSequence and either length <= MaxRun (128), no newline rule. A document
                          holds SubSequence rows or TextSegment rows, never both (SharedSequence's specToSegment
                          makes only SubSequence; mt_engine_submit refuses a document mixing the two kinds);
                          markers and PermutationSegments may sit beside either */
};
#define MT_RUN_MAXRUN 128 /* MaxRun (sharedSequence.ts:12) */

/* seg_kind bit: the record's positions are relative to markers (IRelativePosition, ops.ts:56-61;
 * Client.getValidOpRange client.ts:486-503 resolves them with MergeTree.posFromRelativePos, mergeTree.ts:
 * 1976-1999, under the op's refSeq and client). The spec follows the record's text in the text pool, at
 * text_off + text_len: MT_RELPOS_UNITS UTF-16 units {key id of the marker-id property ("markerId",
 * reservedMarkerIdKey), which (bit 0: pos1, bit 1: pos2 is relative), then per position {value id of the
 * marker id, bits (bit 0: before, bit 1: offset present), offset low 16, offset high 16}}. Sequenced
 * records only, in the client-feature build (caps.dcap or caps.rcap > 0; other engines latch
 * MT_E_UNSUPPORTED), as are a marker id held by more than one marker and one no marker holds (the
 * reference computes -1, or a position from an unlinked segment's stale parent). */
#define MT_SEG_RELPOS 0x80
#define MT_RELPOS_UNITS 10

/* combining ops for annotate (ops.ts ICombiningOp, properties.ts:26-59) */
enum {
    MT_COMBINE_NONE = 0,
    MT_COMBINE_REWRITE = 1,
    /* "incr" / "consensus" (properties.ts:26-59) as addProperties applies them (segmentPropertiesManager.ts:92-106:
     * every key is modified, pending local updates notwithstanding, and combine gets newValue undefined, SURVEY
     * Appendix A2): incr makes the value `current + undefined` — NaN from a number, a boolean or nothing, the string
     * with "undefined" appended from a string or a consensus object ("[object Object]") — and consensus over an absent
     * value a {value: undefined, seq} object; consensus over a present value keeps it. The values the engine derives
     * this way are per-document (MT_VALUE_NAN, MT_VALUE_STRCAT0.., MT_VALUE_CONS0..); telling numbers from strings
     * takes the host's value kinds (mt_engine_set_value_kinds): an incr over a value of undeclared kind latches
     * MT_E_UNSUPPORTED, as does a local consensus annotate (its ack needs annotateMarkerNotifyConsensus's pending
     * consensus, client.ts:982-989). */
    MT_COMBINE_INCR = 2,
    MT_COMBINE_CONSENSUS = 3,
};

typedef struct mt_op_rec {
    uint8_t kind;      /* MT_OP_* | MT_OPF_LOCAL                                          */
    uint8_t seg_kind;  /* insert: MT_SEG_*                                                  */
    uint16_t client;   /* long-client index (doc-local); ignored for local edits            */
    int32_t seq;       /* sequence number; ignored for local edits                           */
    int32_t ref_seq;   /* reference sequence number; ignored for local edits                 */
    int32_t min_seq;   /* minimum sequence number carried by the message                     */
    int32_t pos1;      /* insert position / range start                                      */
    int32_t pos2;      /* range end (exclusive); insert of a marker: its refType             */
    uint32_t text_off; /* insert text: offset in UTF-16 units into the doc text pool         */
    uint16_t text_len; /* insert text: length in UTF-16 units; MT_SEG_PERM: the row count     */
    uint16_t props;    /* 0 = none, else 1-based index into the doc props table              */
} mt_op_rec;

/* One property set carried by an op: nkv (key,value) pairs starting at kv_off in the doc kv
 * pool. value 0 == JSON null (delete the key, segmentPropertiesManager.ts:102-106).
 * Key and value ids index the batch-global string tables (value strings are canonical JSON). */
typedef struct mt_props_rec {
    uint32_t kv_off;
    uint16_t nkv;
    uint8_t combining; /* MT_COMBINE_* */
    uint8_t _pad;
} mt_props_rec;

/* value ids carrying this bit are falsy JSON values (0, "", false); relevant to `rewrite`
 * (segmentPropertiesManager.ts:72: `!newProps[key]`) */
#define MT_VALUE_FALSY 0x8000
/* Values the engine derives from incr / consensus (never in op records; host interners stay below
 * MT_VALUE_DERIVED): NaN; a string String(base) + "undefined" x k (per-document table entries MT_VALUE_STRCAT0 + i);
 * a {value: undefined, seq} consensus object (entries MT_VALUE_CONS0 + i). matchProperties (properties.ts:61-92)
 * never matches NaN (NaN !== NaN) or a consensus object (its `value` is undefined), so a row holding either never
 * takes an append in zamboni. */
#define MT_VALUE_DERIVED 0x7F00
#define MT_VALUE_STRCAT0 0x7F00 /* 128 entries */
#define MT_VALUE_CONS0 0x7F80   /* 127 entries */
#define MT_VALUE_NAN 0x7FFF
/* value kinds the host declares per value id (mt_engine_set_value_kinds): what `value + undefined` makes */
/* (an object or array stays UNKNOWN: String() of one can equal a string's, so `it + undefined` has no canonical base) */
enum { MT_VKIND_UNKNOWN = 0, MT_VKIND_NUMERIC = 1 /* number, boolean: NaN */, MT_VKIND_STRING = 2 /* a string */ };

typedef struct mt_kv {
    uint16_t key;
    uint16_t value;
} mt_kv;

/* ---- canonical segment dump (binary) ------------------------------------------------------
 * Header, then one variable-length record per segment in walkAllSegments order
 * (mergeTree.ts:3002-3016). The per-document digest is FNV-1a-64 over these bytes.
 *
 * header: int32 currentSeq, minSeq, localSeq, localLength, nsegs, nleaf
 * record: uint8 kind (MT_SEG_*: 0 TextSegment, 1 Marker, 2 PermutationSegment, 3 SubSequence);
 *         uint8 flags; uint8 noverlap; uint8 ngroups;
 *         int32 len, seq, client, removedSeq, removedClient, localSeq, localRemovedSeq, leaf;
 *         int32 overlap[noverlap];
 *         uint16 nprops; uint16 refType; (key,value) x nprops sorted by key id, a derived value (MT_VALUE_DERIVED..)
 *         written by its kind — MT_VALUE_STRCAT0, MT_VALUE_CONS0 or MT_VALUE_NAN — not its per-document entry;
 *         then, for each pair whose value is MT_VALUE_STRCAT0 or MT_VALUE_CONS0, in pair order: int32 a, int32 b
 *         (STRCAT: the base value id, 0 = a consensus object's "[object Object]", and the count of "undefined"s;
 *         CONS: the object's seq, 0) — a dump with no derived value is unchanged;
 *         int32 start (MT_DF_HANDLE only: a PermutationSegment's allocated handle, permutationvector.ts:38);
 *         text: len x uint16 (text segments: UTF-16 units; SubSequence segments: item ids)
 * client fields are LONG client indices; -1 = the reference's "original" (LocalClientId).
 */
enum {
    MT_DF_HAS_PROPS = 1,
    MT_DF_REMOVED = 2,
    MT_DF_LSEQ = 4,
    MT_DF_LRSEQ = 8,
    MT_DF_HANDLE = 16, /* a PermutationSegment whose start handle is allocated (never set without MT_OP_NOOP |
                          MT_OPF_LOCAL records, so dumps of other logs are unchanged) */
};

#define MT_FNV_OFFSET 0xcbf29ce484222325ULL
#define MT_FNV_PRIME 0x100000001b3ULL

/* ---- delta event stream (per document, int32 words; enabled by mt_caps.dcap > 0) ---------------
 * One event per reference callback, in the order the reference fires them while a replica applies
 * its event stream: mergeTreeDeltaCallback (INSERT mergeTree.ts:2014-2021, ANNOTATE 2625-2631,
 * REMOVE 2738-2744; what SharedString turns into "sequenceDelta", sequence.ts:136-143) and
 * mergeTreeMaintenanceCallback (SPLIT 2264-2269, APPEND 1368-1373, UNLINK 1343-1348; SharedString
 * "maintenance", sequence.ts:144-150). Snapshot-load records emit nothing (the reference loads with
 * opArgs undefined).
 *   event:   int32 op (MT_DELTA_*), int32 seq (of the record being applied; -1 for a local edit),
 *            then per delta segment: int32 pos, int32 len, int32 nd, nd x int32 (key << 16 | value),
 *            then int32 MT_DELTA_END (no position or length takes that value), int32 nseg.
 *   pos:     Client.getPosition(segment) (client.ts:291, the local view) at callback time for
 *            INSERT / REMOVE / ANNOTATE (what SequenceDeltaEvent.ranges reports,
 *            sequenceDeltaEvent.ts:40-50); -1 for maintenance events.
 *   len:     segment.cachedLength at callback time.
 *   nd:      ANNOTATE: the number of propertyDeltas entries (segmentPropertiesManager.ts:35-111),
 *            -1 when addProperties returned undefined; 0 otherwise. Entries sorted by key id; value
 *            0 = null (the key was absent), else the value id as in the canonical dump.
 * The engine folds every word (little-endian bytes) into a per-document FNV-1a-64, also past the
 * log's capacity, so a full-size run is verified by digest alone. */
enum {
    MT_DELTA_INSERT = 0,
    MT_DELTA_REMOVE = 1,
    MT_DELTA_ANNOTATE = 2,
    MT_DELTA_APPEND = -1, /* MergeTreeMaintenanceType (mergeTreeDeltaCallback.ts:16-30) */
    MT_DELTA_SPLIT = -2,
    MT_DELTA_UNLINK = -3,
    MT_DELTA_REGEN = 3, /* not a callback: the ops regeneratePendingOp returned (pos = pos1, len = the
                           segment's length, nd = the op type; seq -1) */
};
#define MT_DELTA_END ((int32_t)0x80000000) /* ends an event's segment list */
#define MT_REF_SLIDE_ON_REMOVE 0x40 /* ReferenceType.SlideOnRemove (ops.ts) */

#ifdef __cplusplus
}
#endif
#endif
