/*
 * mt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference merge-tree (wizmea/FluidFramework v0.27,
 * packages/dds/merge-tree/src) used as the parity checker for the HIP replay engine and as
 * the `cpu_baseline` ("port") leg of bench.py. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product path (libmtreplay.so) never links it.
 *
 * It keeps the reference's data structures and algorithms: the B-tree of MergeBlocks with
 * MaxNodesInBlock = 8, PartialSequenceLengths per block, the zamboni LRU heap, segment-group
 * FIFOs and SegmentPropertiesManager pending-key counts. Every function cites the reference
 * file:line it follows. Parity pinning: see DESIGN.md §Oracle.
 */
#ifndef MT_ORACLE_H
#define MT_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/mt_oplog.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mto_client mto_client;

/* error codes (latched per replica) */
enum {
    MTO_OK = 0,
    MTO_ERR_INSERT_FAILED = 1,   /* mergeTree.ts:2243-2249 "MergeTree insert failed" */
    MTO_ERR_ASSERT = 2,          /* an `assert` of the reference would have thrown   */
    MTO_ERR_INVALID_RANGE = 3,   /* reserved: a local op rejected by getValidOpRange (client.ts:486-548) is a no-op */
    MTO_ERR_UNSUPPORTED = 4,
};

/* Create a replica. Not collaborating until mto_start_collab (client.ts:1053-1073). */
mto_client* mto_create(void);
void mto_destroy(mto_client* c);
void mto_set_options(mto_client* c, int verify_partials);

/* Client.startOrUpdateCollaboration(longId, minSeq, currentSeq) */
int mto_start_collab(mto_client* c, int long_id, int min_seq, int cur_seq);

/* Apply one event (sequenced message or local edit). text/props/kv are the doc pools. */
int mto_apply(mto_client* c, const mt_op_rec* op, const uint16_t* text, const mt_props_rec* props,
              const mt_kv* kv);
/* Apply a whole stream; returns first error (0 = ok). */
int mto_replay(mto_client* c, const mt_op_rec* ops, int64_t n, const uint16_t* text,
               const mt_props_rec* props, const mt_kv* kv);

int mto_error(const mto_client* c);
/* Client.getLength(): local perspective (client.ts:1051) */
int mto_local_length(const mto_client* c);
/* MergeTree.getLength(refSeq, shortClientId) (mergeTree.ts:1610) */
int mto_get_length(mto_client* c, int ref_seq, int short_client);
/* MergeTreeTextHelper.getText(refSeq, shortClientId) (textSegment.ts:154-172). Returns length;
 * writes at most cap units. short_client = -100 selects the local perspective. */
int64_t mto_get_text(mto_client* c, int ref_seq, int short_client, uint16_t* out, int64_t cap);
/* short id of a long client index, or -1 if unseen */
int mto_short_id(const mto_client* c, int long_id);
int mto_current_seq(const mto_client* c);
int mto_min_seq(const mto_client* c);
int mto_pending_groups(const mto_client* c);

/* canonical binary dump (mt_oplog.h); returns bytes needed; writes if cap large enough */
int64_t mto_dump(mto_client* c, uint8_t* out, int64_t cap);
/* getContainingSegment(pos) under (refSeq, short client; -100 = the local view) and getPosition of
 * that segment: out6 = {found, offset, length, seq, long client, position}; returns found. */
int mto_get_containing(mto_client* c, int pos, int ref_seq, int short_client, int32_t* out6);
uint64_t mto_digest(mto_client* c);

/* statistics for sizing: number of segments / leaf blocks / tree height */
void mto_stats(mto_client* c, int* nsegs, int* nleaf, int* height, int* nlive);

/* verify partial lengths of every block against recursive sums for probe perspectives;
 * returns number of mismatches (H6 in SURVEY.md) */
int mto_check_partials(mto_client* c, int ref_seq, int short_client);

/* Replay many independent documents on `threads` CPU threads (CPU baseline, one replica per
 * doc). Each doc's records are ops[op_off[d] .. op_off[d+1]) and its pools are selected by
 * the per-doc offsets. Returns elapsed wall seconds; digests written per doc if non-NULL. */
double mto_replay_batch(int ndocs, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                        const int64_t* text_off, const mt_props_rec* props, const int64_t* props_off,
                        const mt_kv* kv, const int64_t* kv_off, const int32_t* local_long_id,
                        int threads, uint64_t* digests, int32_t* errors);

#ifdef __cplusplus
}
#endif
#endif
