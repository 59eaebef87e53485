/* mt_gen.h — synthetic op-log generator (see mt_gen.c). Host-side, C ABI. */
#ifndef MT_GEN_H
#define MT_GEN_H
#include <stdint.h>
#include "../../include/mt_oplog.h"
#ifdef __cplusplus
extern "C" {
#endif
enum { MTG_FARM = 1, MTG_OBSERVER = 2, MTG_LAGGED = 3, MTG_MATRIX = 5 };
typedef struct mtg_params {
    int32_t mode;          /* MTG_FARM / MTG_OBSERVER / MTG_LAGGED / MTG_MATRIX          */
    int32_t ops_per_doc;   /* sequenced messages per document                             */
    int32_t nclients;      /* clients per document, replica included (<= 32)              */
    int32_t max_lag;       /* remote refSeq lag upper bound (MTG_LAGGED)                  */
    int32_t local_pct;     /* % of steps that are local edits of the replica (MTG_LAGGED) */
    int32_t ack_lag;       /* a local edit is sequenced 1..ack_lag seqs after it was made */
    int32_t pct_insert, pct_remove; /* op mix; annotate = the rest                       */
    int32_t max_ins_len;   /* insert length U{1..max_ins_len}                             */
    int32_t max_rem_len;   /* remove/annotate span U{1..max_rem_len}, clipped              */
    int32_t distinct_props;/* inserts carry {s: insertIndex mod 4096} (defeats coalescing) */
    int32_t newline_pct;   /* % of inserts whose last unit is '\n' (defeats coalescing)    */
    int32_t model_ncap;    /* model replica node capacity (0: default 2048)                */
    int32_t model_acap;    /* model replica text arena half-size (0: default 128K units)  */
    int32_t perm;          /* inserts are PermutationSegments of U{1..max_ins_len} rows    */
    int32_t round_ops;     /* MTG_FARM: ops generated per round before any is sequenced    */
    int32_t min_length;    /* MTG_FARM: below this local length a client only inserts      */
    int32_t group_pct;     /* MTG_LAGGED: % of edits that are replaceRange groups (insert + remove,
                              one sequenced GROUP message; sequence.ts:455-469)             */
    int32_t rewrite_pct;   /* % of annotates that carry combiningOp {name: "rewrite"}
                              (segmentPropertiesManager.ts:49-79): 1-2 keys, every other key of
                              the segment deleted unless a local update of it is pending       */
    int32_t _pad0;
    uint64_t seed_base;    /* doc d uses splitmix64 seed seed_base + d                     */
} mtg_params;
int mtg_generate(const mtg_params* P, int64_t doc_base, int64_t ndocs, int64_t op_stride, int64_t text_stride,
                 mt_op_rec* ops, int64_t* nops, uint16_t* text, int64_t* ntext, int threads);
int mtg_generate_ids(const mtg_params* P, const int64_t* ids, int64_t ndocs, int64_t op_stride, int64_t text_stride,
                     mt_op_rec* ops, int64_t* nops, uint16_t* text, int64_t* ntext, int threads);
int mtg_props_table(mt_props_rec* props, mt_kv* kv);
#ifdef __cplusplus
}
#endif
#endif
