/* mt_core_host.h — serial host build of the replay core (see mt_core_host.cpp). */
#pragma once
#include <stdint.h>
#include "../../include/mt_oplog.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct mth_store mth_store;
mth_store* mth_create(int64_t ndocs, const int32_t* caps6);
mth_store* mth_create_dl(int64_t ndocs, const int32_t* caps6, int32_t dcap);
mth_store* mth_create_fx(int64_t ndocs, const int32_t* caps6, int32_t dcap, int32_t rcap);
mth_store* mth_create_fx2(int64_t ndocs, const int32_t* caps6, int32_t dcap, int32_t rcap, int32_t pcap);
int64_t mth_handle_table(mth_store* s, int64_t doc, int32_t* out, int64_t cap);
int32_t mth_get_handle(mth_store* s, int64_t doc, int32_t pos, int32_t* out);
int32_t mth_ref_positions(mth_store* s, int64_t doc, int32_t* out, int32_t cap);
int32_t mth_pending(mth_store* s, int64_t doc);
int64_t mth_deltas(mth_store* s, int64_t doc, int32_t* out, int64_t cap, uint64_t* hash);
void mth_destroy(mth_store* s);
void mth_start_collab(mth_store* s, int64_t doc, int32_t long_id, int32_t min_seq, int32_t cur_seq);
int32_t mth_apply(mth_store* s, int64_t doc, const mt_op_rec* op, const uint16_t* text, const mt_props_rec* props,
                  const mt_kv* kv);
int32_t mth_replay(mth_store* s, int64_t doc, const mt_op_rec* ops, int64_t n, const uint16_t* text,
                   const mt_props_rec* props, const mt_kv* kv);
void mth_set_value_kinds(mth_store* s, const uint8_t* kinds, int32_t n);
int32_t mth_error(mth_store* s, int64_t doc);
int32_t mth_error_op(mth_store* s, int64_t doc);
int32_t mth_length(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client);
int32_t mth_length_local(mth_store* s, int64_t doc);
int64_t mth_text(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client, uint16_t* out, int64_t cap);
int32_t mth_pos_from_relpos(mth_store* s, int64_t doc, int32_t kid, int32_t vid, int32_t before, int32_t has_off,
                            int32_t off, int32_t ref_seq, int32_t long_client, int32_t* out);
int64_t mth_text_range(mth_store* s, int64_t doc, int32_t ref_seq, int32_t long_client, const uint16_t* ph,
                       int32_t pl, int32_t start, int32_t end, uint16_t* out, int64_t cap);
int64_t mth_items(mth_store* s, int64_t doc, int32_t start, int32_t end, uint16_t* out, int64_t cap);
int64_t mth_dump(mth_store* s, int64_t doc, uint8_t* out, int64_t cap);
uint64_t mth_digest(mth_store* s, int64_t doc);
void mth_stats(mth_store* s, int64_t doc, int32_t* out8);
int32_t mth_containing(mth_store* s, int64_t doc, int32_t pos, int32_t ref_seq, int32_t long_client, int32_t* out6);
#ifdef __cplusplus
}
#endif
