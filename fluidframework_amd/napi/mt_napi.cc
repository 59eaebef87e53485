/*
 * mt_napi.cc — the Node-API addon over the engine's C ABI (include/mt_engine.h).
 *
 * The reference's hot path is the TypeScript module @fluidframework/merge-tree; its callers
 * (SharedSegmentSequence, sequence.ts:579-616; SharedMatrix, matrix.ts:568-578) would reach the
 * MI355X engine through this addon and the JS facade next to it (../js/mergetree_gpu.js), which
 * keeps the Client surface (applyMsg, the *Local edits, getLength, getText,
 * getContainingSegment, getPosition). The addon is a thin, synchronous marshalling layer: typed
 * arrays in, numbers / strings / typed arrays out, one engine handle per batch of documents (an
 * external with a finalizer). Engine status codes become thrown JS errors, as the reference throws
 * synchronously (client.ts:462-465, mergeTree.ts:2243-2249).
 *
 * Build: g++ -shared -fPIC against the vendored Node-API headers (include/, NAPI 8, node 12),
 * linked to libmtreplay.so with an $ORIGIN rpath (native.build_napi). napi_* symbols resolve from
 * the node binary at load time.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/mt_engine.h"

#define NAPI_OK(call)                                                     \
    do {                                                                  \
        if ((call) != napi_ok) {                                          \
            napi_throw_error(env, nullptr, "N-API call failed: " #call); \
            return nullptr;                                               \
        }                                                                 \
    } while (0)

static napi_value throw_status(napi_env env, mt_engine* e, int32_t rc, const char* what) {
    std::string msg = std::string(what) + " failed: status " + std::to_string(rc);
    if (e) msg += std::string(": ") + mt_engine_last_error(e);
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

static void finalize_engine(napi_env, void* data, void*) { mt_engine_destroy((mt_engine*)data); }

static bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < want) {
        napi_throw_type_error(env, nullptr, "missing arguments");
        return false;
    }
    return true;
}

static mt_engine* engine_of(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, "not an engine handle");
        return nullptr;
    }
    return (mt_engine*)p;
}

static bool i32_of(napi_env env, napi_value v, int32_t* out) {
    if (napi_get_value_int32(env, v, out) != napi_ok) {
        napi_throw_type_error(env, nullptr, "expected a number");
        return false;
    }
    return true;
}
static bool i64_of(napi_env env, napi_value v, int64_t* out) {
    if (napi_get_value_int64(env, v, out) != napi_ok) {
        napi_throw_type_error(env, nullptr, "expected a number");
        return false;
    }
    return true;
}

/* any typed array: its bytes and element count */
static bool view_of(napi_env env, napi_value v, void** data, size_t* len, napi_typedarray_type want) {
    napi_typedarray_type t;
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok || t != want) {
        napi_throw_type_error(env, nullptr, "unexpected typed array type");
        return false;
    }
    return true;
}

static napi_value num(napi_env env, double x) {
    napi_value v;
    napi_create_double(env, x, &v);
    return v;
}

/* create(device, ndocs, {ncap, hcap, acap, mcap, gcap, ccap}) -> handle */
static napi_value js_create(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    int32_t device;
    int64_t ndocs;
    if (!i32_of(env, argv[0], &device) || !i64_of(env, argv[1], &ndocs)) return nullptr;
    mt_caps caps = {};
    const char* names[6] = {"ncap", "hcap", "acap", "mcap", "gcap", "ccap"};
    int32_t* fields[6] = {&caps.ncap, &caps.hcap, &caps.acap, &caps.mcap, &caps.gcap, &caps.ccap};
    for (int i = 0; i < 6; i++) {
        napi_value f;
        NAPI_OK(napi_get_named_property(env, argv[2], names[i], &f));
        if (!i32_of(env, f, fields[i])) return nullptr;
    }
    /* optional: delta event log words (mt_caps.dcap), local references (mt_caps.rcap) and PermutationVector
     * handles (mt_caps.pcap) per doc */
    const char* opt[3] = {"dcap", "rcap", "pcap"};
    int32_t* ofield[3] = {&caps.dcap, &caps.rcap, &caps.pcap};
    for (int i = 0; i < 3; i++) {
        bool has = false;
        NAPI_OK(napi_has_named_property(env, argv[2], opt[i], &has));
        if (!has) continue;
        napi_value f;
        NAPI_OK(napi_get_named_property(env, argv[2], opt[i], &f));
        if (!i32_of(env, f, ofield[i])) return nullptr;
    }
    mt_engine* e = nullptr;
    int32_t rc = mt_engine_create(device, ndocs, &caps, &e);
    if (rc) return throw_status(env, nullptr, rc, "mt_engine_create");
    napi_value h;
    NAPI_OK(napi_create_external(env, e, finalize_engine, nullptr, &h));
    return h;
}

/* startCollab(h, Int32Array localLongIds, minSeq | Int32Array minSeqs, curSeq | Int32Array curSeqs):
 * one (minSeq, currentSeq) for every document, or each document's own (mt_engine_start_collab_docs) */
static bool seqs_of(napi_env env, napi_value v, int64_t nd, std::vector<int32_t>* out) {
    bool typed = false;
    if (napi_is_typedarray(env, v, &typed) == napi_ok && typed) {
        void* p;
        size_t n;
        if (!view_of(env, v, &p, &n, napi_int32_array)) return false;
        if ((int64_t)n != nd) {
            napi_throw_range_error(env, nullptr, "one sequence number per document");
            return false;
        }
        out->assign((const int32_t*)p, (const int32_t*)p + n);
        return true;
    }
    int32_t x;
    if (!i32_of(env, v, &x)) return false;
    out->assign((size_t)nd, x);
    return true;
}
static napi_value js_start_collab(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    void* ids;
    size_t n;
    if (!e || !view_of(env, argv[1], &ids, &n, napi_int32_array)) return nullptr;
    int64_t nd = mt_engine_ndocs(e);
    if ((int64_t)n != nd) return throw_status(env, e, MT_E_ARG, "startCollab (one id per doc)");
    std::vector<int32_t> mins, curs;
    if (!seqs_of(env, argv[2], nd, &mins) || !seqs_of(env, argv[3], nd, &curs)) return nullptr;
    int32_t rc = mt_engine_start_collab_docs(e, (const int32_t*)ids, mins.data(), curs.data());
    if (rc) return throw_status(env, e, rc, "mt_engine_start_collab_docs");
    return nullptr;
}

/* submit(h, Uint8Array ops, BigInt64Array opOff, Uint16Array text, BigInt64Array textOff,
 *        Uint8Array props, BigInt64Array propsOff, Uint8Array kv, BigInt64Array kvOff) */
static napi_value js_submit(napi_env env, napi_callback_info info) {
    napi_value argv[9];
    if (!get_args(env, info, 9, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    void *ops, *op_off, *text, *text_off, *props, *props_off, *kv, *kv_off;
    size_t nops_b, noo, ntext, nto, nprops_b, npo, nkv_b, nko;
    if (!view_of(env, argv[1], &ops, &nops_b, napi_uint8_array) ||
        !view_of(env, argv[2], &op_off, &noo, napi_bigint64_array) ||
        !view_of(env, argv[3], &text, &ntext, napi_uint16_array) ||
        !view_of(env, argv[4], &text_off, &nto, napi_bigint64_array) ||
        !view_of(env, argv[5], &props, &nprops_b, napi_uint8_array) ||
        !view_of(env, argv[6], &props_off, &npo, napi_bigint64_array) ||
        !view_of(env, argv[7], &kv, &nkv_b, napi_uint8_array) ||
        !view_of(env, argv[8], &kv_off, &nko, napi_bigint64_array))
        return nullptr;
    int64_t nd = mt_engine_ndocs(e);
    if ((int64_t)noo != nd + 1 || (int64_t)nto < nd || (int64_t)npo < nd || (int64_t)nko < nd ||
        nops_b % sizeof(mt_op_rec) || nprops_b % sizeof(mt_props_rec) || nkv_b % sizeof(mt_kv) ||
        ((const int64_t*)op_off)[nd] * (int64_t)sizeof(mt_op_rec) > (int64_t)nops_b)
        return throw_status(env, e, MT_E_ARG, "submit (array shapes)");
    int32_t rc = mt_engine_submit(e, (const mt_op_rec*)ops, (const int64_t*)op_off, (const uint16_t*)text,
                                  (int64_t)ntext, (const int64_t*)text_off, (const mt_props_rec*)props,
                                  (int64_t)(nprops_b / sizeof(mt_props_rec)), (const int64_t*)props_off,
                                  (const mt_kv*)kv, (int64_t)(nkv_b / sizeof(mt_kv)), (const int64_t*)kv_off);
    if (rc) return throw_status(env, e, rc, "mt_engine_submit");
    return nullptr;
}

/* submitDocs(h, BigInt64Array docs, Uint8Array ops, BigInt64Array opOff, Uint16Array text, BigInt64Array textOff,
 *            Uint8Array props, BigInt64Array propsOff, Uint8Array kv, BigInt64Array kvOff): records for the listed
 * documents only, one offset entry per listed document (mt_engine_submit_docs) */
static napi_value js_submit_docs(napi_env env, napi_callback_info info) {
    napi_value argv[10];
    if (!get_args(env, info, 10, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    void *docs, *ops, *op_off, *text, *text_off, *props, *props_off, *kv, *kv_off;
    size_t m, nops_b, noo, ntext, nto, nprops_b, npo, nkv_b, nko;
    if (!view_of(env, argv[1], &docs, &m, napi_bigint64_array) ||
        !view_of(env, argv[2], &ops, &nops_b, napi_uint8_array) ||
        !view_of(env, argv[3], &op_off, &noo, napi_bigint64_array) ||
        !view_of(env, argv[4], &text, &ntext, napi_uint16_array) ||
        !view_of(env, argv[5], &text_off, &nto, napi_bigint64_array) ||
        !view_of(env, argv[6], &props, &nprops_b, napi_uint8_array) ||
        !view_of(env, argv[7], &props_off, &npo, napi_bigint64_array) ||
        !view_of(env, argv[8], &kv, &nkv_b, napi_uint8_array) ||
        !view_of(env, argv[9], &kv_off, &nko, napi_bigint64_array))
        return nullptr;
    if (noo != m + 1 || nto < m || npo < m || nko < m || nops_b % sizeof(mt_op_rec) || nprops_b % sizeof(mt_props_rec) ||
        nkv_b % sizeof(mt_kv) || ((const int64_t*)op_off)[m] * (int64_t)sizeof(mt_op_rec) > (int64_t)nops_b)
        return throw_status(env, e, MT_E_ARG, "submitDocs (array shapes)");
    int32_t rc = mt_engine_submit_docs(e, (int64_t)m, (const int64_t*)docs, (const mt_op_rec*)ops, (const int64_t*)op_off,
                                       (const uint16_t*)text, (int64_t)ntext, (const int64_t*)text_off,
                                       (const mt_props_rec*)props, (int64_t)(nprops_b / sizeof(mt_props_rec)),
                                       (const int64_t*)props_off, (const mt_kv*)kv, (int64_t)(nkv_b / sizeof(mt_kv)),
                                       (const int64_t*)kv_off);
    if (rc) return throw_status(env, e, rc, "mt_engine_submit_docs");
    return nullptr;
}

/* setValueKinds(h, Uint8Array kinds): MT_VKIND_* per value id (mt_engine_set_value_kinds) */
static napi_value js_set_value_kinds(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    void* k;
    size_t n;
    if (!e || !view_of(env, argv[1], &k, &n, napi_uint8_array)) return nullptr;
    int32_t rc = mt_engine_set_value_kinds(e, (const uint8_t*)k, (int32_t)n);
    if (rc) return throw_status(env, e, rc, "mt_engine_set_value_kinds");
    return nullptr;
}

/* docError(h, doc) -> [err, errOp] of one document (mt_engine_doc_error) */
static napi_value js_doc_error(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    int32_t err = 0, op = 0;
    int32_t rc = mt_engine_doc_error(e, doc, &err, &op);
    if (rc) return throw_status(env, e, rc, "mt_engine_doc_error");
    napi_value out;
    NAPI_OK(napi_create_array_with_length(env, 2, &out));
    NAPI_OK(napi_set_element(env, out, 0, num(env, err)));
    NAPI_OK(napi_set_element(env, out, 1, num(env, op)));
    return out;
}

#define SIMPLE(name, call)                                            \
    static napi_value name(napi_env env, napi_callback_info info) {   \
        napi_value argv[1];                                           \
        if (!get_args(env, info, 1, argv)) return nullptr;            \
        mt_engine* e = engine_of(env, argv[0]);                       \
        if (!e) return nullptr;                                       \
        int32_t rc = call(e);                                         \
        if (rc) return throw_status(env, e, rc, #call);               \
        return nullptr;                                               \
    }
SIMPLE(js_run, mt_engine_run)
SIMPLE(js_sync, mt_engine_sync)
SIMPLE(js_reset, mt_engine_reset)

/* errors(h) -> [Int32Array err, Int32Array errOp] */
static napi_value js_errors(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    int64_t nd = mt_engine_ndocs(e);
    napi_value out, ab[2], ta[2];
    void* p[2];
    for (int i = 0; i < 2; i++) {
        NAPI_OK(napi_create_arraybuffer(env, 4 * nd, &p[i], &ab[i]));
        NAPI_OK(napi_create_typedarray(env, napi_int32_array, nd, ab[i], 0, &ta[i]));
    }
    int32_t rc = mt_engine_errors(e, (int32_t*)p[0], (int32_t*)p[1]);
    if (rc) return throw_status(env, e, rc, "mt_engine_errors");
    NAPI_OK(napi_create_array_with_length(env, 2, &out));
    NAPI_OK(napi_set_element(env, out, 0, ta[0]));
    NAPI_OK(napi_set_element(env, out, 1, ta[1]));
    return out;
}

/* digests(h) -> BigUint64Array */
static napi_value js_digests(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    int64_t nd = mt_engine_ndocs(e);
    napi_value ab, ta;
    void* p;
    NAPI_OK(napi_create_arraybuffer(env, 8 * nd, &p, &ab));
    NAPI_OK(napi_create_typedarray(env, napi_biguint64_array, nd, ab, 0, &ta));
    int32_t rc = mt_engine_digests(e, (uint64_t*)p);
    if (rc) return throw_status(env, e, rc, "mt_engine_digests");
    return ta;
}

/* refPositions(h) -> [Int32Array nref (per doc), Int32Array positions (ndocs x rcap)]:
 * LocalReference.toPosition() of every local reference (mt_engine_ref_positions) */
static napi_value js_ref_positions(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    int64_t nd = mt_engine_ndocs(e);
    int32_t rcap = mt_engine_ref_capacity(e);
    if (rcap <= 0) return throw_status(env, e, MT_E_ARG, "refPositions (engine created without caps.rcap)");
    napi_value out, ab[2], ta[2];
    void* p[2];
    size_t len[2] = {(size_t)nd, (size_t)nd * (size_t)rcap};
    for (int i = 0; i < 2; i++) {
        NAPI_OK(napi_create_arraybuffer(env, 4 * len[i], &p[i], &ab[i]));
        NAPI_OK(napi_create_typedarray(env, napi_int32_array, len[i], ab[i], 0, &ta[i]));
    }
    int32_t rc = mt_engine_ref_positions(e, (int32_t*)p[0], (int32_t*)p[1]);
    if (rc) return throw_status(env, e, rc, "mt_engine_ref_positions");
    NAPI_OK(napi_create_array_with_length(env, 2, &out));
    NAPI_OK(napi_set_element(env, out, 0, ta[0]));
    NAPI_OK(napi_set_element(env, out, 1, ta[1]));
    return out;
}

/* deltas(h, doc) -> Int32Array: the doc's logged delta-stream words (include/mt_oplog.h MT_DELTA_*) */
static napi_value js_deltas(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    int64_t n = mt_engine_deltas(e, doc, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_deltas");
    /* a full log holds only the first dcap words (cut mid-event): the stream is not decodable */
    std::vector<int64_t> emitted((size_t)mt_engine_ndocs(e));
    int32_t rc = mt_engine_delta_state(e, emitted.data(), nullptr);
    if (rc) return throw_status(env, e, rc, "mt_engine_delta_state");
    if (emitted[(size_t)doc] > n) {
        napi_throw_error(env, nullptr, "delta log full: the engine's caps.dcap is too small for this document's events");
        return nullptr;
    }
    std::vector<int32_t> tmp((size_t)(n > 0 ? n : 1));
    int64_t m = mt_engine_deltas(e, doc, tmp.data(), n);
    if (m < 0) return throw_status(env, e, (int32_t)-m, "mt_engine_deltas");
    napi_value ab, ta;
    void* p;
    NAPI_OK(napi_create_arraybuffer(env, 4 * (size_t)m, &p, &ab));
    memcpy(p, tmp.data(), 4 * (size_t)m);
    NAPI_OK(napi_create_typedarray(env, napi_int32_array, (size_t)m, ab, 0, &ta));
    return ta;
}

/* getLength(h, doc, refSeq, longClient) -> number (longClient < 0: Client.getLength) */
static napi_value js_get_length(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t ref, cl, out = 0;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &ref) || !i32_of(env, argv[3], &cl)) return nullptr;
    int32_t rc = mt_engine_get_length(e, doc, ref, cl, &out);
    if (rc) return throw_status(env, e, rc, "mt_engine_get_length");
    return num(env, out);
}

/* getText(h, doc, refSeq, longClient[, placeholder[, start[, end]]]) -> string: MergeTreeTextHelper.getText
 * (textSegment.ts:154-186); an undefined placeholder is "", an undefined start / end is getValidRange's
 * default (mt_engine_get_text_range) */
static bool opt_undefined(napi_env env, napi_value v) {
    napi_valuetype t;
    return napi_typeof(env, v, &t) == napi_ok && (t == napi_undefined || t == napi_null);
}
static napi_value js_get_text(napi_env env, napi_callback_info info) {
    napi_value argv[7];
    size_t argc = 7;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < 4) {
        napi_throw_type_error(env, nullptr, "missing arguments");
        return nullptr;
    }
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t ref, cl, start = MT_TEXT_DEFAULT, end = MT_TEXT_DEFAULT;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &ref) || !i32_of(env, argv[3], &cl)) return nullptr;
    std::vector<uint16_t> ph;
    if (argc > 4 && !opt_undefined(env, argv[4])) {
        size_t len = 0;
        if (napi_get_value_string_utf16(env, argv[4], nullptr, 0, &len) != napi_ok) {
            napi_throw_type_error(env, nullptr, "placeholder: expected a string");
            return nullptr;
        }
        ph.resize(len + 1);
        NAPI_OK(napi_get_value_string_utf16(env, argv[4], (char16_t*)ph.data(), len + 1, &len));
        ph.resize(len);
    }
    if (argc > 5 && !opt_undefined(env, argv[5]) && !i32_of(env, argv[5], &start)) return nullptr;
    if (argc > 6 && !opt_undefined(env, argv[6]) && !i32_of(env, argv[6], &end)) return nullptr;
    const uint16_t* pp = ph.empty() ? nullptr : ph.data();
    int32_t pl = (int32_t)ph.size();
    int64_t n = mt_engine_get_text_range(e, doc, ref, cl, pp, pl, start, end, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_get_text_range");
    std::vector<uint16_t> buf((size_t)n + 1);
    int64_t m = mt_engine_get_text_range(e, doc, ref, cl, pp, pl, start, end, buf.data(), n);
    if (m < 0) return throw_status(env, e, (int32_t)-m, "mt_engine_get_text_range");
    napi_value s;
    NAPI_OK(napi_create_string_utf16(env, (const char16_t*)buf.data(), (size_t)n, &s));
    return s;
}

/* getItems(h, doc, start[, end]) -> item ids: SharedSequence.getItems (sequence sharedSequence.ts:150-183) of a
 * SubSequence document in the local view (mt_engine_get_items; an undefined end is the reference's undefined) */
static napi_value js_get_items(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    size_t argc = 4;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < 3) {
        napi_throw_type_error(env, nullptr, "missing arguments");
        return nullptr;
    }
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t start, end = MT_TEXT_DEFAULT;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &start)) return nullptr;
    if (argc > 3 && !opt_undefined(env, argv[3]) && !i32_of(env, argv[3], &end)) return nullptr;
    int64_t n = mt_engine_get_items(e, doc, start, end, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_get_items");
    std::vector<uint16_t> buf((size_t)n + 1);
    int64_t m = mt_engine_get_items(e, doc, start, end, buf.data(), n);
    if (m < 0) return throw_status(env, e, (int32_t)-m, "mt_engine_get_items");
    napi_value arr;
    NAPI_OK(napi_create_array_with_length(env, (size_t)n, &arr));
    for (int64_t i = 0; i < n; i++) NAPI_OK(napi_set_element(env, arr, (uint32_t)i, num(env, buf[(size_t)i])));
    return arr;
}

/* an mt_seg_ref as {rid, gen, offset, length, seq, client, removedSeq, removedClient, ordinal}; undefined for none
 * (removedSeq: undefined when not removed, as the reference's ISegment.removedSeq) */
static napi_value seg_ref_value(napi_env env, const mt_seg_ref& r) {
    napi_value out;
    if (r.rid < 0) {
        NAPI_OK(napi_get_undefined(env, &out));
        return out;
    }
    NAPI_OK(napi_create_object(env, &out));
    const char* names[8] = {"rid", "gen", "offset", "length", "seq", "client", "removedClient", "ordinal"};
    int32_t vals[8] = {r.rid, r.gen, r.offset, r.length, r.seq, r.client, r.removed_client, r.ordinal};
    for (int i = 0; i < 8; i++) NAPI_OK(napi_set_named_property(env, out, names[i], num(env, vals[i])));
    napi_value rs;
    if (r.removed_seq == MT_NOT_REMOVED)
        NAPI_OK(napi_get_undefined(env, &rs));
    else
        rs = num(env, r.removed_seq);
    NAPI_OK(napi_set_named_property(env, out, "removedSeq", rs));
    return out;
}

/* getContainingSegment(h, doc, pos, refSeq, longClient) -> {rid, gen, offset, length, seq, client, ...} | undefined */
static napi_value js_get_containing(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t pos, ref, cl;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &pos) || !i32_of(env, argv[3], &ref) ||
        !i32_of(env, argv[4], &cl))
        return nullptr;
    mt_seg_ref r;
    int32_t rc = mt_engine_get_containing_segment(e, doc, pos, ref, cl, &r);
    if (rc) return throw_status(env, e, rc, "mt_engine_get_containing_segment");
    napi_value out;
    if (r.rid < 0) {
        NAPI_OK(napi_get_undefined(env, &out));
        return out;
    }
    return seg_ref_value(env, r);
}

/* getPosition(h, doc, rid, gen, refSeq, longClient) -> number */
static napi_value js_get_position(napi_env env, napi_callback_info info) {
    napi_value argv[6];
    if (!get_args(env, info, 6, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t rid, gen, ref, cl, out = 0;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &rid) || !i32_of(env, argv[3], &gen) ||
        !i32_of(env, argv[4], &ref) || !i32_of(env, argv[5], &cl))
        return nullptr;
    int32_t rc = mt_engine_get_position(e, doc, rid, gen, ref, cl, &out);
    if (rc) return throw_status(env, e, rc, "mt_engine_get_position (stale segment handle?)");
    return num(env, out);
}

/* handleTable(h, doc) -> Int32Array: PermutationVector's HandleTable.snapshot() (mt_engine_handle_table) */
static napi_value js_handle_table(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    int64_t n = mt_engine_handle_table(e, doc, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_handle_table (engine created without caps.pcap)");
    void* data = nullptr;
    napi_value ab, arr;
    NAPI_OK(napi_create_arraybuffer(env, 4 * (size_t)n, &data, &ab));
    int64_t m = mt_engine_handle_table(e, doc, (int32_t*)data, n);
    if (m < 0) return throw_status(env, e, (int32_t)-m, "mt_engine_handle_table");
    NAPI_OK(napi_create_typedarray(env, napi_int32_array, (size_t)n, ab, 0, &arr));
    return arr;
}

/* getHandle(h, doc, pos) -> number: getMaybeHandle (start + offset; -2^31 = Handle.unallocated) */
static napi_value js_get_handle(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t pos, out = 0;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &pos)) return nullptr;
    int32_t rc = mt_engine_get_handle(e, doc, pos, &out);
    if (rc) return throw_status(env, e, rc, "mt_engine_get_handle");
    return num(env, out);
}

/* posFromRelativePos(h, doc, keyId, valueId, before, hasOffset, offset, refSeq, longClient) -> number */
static napi_value js_pos_from_relpos(napi_env env, napi_callback_info info) {
    napi_value argv[9];
    if (!get_args(env, info, 9, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t a[7], out = 0;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    for (int i = 0; i < 7; i++)
        if (!i32_of(env, argv[2 + i], &a[i])) return nullptr;
    int32_t rc = mt_engine_pos_from_relative_pos(e, doc, a[0], a[1], a[2], a[3], a[4], a[5], a[6], &out);
    if (rc) return throw_status(env, e, rc, "mt_engine_pos_from_relative_pos");
    return num(env, out);
}

/* resolveRemoteClientPosition(h, doc, pos, refSeq, longClient) / adjustPosition(h, doc, pos, fromSeq,
 * longClient) -> number | undefined */
static napi_value remote_pos(napi_env env, napi_callback_info info, bool adjust) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t pos, ref, cl, out = -1;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &pos) || !i32_of(env, argv[3], &ref) ||
        !i32_of(env, argv[4], &cl))
        return nullptr;
    int32_t rc = adjust ? mt_engine_adjust_position(e, doc, pos, ref, cl, &out)
                        : mt_engine_resolve_remote_client_position(e, doc, pos, ref, cl, &out);
    if (rc) return throw_status(env, e, rc, adjust ? "mt_engine_adjust_position" : "mt_engine_resolve_remote_client_position");
    napi_value v;
    if (out < 0)
        NAPI_OK(napi_get_undefined(env, &v));
    else
        v = num(env, out);
    return v;
}
static napi_value js_resolve_remote(napi_env env, napi_callback_info info) { return remote_pos(env, info, false); }
static napi_value js_adjust_position(napi_env env, napi_callback_info info) { return remote_pos(env, info, true); }

/* handleToPosition(h, doc, handle, localSeq) -> number */
static napi_value js_handle_to_position(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t hnd, ls, out = 0;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &hnd) || !i32_of(env, argv[3], &ls)) return nullptr;
    int32_t rc = mt_engine_handle_to_position(e, doc, hnd, ls, &out);
    if (rc) return throw_status(env, e, rc, "mt_engine_handle_to_position");
    return num(env, out);
}

/* getMarkerFromId(h, doc, keyId, valueId) -> segment handle | undefined */
static napi_value js_marker_from_id(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    int32_t k, v;
    if (!e || !i64_of(env, argv[1], &doc) || !i32_of(env, argv[2], &k) || !i32_of(env, argv[3], &v)) return nullptr;
    mt_seg_ref r;
    int32_t rc = mt_engine_get_marker_from_id(e, doc, k, v, &r);
    if (rc) return throw_status(env, e, rc, "mt_engine_get_marker_from_id");
    return seg_ref_value(env, r);
}

/* dump(h, doc) -> Uint8Array: the canonical segment dump (include/mt_oplog.h) */
static napi_value js_dump(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    int64_t n = mt_engine_dump(e, doc, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_dump");
    void* data = nullptr;
    napi_value ab, arr;
    NAPI_OK(napi_create_arraybuffer(env, (size_t)n, &data, &ab));
    int64_t m = mt_engine_dump(e, doc, (uint8_t*)data, n);
    if (m != n) return throw_status(env, e, MT_E_ARG, "mt_engine_dump");
    NAPI_OK(napi_create_typedarray(env, napi_uint8_array, (size_t)n, ab, 0, &arr));
    return arr;
}

/* segmentIds(h, doc) -> Int32Array [rid, gen] per segment in dump order (mt_engine_segment_ids) */
static napi_value js_segment_ids(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    int64_t doc;
    if (!e || !i64_of(env, argv[1], &doc)) return nullptr;
    int64_t n = mt_engine_segment_ids(e, doc, nullptr, 0);
    if (n < 0) return throw_status(env, e, (int32_t)-n, "mt_engine_segment_ids");
    void* data = nullptr;
    napi_value ab, arr;
    NAPI_OK(napi_create_arraybuffer(env, 8 * (size_t)n, &data, &ab));
    int64_t m = mt_engine_segment_ids(e, doc, (int32_t*)data, n);
    if (m != n) return throw_status(env, e, MT_E_ARG, "mt_engine_segment_ids");
    NAPI_OK(napi_create_typedarray(env, napi_int32_array, 2 * (size_t)n, ab, 0, &arr));
    return arr;
}

static napi_value js_ndocs(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    return num(env, (double)mt_engine_ndocs(e));
}

static napi_value js_last_run_ms(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_engine* e = engine_of(env, argv[0]);
    if (!e) return nullptr;
    return num(env, mt_engine_last_run_ms(e));
}

static napi_value init(napi_env env, napi_value exports) {
    struct {
        const char* name;
        napi_callback cb;
    } fns[] = {{"create", js_create},       {"startCollab", js_start_collab}, {"submit", js_submit},
               {"run", js_run},             {"sync", js_sync},                {"reset", js_reset},
               {"errors", js_errors},       {"digests", js_digests},          {"getLength", js_get_length},
               {"getText", js_get_text}, {"getItems", js_get_items}, {"posFromRelativePos", js_pos_from_relpos},
               {"handleTable", js_handle_table},     {"getHandle", js_get_handle},    {"getContainingSegment", js_get_containing},
               {"getPosition", js_get_position}, {"ndocs", js_ndocs},        {"lastRunMs", js_last_run_ms},
               {"deltas", js_deltas},       {"refPositions", js_ref_positions},
               {"resolveRemoteClientPosition", js_resolve_remote}, {"adjustPosition", js_adjust_position},
               {"handleToPosition", js_handle_to_position}, {"getMarkerFromId", js_marker_from_id},
               {"dump", js_dump},           {"segmentIds", js_segment_ids},
               {"submitDocs", js_submit_docs}, {"docError", js_doc_error}, {"setValueKinds", js_set_value_kinds}};
    for (auto& f : fns) {
        napi_value fn;
        NAPI_OK(napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &fn));
        NAPI_OK(napi_set_named_property(env, exports, f.name, fn));
    }
    napi_value sz;
    NAPI_OK(napi_create_int32(env, (int32_t)sizeof(mt_op_rec), &sz));
    NAPI_OK(napi_set_named_property(env, exports, "OP_RECORD_BYTES", sz));
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
