/*
 * mt_gen.cpp — deterministic synthetic op-log generator (BASELINE.md "Synthetic inputs").
 *
 * Produces, per document, ONE replica's arrival-ordered event stream in the packed format of
 * include/mt_oplog.h. Positions must be valid in the perspective (refSeq, clientId) of the
 * client that issues each op, so the generator drives a model replica — the serial host build
 * of the engine's own replay core (mt_core.h) — through exactly the events it emits, and draws
 * every position from that replica's length under the issuing perspective (getLength,
 * mergeTree.ts:1610). Per-doc PRNG: xoshiro256** seeded with splitmix64(seed_base + doc).
 *
 * Workloads (configs in BASELINE.json):
 *   MTG_FARM      (config 1): the reference's TestClient conflict farm
 *                  (test/mergeTreeOperationRunner.ts:58-178): nclients replicas of ONE document,
 *                  clients 1..n-1 make local edits, client 0 only observes; each round first makes
 *                  round_ops local edits (refSeq = the editor's currentSeq, MSN = round start), then
 *                  sequences them in order and applies every message to every replica. Doc
 *                  f * nclients + c is replica c of farm f (its local edits and every message).
 *   MTG_OBSERVER  (config 2): clients 1..n-1 edit, the replica (long id 0) only observes;
 *                  refSeq = MSN = seq - 1.
 *   MTG_LAGGED    (config 3): replica = long id 1 with local edits acked up to ack_lag later;
 *                  remote refSeq lag U{0..max_lag}; MSN = min over clients' last refSeq.
 *   MTG_MATRIX    (config 5): one SharedMatrix = two PermutationVector replicas (rows, cols)
 *                  fed from ONE sequenced stream: every message targets one vector
 *                  (SharedMatrix.processCore, matrix.ts:568-578), so each vector sees the
 *                  matrix's sequence numbers with gaps, and refSeq/MSN are matrix-global.
 *                  Doc 2m is matrix m's rows vector, doc 2m+1 its cols vector.
 * Both take an op mix, insert/remove length ranges and optional coalescing defeaters
 * (distinct insert props, trailing newlines) used by the large-doc config.
 */
#include <pthread.h>
#include <initializer_list>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mt_oplog.h"
#include "mt_core.h"
#include "mt_gen.h"
#include "mt_store.h"
#include "mt_wave.h"

using namespace mt;

/* ---- PRNG ------------------------------------------------------------------------------- */
static uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
typedef struct {
    uint64_t s[4];
} rng_t;
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t next64(rng_t* r) { /* xoshiro256** */
    uint64_t res = rotl(r->s[1] * 5, 7) * 9;
    uint64_t t = r->s[1] << 17;
    r->s[2] ^= r->s[0];
    r->s[3] ^= r->s[1];
    r->s[1] ^= r->s[2];
    r->s[0] ^= r->s[3];
    r->s[2] ^= t;
    r->s[3] = rotl(r->s[3], 45);
    return res;
}
static void seed(rng_t* r, uint64_t s) {
    uint64_t x = s;
    for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&x);
}
/* uniform integer in [lo, hi] */
static int32_t uni(rng_t* r, int32_t lo, int32_t hi) {
    if (hi <= lo) return lo;
    uint64_t span = (uint64_t)(hi - lo) + 1;
    return lo + (int32_t)(next64(r) % span);
}

/* ---- model replica ---------------------------------------------------------------------- */
template <class HT>
struct Model {
    Store<HT> st;
    uint8_t* mem;
    Replica<WaveHost, HT>* r;
    const mt_props_rec* props;
    const mt_kv* kv;
    const uint16_t* text;
    bool ok;
};
template <class HT>
static void model_init(Model<HT>* m, const mtg_params* P, int32_t local_long) {
    Caps k = {P->model_acap > 0 ? P->model_acap : (1 << 17), 1 << 14, 4096};
    int64_t bytes = store_layout(m->st, k, 1);
    m->mem = host_store_alloc(bytes);
    m->ok = m->mem != nullptr;
    if (!m->ok) return;
    m->st.base = m->mem;
    m->r = new Replica<WaveHost, HT>(m->st.doc(0), WaveHost());
    m->r->init();
    m->r->start_collab(local_long, 0, 0);
}
template <class HT>
static void model_free(Model<HT>* m) {
    delete m->r;
    free(m->mem);
}
/* length under the perspective of long client `cl` at refSeq (lp: the replica's local view) */
template <class HT>
static int32_t m_length(Model<HT>* m, int32_t refSeq, int32_t cl, int lp) {
    if (lp) return m->r->length_local();
    int32_t sh = m->r->short_of(cl);
    if (sh < 0) sh = 0x7fff;
    return m->r->length(refSeq, sh);
}
template <class HT>
static void m_apply(Model<HT>* m, const mt_op_rec* e) {
    Pools p = {e, 1, m->text, m->props, m->kv};
    m->r->apply(*e, p);
}

/* ---- event emission ---------------------------------------------------------------------- */
typedef struct {
    mt_op_rec* ops;
    int64_t nops, cap;
    uint16_t* text;
    int64_t ntext, tcap;
    int overflow;
} Out;

static mt_op_rec* emit(Out* o) {
    if (o->nops >= o->cap) {
        o->overflow = 1;
        return NULL;
    }
    mt_op_rec* r = &o->ops[o->nops++];
    memset(r, 0, sizeof(*r));
    return r;
}
static const char ALNUM[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

/* fixed props table: annotate {key in b,i,u,c : value in 0,1,2,3,null} -> records 1..20;
 * insert props {s: v} for v in 0..4095 -> records 21..4116 (see mtg_props_table). */
#define ANN_RECORDS 20
#define INS_RECORDS 4096
#define CLIENT_RECORDS 32 /* {client: "<name>"} for the farm's annotateRange (mergeTreeOperationRunner.ts:22-24) */
#define REW1_RECORDS 20   /* the annotate records again, with combiningOp "rewrite" */
#define REW2_RECORDS 8    /* two-key rewrites {k1: v1, k2: v2} */
#define REW_BASE (1 + ANN_RECORDS + INS_RECORDS + CLIENT_RECORDS)
static int ann_props(rng_t* r) { return 1 + uni(r, 0, ANN_RECORDS - 1); }
/* an annotate's props record: a rewrite one for rewrite_pct % of them (no draw when rewrite_pct == 0,
 * so the other workloads' streams are unchanged) */
static int ann_props_mix(const mtg_params* P, rng_t* r) {
    if (P->rewrite_pct > 0 && uni(r, 0, 99) < P->rewrite_pct) return REW_BASE + uni(r, 0, REW1_RECORDS + REW2_RECORDS - 1);
    return ann_props(r);
}

/* Draw an op valid for perspective (refSeq, client); kind forced to insert on an empty view. */
template <class HT>
static void gen_op(const mtg_params* P, rng_t* r, Model<HT>* m, int32_t refSeq, int32_t client, int lp, Out* o,
                   mt_op_rec* e, int insert_index) {
    int32_t len = m_length(m, refSeq, client, lp);
    int roll = uni(r, 0, 99);
    int kind;
    if (len == 0 || roll < P->pct_insert)
        kind = MT_OP_INSERT;
    else if (roll < P->pct_insert + P->pct_remove)
        kind = MT_OP_REMOVE;
    else
        kind = MT_OP_ANNOTATE;
    e->kind = (uint8_t)kind;
    if (kind == MT_OP_INSERT && P->perm) { /* PermutationVector.insert(start, length) (147-151) */
        e->pos1 = uni(r, 0, len);
        e->seg_kind = MT_SEG_PERM;
        e->text_off = 0;
        e->text_len = (uint16_t)uni(r, 1, P->max_ins_len);
        if (P->distinct_props) e->props = (uint16_t)(1 + ANN_RECORDS + (insert_index % 4096));
    } else if (kind == MT_OP_INSERT) {
        e->pos1 = uni(r, 0, len);
        int tl = uni(r, 1, P->max_ins_len);
        if (o->ntext + tl > o->tcap) {
            o->overflow = 1;
            tl = 0;
        }
        e->text_off = (uint32_t)o->ntext;
        for (int i = 0; i < tl; i++) o->text[o->ntext++] = (uint16_t)ALNUM[uni(r, 0, 61)];
        if (tl && P->newline_pct && uni(r, 0, 99) < P->newline_pct) o->text[o->ntext - 1] = '\n';
        e->text_len = (uint16_t)tl;
        if (P->distinct_props) e->props = (uint16_t)(1 + ANN_RECORDS + (insert_index % 4096));
    } else {
        e->pos1 = uni(r, 0, len - 1);
        int span = uni(r, 1, P->max_rem_len);
        e->pos2 = e->pos1 + span > len ? len : e->pos1 + span;
        if (kind == MT_OP_ANNOTATE) e->props = (uint16_t)ann_props_mix(P, r);
    }
}

typedef struct {
    mt_op_rec op, op2; /* op2: the remove of a replaceRange group (nmem == 2) */
    int32_t target, nmem;
} Pending;

/* SharedString.replaceRange (sequence.ts:455-469) as the generator issues it: under perspective
 * (refSeq, client) of a document of length len > 0, insert text at end, then remove [start, end)
 * (positions of the client's view after its own insert). Fills the two member ops; the caller
 * applies the first before drawing the second is not needed: [start, end) precedes the insert. */
static void gen_replace(const mtg_params* P, rng_t* r, int32_t len, Out* o, mt_op_rec* ins, mt_op_rec* rem,
                        int insert_index) {
    int32_t start = uni(r, 0, len - 1);
    int32_t end = start + uni(r, 1, P->max_rem_len);
    if (end > len) end = len;
    memset(ins, 0, sizeof *ins);
    memset(rem, 0, sizeof *rem);
    ins->kind = MT_OP_INSERT;
    ins->pos1 = end;
    int tl = uni(r, 1, P->max_ins_len);
    if (o->ntext + tl > o->tcap) {
        o->overflow = 1;
        tl = 0;
    }
    ins->text_off = (uint32_t)o->ntext;
    for (int i = 0; i < tl; i++) o->text[o->ntext++] = (uint16_t)ALNUM[uni(r, 0, 61)];
    ins->text_len = (uint16_t)tl;
    if (P->distinct_props) ins->props = (uint16_t)(1 + ANN_RECORDS + (insert_index % 4096));
    rem->kind = MT_OP_REMOVE;
    rem->pos1 = start;
    rem->pos2 = end;
}

template <class HT>
static void gen_doc_t(const mtg_params* P, int64_t doc, Out* o, const mt_props_rec* props, const mt_kv* kv) {
    rng_t r;
    seed(&r, P->seed_base + (uint64_t)doc);
    int nclients = P->nclients < 2 ? 2 : P->nclients;
    if (nclients > 32) nclients = 32;
    int me = P->mode == MTG_OBSERVER ? 0 : 1;
    Model<HT> m;
    model_init(&m, P, me);
    if (!m.ok) {
        o->overflow = 1;
        return;
    }
    m.props = props;
    m.kv = kv;
    m.text = o->text;
    int32_t lastRef[32] = {0};
    int insert_index = 0;
    int32_t seq = 0;
    if (P->mode == MTG_OBSERVER) {
        while (seq < P->ops_per_doc && !o->overflow && !m.r->h.err) {
            int client = uni(&r, 1, nclients - 1);
            int32_t ref = seq; /* refSeq = seq - 1 for the op sequenced now */
            mt_op_rec* e = emit(o);
            if (!e) break;
            gen_op(P, &r, &m, ref, client, 0, o, e, insert_index);
            seq++;
            e->client = (uint16_t)client;
            e->seq = seq;
            e->ref_seq = ref;
            e->min_seq = seq - 1;
            if (e->kind == MT_OP_INSERT) insert_index++;
            m_apply(&m, e);
        }
    } else { /* MTG_LAGGED */
        /* A replica that never edits (local_pct == 0) is a caught-up reader: its refSeq follows the
         * stream (the service learns it from the client's noops), so it never holds the MSN back. */
        bool me_in_msn = P->local_pct > 0;
        Pending* q = (Pending*)malloc(sizeof(Pending) * (P->ops_per_doc + 16));
        int qh = 0, qn = 0;
        int32_t lastTarget = 0, msn = 0;
        while (seq < P->ops_per_doc && !o->overflow && !m.r->h.err) {
            int32_t cur = m.r->h.currentSeq;
            /* 1. a local edit, made against the local view (client.ts:164-211) */
            if (P->local_pct && uni(&r, 0, 99) < P->local_pct && qn < 4000) {
                int32_t llen = m_length(&m, cur, me, 1);
                if (P->group_pct && llen > 0 && uni(&r, 0, 99) < P->group_pct) { /* local replaceRange */
                    mt_op_rec ins, rem;
                    gen_replace(P, &r, llen, o, &ins, &rem, insert_index);
                    if (ins.text_len == 0) continue;
                    insert_index++;
                    mt_op_rec* e1 = emit(o);
                    mt_op_rec* e2 = e1 ? emit(o) : NULL;
                    if (!e2) break;
                    *e1 = ins;
                    *e2 = rem;
                    for (mt_op_rec* e : {e1, e2}) {
                        e->kind |= MT_OPF_LOCAL;
                        e->client = (uint16_t)me;
                        e->seq = -1;
                        e->ref_seq = cur;
                        m_apply(&m, e);
                    }
                    int32_t target = cur + uni(&r, 1, P->ack_lag > 0 ? P->ack_lag : 1);
                    if (target <= lastTarget) target = lastTarget + 1;
                    lastTarget = target;
                    Pending pe;
                    pe.op = ins;
                    pe.op2 = rem;
                    pe.op.ref_seq = pe.op2.ref_seq = cur;
                    pe.op.client = pe.op2.client = (uint16_t)me;
                    pe.target = target;
                    pe.nmem = 2;
                    q[qh + qn++] = pe;
                    continue;
                }
                mt_op_rec* e = emit(o);
                if (!e) break;
                gen_op(P, &r, &m, cur, me, 1, o, e, insert_index);
                if (e->kind == MT_OP_INSERT && e->text_len == 0) {
                    o->nops--;
                    continue;
                }
                e->kind |= MT_OPF_LOCAL;
                e->client = (uint16_t)me;
                e->seq = -1;
                e->ref_seq = cur;
                if ((e->kind & MT_OP_KIND_MASK) == MT_OP_INSERT) insert_index++;
                m_apply(&m, e);
                int32_t target = cur + uni(&r, 1, P->ack_lag > 0 ? P->ack_lag : 1);
                if (target <= lastTarget) target = lastTarget + 1;
                lastTarget = target;
                Pending pe;
                pe.op = *e;
                pe.op.kind &= (uint8_t)~MT_OPF_LOCAL;
                pe.op.ref_seq = cur;
                pe.target = target;
                pe.nmem = 1;
                q[qh + qn++] = pe;
                continue;
            }
            /* 2. the next sequenced message: our own op (ack) when due, else a remote op */
            seq++;
            mt_op_rec* e = emit(o);
            if (!e) break;
            if (qn > 0 && q[qh].target <= seq) {
                Pending pe = q[qh++];
                qn--;
                if (pe.op.ref_seq > lastRef[me]) lastRef[me] = pe.op.ref_seq;
                int32_t mn = INT32_MAX;
                for (int k = 0; k < nclients; k++)
                    if (lastRef[k] < mn) mn = lastRef[k];
                if (mn > msn) msn = mn;
                *e = pe.op;
                e->seq = seq;
                e->min_seq = msn;
                if (pe.nmem == 2) { /* the group's first member, then the last (below) */
                    e->kind |= MT_OPF_GROUPED;
                    m_apply(&m, e);
                    e = emit(o);
                    if (!e) break;
                    *e = pe.op2;
                    e->seq = seq;
                    e->min_seq = msn;
                }
            } else {
                int client = uni(&r, 0, nclients - 2);
                if (client >= me) client++;
                int32_t ref = cur - uni(&r, 0, P->max_lag);
                if (ref < lastRef[client]) ref = lastRef[client];
                if (ref < msn) ref = msn;
                lastRef[client] = ref;
                int32_t mn = INT32_MAX;
                for (int k = 0; k < nclients; k++)
                    if (lastRef[k] < mn && (k != me || me_in_msn)) mn = lastRef[k];
                if (mn > msn) msn = mn;
                int32_t rlen = P->group_pct ? m_length(&m, ref, client, 0) : 0;
                if (P->group_pct && rlen > 0 && uni(&r, 0, 99) < P->group_pct) { /* remote replaceRange */
                    mt_op_rec ins, rem;
                    gen_replace(P, &r, rlen, o, &ins, &rem, insert_index);
                    insert_index++;
                    for (mt_op_rec* x : {&ins, &rem}) {
                        x->client = (uint16_t)client;
                        x->seq = seq;
                        x->ref_seq = ref;
                        x->min_seq = msn;
                    }
                    if (ins.text_len == 0) { /* nothing to insert: a plain remove message */
                        *e = rem;
                    } else {
                        *e = ins;
                        e->kind |= MT_OPF_GROUPED;
                        m_apply(&m, e);
                        e = emit(o);
                        if (!e) break;
                        *e = rem;
                    }
                } else {
                    gen_op(P, &r, &m, ref, client, 0, o, e, insert_index);
                    e->client = (uint16_t)client;
                    e->seq = seq;
                    e->ref_seq = ref;
                    e->min_seq = msn;
                    if (e->kind == MT_OP_INSERT) insert_index++;
                }
            }
            m_apply(&m, e);
        }
        free(q);
    }
    if (m.r->h.err) o->overflow = 2;
    model_free(&m);
}
/* MTG_MATRIX: matrix `doc >> 1`, emitting only the events of vector `doc & 1` (the other
 * vector's model is still driven, so both docs of a matrix draw the same random stream). */
template <class HT>
static void gen_matrix_t(const mtg_params* P, int64_t doc, Out* o, const mt_props_rec* props, const mt_kv* kv) {
    rng_t r;
    seed(&r, P->seed_base + (uint64_t)(doc >> 1));
    int which = (int)(doc & 1);
    int nclients = P->nclients < 2 ? 2 : P->nclients;
    if (nclients > 32) nclients = 32;
    const int me = 1;
    Model<HT> m[2];
    Out scratch = {(mt_op_rec*)malloc(sizeof(mt_op_rec) * o->cap), 0, o->cap, NULL, 0, 0, 0};
    Out* out[2];
    out[which] = o;
    out[which ^ 1] = &scratch;
    for (int t = 0; t < 2; t++) {
        model_init(&m[t], P, me);
        if (!m[t].ok || !scratch.ops) {
            o->overflow = 1;
            return;
        }
        m[t].props = props;
        m[t].kv = kv;
        m[t].text = o->text;
    }
    Pending* q = (Pending*)malloc(sizeof(Pending) * (2 * P->ops_per_doc + 16));
    int32_t lastRef[32] = {0};
    int insert_index[2] = {0, 0};
    int32_t nseq[2] = {0, 0}; /* sequenced messages per vector */
    int32_t seq = 0, msn = 0, lastTarget = 0;
    int qh = 0, qn = 0;
    while ((nseq[0] < P->ops_per_doc || nseq[1] < P->ops_per_doc) && !o->overflow && !scratch.overflow &&
           !m[0].r->h.err && !m[1].r->h.err) {
        int t = uni(&r, 0, 1);
        if (nseq[t] >= P->ops_per_doc) t ^= 1;
        /* 1. a local edit of vector t (PermutationVector.insert/remove, permutationvector.ts:147-157) */
        if (P->local_pct && uni(&r, 0, 99) < P->local_pct && qn < 4000) {
            mt_op_rec* e = emit(out[t]);
            if (!e) break;
            int32_t cur = m[t].r->h.currentSeq;
            gen_op(P, &r, &m[t], cur, me, 1, out[t], e, insert_index[t]);
            e->kind |= MT_OPF_LOCAL;
            e->client = (uint16_t)me;
            e->seq = -1;
            e->ref_seq = cur;
            if ((e->kind & MT_OP_KIND_MASK) == MT_OP_INSERT) insert_index[t]++;
            m_apply(&m[t], e);
            int32_t target = seq + uni(&r, 1, P->ack_lag > 0 ? P->ack_lag : 1);
            if (target <= lastTarget) target = lastTarget + 1;
            lastTarget = target;
            Pending pe;
            pe.op = *e;
            pe.op.kind &= (uint8_t)~MT_OPF_LOCAL;
            pe.op.ref_seq = seq; /* the matrix-global refSeq the runtime stamps */
            pe.target = target * 2 + t;
            q[qh + qn++] = pe;
            continue;
        }
        /* 2. the next sequenced message of the matrix: our own op (ack) when due, else remote */
        seq++;
        if (qn > 0 && (q[qh].target >> 1) <= seq) {
            Pending pe = q[qh++];
            qn--;
            int tt = pe.target & 1;
            mt_op_rec* e = emit(out[tt]);
            if (!e) break;
            if (pe.op.ref_seq > lastRef[me]) lastRef[me] = pe.op.ref_seq;
            int32_t mn = INT32_MAX;
            for (int k = 0; k < nclients; k++)
                if (lastRef[k] < mn) mn = lastRef[k];
            if (mn > msn) msn = mn;
            *e = pe.op;
            e->seq = seq;
            e->min_seq = msn;
            m_apply(&m[tt], e);
            nseq[tt]++;
        } else {
            mt_op_rec* e = emit(out[t]);
            if (!e) break;
            int client = uni(&r, 0, nclients - 2);
            if (client >= me) client++;
            int32_t ref = (seq - 1) - uni(&r, 0, P->max_lag);
            if (ref < lastRef[client]) ref = lastRef[client];
            if (ref < msn) ref = msn;
            lastRef[client] = ref;
            int32_t mn = INT32_MAX;
            for (int k = 0; k < nclients; k++)
                if (lastRef[k] < mn) mn = lastRef[k];
            if (mn > msn) msn = mn;
            gen_op(P, &r, &m[t], ref, client, 0, out[t], e, insert_index[t]);
            e->client = (uint16_t)client;
            e->seq = seq;
            e->ref_seq = ref;
            e->min_seq = msn;
            if (e->kind == MT_OP_INSERT) insert_index[t]++;
            m_apply(&m[t], e);
            nseq[t]++;
        }
    }
    if (scratch.overflow) o->overflow = 1;
    if (m[0].r->h.err || m[1].r->h.err) o->overflow = 2;
    free(q);
    free(scratch.ops);
    model_free(&m[0]);
    model_free(&m[1]);
}


/* MTG_FARM (config 1): runMergeTreeOperationRunner / generateOperationMessagesForClients /
 * applyMessages (mergeTreeOperationRunner.ts:58-178) with the farm's op set
 * [removeRange, annotateRange, insert] (client.conflictFarm.spec.ts:25-29; the insert is
 * position-based, insertSegmentLocal, instead of insertAtReferencePosition). Every replica is
 * modelled; doc `doc` emits the stream of replica doc % nclients of farm doc / nclients. */
template <class HT>
static void gen_farm_t(const mtg_params* P, int64_t doc, Out* o, const mt_props_rec* props, const mt_kv* kv) {
    int n = P->nclients < 2 ? 2 : P->nclients;
    if (n > 32) n = 32;
    int me = (int)(doc % n);
    rng_t r;
    seed(&r, P->seed_base + (uint64_t)(doc / n));
    Model<HT>* m = new Model<HT>[n];
    for (int c = 0; c < n; c++) {
        model_init(&m[c], P, c);
        if (!m[c].ok) {
            o->overflow = 1;
            delete[] m;
            return;
        }
        m[c].props = props;
        m[c].kv = kv;
        m[c].text = o->text;
    }
    int round_ops = P->round_ops > 0 ? P->round_ops : 100;
    mt_op_rec* round = (mt_op_rec*)malloc(sizeof(mt_op_rec) * round_ops);
    int32_t seq = 0;
    int done = 0;
    bool bad = false;
    while (done < P->ops_per_doc && !o->overflow && !bad) {
        int32_t msn = seq; /* minimumSequenceNumber = the round's starting seq (runner.ts:103, 138) */
        int nr = 0;
        for (int i = 0; i < round_ops && done + nr < P->ops_per_doc; i++) {
            int c = uni(&r, 1, n - 1);
            int32_t len = m[c].r->length_local();
            mt_op_rec e;
            memset(&e, 0, sizeof e);
            int kind;
            int32_t start, end = 0;
            if (len == 0 || len < P->min_length) {
                kind = MT_OP_INSERT;
                start = uni(&r, 0, len);
            } else {
                int oi = uni(&r, 0, 2); /* [removeRange, annotateRange, insert] */
                start = uni(&r, 0, len - 1);
                end = uni(&r, start + 1, len);
                kind = oi == 0 ? MT_OP_REMOVE : oi == 1 ? MT_OP_ANNOTATE : MT_OP_INSERT;
            }
            e.kind = (uint8_t)kind;
            e.pos1 = start;
            if (kind == MT_OP_INSERT) { /* text = longClientId.repeat(1..3) (runner.ts:29, 113) */
                int rep = uni(&r, 1, 3);
                if (o->ntext + rep > o->tcap) {
                    o->overflow = 1;
                    break;
                }
                e.text_off = (uint32_t)o->ntext;
                for (int k = 0; k < rep; k++) o->text[o->ntext++] = (uint16_t)ALNUM[c];
                e.text_len = (uint16_t)rep;
            } else {
                e.pos2 = end;
                if (kind == MT_OP_ANNOTATE) e.props = (uint16_t)(1 + ANN_RECORDS + INS_RECORDS + c);
            }
            e.client = (uint16_t)c;
            e.seq = -1;
            e.ref_seq = m[c].r->h.currentSeq; /* makeOpMessage: getCurrentSeq() (testClient.ts:213-234) */
            e.min_seq = msn;
            mt_op_rec loc = e;
            loc.kind |= MT_OPF_LOCAL;
            m_apply(&m[c], &loc);
            if (c == me) {
                mt_op_rec* x = emit(o);
                if (!x) break;
                *x = loc;
            }
            round[nr++] = e;
        }
        /* applyMessages: sequence in order, every replica applies every message */
        for (int i = 0; i < nr && !o->overflow; i++) {
            mt_op_rec e = round[i];
            e.seq = ++seq;
            for (int c = 0; c < n; c++) m_apply(&m[c], &e);
            mt_op_rec* x = emit(o);
            if (!x) break;
            *x = e;
        }
        done += nr;
        for (int c = 0; c < n; c++)
            if (m[c].r->h.err) bad = true;
    }
    if (bad) o->overflow = 2;
    free(round);
    for (int c = 0; c < n; c++) model_free(&m[c]);
    delete[] m;
}

static void gen_doc(const mtg_params* P, int64_t doc, Out* o, const mt_props_rec* props, const mt_kv* kv) {
    if (P->mode == MTG_FARM)
        gen_farm_t<HotMid>(P, doc, o, props, kv);
    else if (P->mode == MTG_MATRIX)
        gen_matrix_t<HotMid>(P, doc, o, props, kv);
    else if (P->model_ncap > HotBig::N)
        gen_doc_t<HotHuge>(P, doc, o, props, kv);
    else if (P->model_ncap > HotMid::N)
        gen_doc_t<HotBig>(P, doc, o, props, kv);
    else
        gen_doc_t<HotMid>(P, doc, o, props, kv);
}

/* ---- batch API --------------------------------------------------------------------------- */
typedef struct {
    const mtg_params* P;
    const int64_t* ids; /* document ids to generate (nullptr: doc_base + i) */
    int64_t doc_base, ndocs, op_stride, text_stride;
    int tid, threads;
    mt_op_rec* ops;
    int64_t* nops;
    uint16_t* text;
    int64_t* ntext;
    int* status;
    const mt_props_rec* props;
    const mt_kv* kv;
} Job;
static void* worker(void* p) {
    Job* j = (Job*)p;
    for (int64_t d = j->tid; d < j->ndocs; d += j->threads) {
        Out o = {j->ops + d * j->op_stride, 0, j->op_stride, j->text + d * j->text_stride, 0, j->text_stride, 0};
        gen_doc(j->P, j->ids ? j->ids[d] : j->doc_base + d, &o, j->props, j->kv);
        j->nops[d] = o.nops;
        j->ntext[d] = o.ntext;
        if (o.overflow) *j->status = o.overflow == 2 ? -2 : -1;
    }
    return NULL;
}
static int generate(const mtg_params* P, const int64_t* ids, int64_t doc_base, int64_t ndocs, int64_t op_stride,
                    int64_t text_stride, mt_op_rec* ops, int64_t* nops, uint16_t* text, int64_t* ntext, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    static mt_props_rec props[REW_BASE - 1 + REW1_RECORDS + REW2_RECORDS];
    static mt_kv kv[REW_BASE - 1 + REW1_RECORDS + 3 * REW2_RECORDS];
    mtg_props_table(props, kv);
    pthread_t th[256];
    Job jobs[256];
    int status = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = Job{P, ids, doc_base, ndocs, op_stride, text_stride, t, threads, ops, nops, text, ntext, &status,
                      props, kv};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return status;
}
extern "C" int mtg_generate(const mtg_params* P, int64_t doc_base, int64_t ndocs, int64_t op_stride,
                            int64_t text_stride, mt_op_rec* ops, int64_t* nops, uint16_t* text, int64_t* ntext,
                            int threads) {
    return generate(P, nullptr, doc_base, ndocs, op_stride, text_stride, ops, nops, text, ntext, threads);
}
/* the same for an explicit list of document ids (a rank's bin-packed shard, shard.assign) */
extern "C" int mtg_generate_ids(const mtg_params* P, const int64_t* ids, int64_t ndocs, int64_t op_stride,
                                int64_t text_stride, mt_op_rec* ops, int64_t* nops, uint16_t* text, int64_t* ntext,
                                int threads) {
    return generate(P, ids, 0, ndocs, op_stride, text_stride, ops, nops, text, ntext, threads);
}

/* The fixed props table every generated doc shares: records 1..20 annotate one key of
 * {b,i,u,c} (key ids 1..4) with value ids for JSON 0,1,2,3 (value id = v + 1; "0" is falsy)
 * or null; records 21..4116 are insert props {s: v}, key id 5, v in 0..4095; records
 * 4117..4148 are the farm's {client: "<name of client k>"}, key id 6, value id 4097 + k;
 * records 4149..4168 are records 1..20 with combiningOp "rewrite", and 4169..4176 two-key rewrites
 * {k1: v1, k2: v2} over {b,i,u,c} (their key/value entries follow the single-entry ones). */
extern "C" int mtg_props_table(mt_props_rec* props, mt_kv* kv) {
    int n = 0;
    for (int k = 0; k < 4; k++)
        for (int v = 0; v < 5; v++) {
            props[n].kv_off = (uint32_t)n;
            props[n].nkv = 1;
            props[n].combining = MT_COMBINE_NONE;
            props[n]._pad = 0;
            kv[n].key = (uint16_t)(k + 1);
            kv[n].value = v == 4 ? 0 : (uint16_t)((v + 1) | (v == 0 ? MT_VALUE_FALSY : 0));
            n++;
        }
    for (int v = 0; v < 4096; v++) {
        props[n].kv_off = (uint32_t)n;
        props[n].nkv = 1;
        props[n].combining = MT_COMBINE_NONE;
        props[n]._pad = 0;
        kv[n].key = 5;
        kv[n].value = (uint16_t)((v + 1) | (v == 0 ? MT_VALUE_FALSY : 0));
        n++;
    }
    for (int k = 0; k < CLIENT_RECORDS; k++) {
        props[n].kv_off = (uint32_t)n;
        props[n].nkv = 1;
        props[n].combining = MT_COMBINE_NONE;
        props[n]._pad = 0;
        kv[n].key = 6;
        kv[n].value = (uint16_t)(INS_RECORDS + 1 + k);
        n++;
    }
    for (int k = 0; k < 4; k++)
        for (int v = 0; v < 5; v++) {
            props[n].kv_off = (uint32_t)n;
            props[n].nkv = 1;
            props[n].combining = MT_COMBINE_REWRITE;
            props[n]._pad = 0;
            kv[n].key = (uint16_t)(k + 1);
            kv[n].value = v == 4 ? 0 : (uint16_t)((v + 1) | (v == 0 ? MT_VALUE_FALSY : 0));
            n++;
        }
    int nkv = n + REW2_RECORDS; /* the single-entry records' kv slots end at n + REW2_RECORDS */
    for (int i = 0; i < REW2_RECORDS; i++) {
        int k1 = i % 4, k2 = (i + 1 + i / 4) % 4; /* two distinct keys */
        int v1 = (i % 3) + 1, v2 = (i % 2) ? 0 : 3; /* v2 = null on odd records: "delete k2" */
        props[n].kv_off = (uint32_t)nkv;
        props[n].nkv = 2;
        props[n].combining = MT_COMBINE_REWRITE;
        props[n]._pad = 0;
        kv[n].key = 0; /* unused slot (keeps kv index == record index for the single-entry records) */
        kv[n].value = 0;
        kv[nkv].key = (uint16_t)(k1 + 1);
        kv[nkv].value = (uint16_t)(v1 + 1);
        kv[nkv + 1].key = (uint16_t)(k2 + 1);
        kv[nkv + 1].value = v2 == 0 ? 0 : (uint16_t)(v2 + 1);
        nkv += 2;
        n++;
    }
    return n;
}
