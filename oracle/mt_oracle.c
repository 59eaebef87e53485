/*
 * mt_oracle.c — TEST INFRASTRUCTURE ONLY (see mt_oracle.h).
 *
 * Restatement of packages/dds/merge-tree/src/{mergeTree,partialLengths,client,textSegment,
 * properties,segmentPropertiesManager,segmentGroupCollection,collections}.ts of the reference.
 * All paths below are relative to that directory. Branching (localBranchId > 0), local
 * references, tracking groups and delta callbacks are not on the replay path and are absent;
 * the places where the reference consults them are marked and evaluate to the values they
 * always have on this path (branch id 0, empty tracking collections, no local refs).
 */
#define _GNU_SOURCE
#include "mt_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------------------------
 * constants.ts:11-15, mergeTree.ts:333, 1093-1095
 * ---------------------------------------------------------------------------------------- */
#define UniversalSequenceNumber 0
#define UnassignedSequenceNumber (-1)
#define TreeMaintenanceSequenceNumber (-2)
#define LocalClientId (-1)
#define NonCollabClient (-2)
#define MaxNodesInBlock 8
#define TextSegmentGranularity 256
#define zamboniSegmentsMaxCount 2
#define MAX_OVERLAP 16

typedef struct Block Block;
typedef struct Seg Seg;
typedef struct Group Group;

/* IMergeNodeCommon (mergeTree.ts:52-58) */
typedef struct Node {
    int isLeaf;
    Block* parent;
    int index;
    int cachedLength;
} Node;

typedef struct KV {
    int key, val; /* val > 0 */
} KV;

typedef struct KVSet { /* small map kept sorted by key (JS key order is not observable here) */
    int n, cap;
    KV* a;
} KVSet;

/* collections.ts:60-200 List used as a FIFO of segment groups */
typedef struct GroupQ {
    int head, n, cap;
    Group** a;
} GroupQ;

struct Seg { /* BaseSegment (mergeTree.ts:428-572) + TextSegment/Marker */
    Node hdr;
    int kind;    /* MT_SEG_TEXT / MT_SEG_MARKER / MT_SEG_PERM / MT_SEG_RUN (SubSequence: text = item ids) */
    int refType; /* Marker.refType */
    uint16_t* text;
    int tcap;
    int seq, clientId;
    int hasRemoved, removedSeq, removedClientId;
    int nov;
    int ov[MAX_OVERLAP]; /* removedClientOverlap, in push order */
    int hasLocalSeq, localSeq;
    int hasLocalRemovedSeq, localRemovedSeq;
    int hasProps;   /* segment.properties !== undefined */
    KVSet props;    /* properties */
    int hasPM;      /* propertyManager !== undefined */
    int pendingRewriteCount;
    KVSet pendingKeys; /* pendingKeyUpdateCount */
    GroupQ groups;     /* segmentGroups (segmentGroupCollection.ts:9-40) */
};

/* partialLengths.ts:19-22, 49-55 */
typedef struct OvlC {
    int clientId, seglen;
} OvlC;
typedef struct PL {
    int seq, len, seglen, clientId;
    int hasOv;
    int nov, ovcap;
    OvlC* ov; /* RedBlackTree<number, IOverlapClient> keyed by clientId: kept sorted */
} PL;
typedef struct PLArr {
    int n, cap;
    PL* a;
} PLArr;
typedef struct PSL { /* PartialSequenceLengths (partialLengths.ts:62-732) */
    int minSeq, minLength, segmentCount;
    PLArr partialLengths;
    int ncli;
    PLArr* cli;    /* clientSeqNumbers[clientId] */
    char* cliDef;  /* clientSeqNumbers[clientId] !== undefined */
} PSL;

struct Block { /* MergeBlock (mergeTree.ts:335-382) */
    Node hdr;
    int childCount;
    Node* children[MaxNodesInBlock];
    int needsScour; /* -1 undefined, 0 false, 1 true */
    PSL* partialLengths;
};

struct Group { /* SegmentGroup (mergeTree.ts:199-202) */
    int nseg, cap;
    Seg** segs;
    int localSeq;
};

typedef struct LRU { /* LRUSegment (mergeTree.ts:952-955) */
    Seg* segment;
    int maxSeq;
} LRU;

typedef struct Heap { /* collections.ts:212-264, L[0] = comparer.min */
    int n, cap; /* n = L.length */
    LRU* L;
} Heap;

typedef struct Alloc { /* everything is freed with the replica */
    int n, cap;
    void** p;
    char* tag; /* 'S' segment, 'B' block, 'G' group */
} Alloc;

struct mto_client {
    /* MergeTree (mergeTree.ts:1084-1146) */
    Block* root;
    struct {
        int clientId, collaborating, minSeq, currentSeq, localSeq;
    } cw; /* CollaborationWindow (mergeTree.ts:856-873) */
    GroupQ pending;  /* pendingSegments */
    Heap scour;      /* segmentsToScour */
    /* Client (client.ts:43-84) */
    int longClientId; /* -1 = undefined */
    int nshort, shortcap;
    int* shortToLong;
    int longcap;
    int* longToShort;
    int err;
    int verify;
    Alloc alloc;
    /* snapshot header being reloaded (MT_OP_RELOAD records) */
    int nreload, reloadcap;
    Node** reload;
    int loadPos; /* next insert position of the open loadBody batch */
    /* replay scratch: op text/props */
    const uint16_t* textPool;
    const mt_props_rec* propsPool;
    const mt_kv* kvPool;
};

/* ------------------------------------------------------------------------------------------
 * small helpers
 * ---------------------------------------------------------------------------------------- */
static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "mt_oracle: out of memory\n");
        abort();
    }
    return p;
}
static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s ? s : 1);
    if (!p) {
        fprintf(stderr, "mt_oracle: out of memory\n");
        abort();
    }
    return p;
}
static void* xrealloc(void* p, size_t n) {
    p = realloc(p, n ? n : 1);
    if (!p) {
        fprintf(stderr, "mt_oracle: out of memory\n");
        abort();
    }
    return p;
}
static void track(mto_client* c, void* p, char tag) {
    if (c->alloc.n == c->alloc.cap) {
        c->alloc.cap = c->alloc.cap ? c->alloc.cap * 2 : 256;
        c->alloc.p = xrealloc(c->alloc.p, sizeof(void*) * c->alloc.cap);
        c->alloc.tag = xrealloc(c->alloc.tag, c->alloc.cap);
    }
    c->alloc.tag[c->alloc.n] = tag;
    c->alloc.p[c->alloc.n++] = p;
}
#define FAIL(c, code)            \
    do {                         \
        if (!(c)->err) (c)->err = (code); \
    } while (0)

static int kv_get(const KVSet* s, int key) {
    for (int i = 0; i < s->n; i++)
        if (s->a[i].key == key) return s->a[i].val;
    return 0;
}
static void kv_set(KVSet* s, int key, int val) {
    int i = 0;
    for (; i < s->n; i++) {
        if (s->a[i].key == key) {
            s->a[i].val = val;
            return;
        }
        if (s->a[i].key > key) break;
    }
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 4;
        s->a = xrealloc(s->a, sizeof(KV) * s->cap);
    }
    memmove(&s->a[i + 1], &s->a[i], sizeof(KV) * (s->n - i));
    s->a[i].key = key;
    s->a[i].val = val;
    s->n++;
}
static void kv_del(KVSet* s, int key) {
    for (int i = 0; i < s->n; i++)
        if (s->a[i].key == key) {
            memmove(&s->a[i], &s->a[i + 1], sizeof(KV) * (s->n - i - 1));
            s->n--;
            return;
        }
}
static void kv_copy(KVSet* d, const KVSet* s) {
    d->n = 0;
    for (int i = 0; i < s->n; i++) kv_set(d, s->a[i].key, s->a[i].val);
}
static void kv_free(KVSet* s) {
    free(s->a);
    s->a = NULL;
    s->n = s->cap = 0;
}

static void gq_push(GroupQ* q, Group* g) {
    if (q->head + q->n == q->cap) {
        if (q->head > 0) {
            memmove(q->a, q->a + q->head, sizeof(Group*) * q->n);
            q->head = 0;
        }
        if (q->n == q->cap) {
            q->cap = q->cap ? q->cap * 2 : 4;
            q->a = xrealloc(q->a, sizeof(Group*) * q->cap);
        }
    }
    q->a[q->head + q->n++] = g;
}
static Group* gq_pop(GroupQ* q) {
    if (!q->n) return NULL;
    Group* g = q->a[q->head++];
    q->n--;
    if (!q->n) q->head = 0;
    return g;
}

/* ------------------------------------------------------------------------------------------
 * node construction
 * ---------------------------------------------------------------------------------------- */
/* makeBlock (mergeTree.ts:1148-1157) */
static Block* makeBlock(mto_client* c, int childCount) {
    Block* b = xcalloc(1, sizeof(Block));
    track(c, b, 'B');
    b->hdr.isLeaf = 0;
    b->childCount = childCount;
    b->needsScour = -1;
    return b;
}

static Seg* newSeg(mto_client* c, int kind, const uint16_t* text, int len, int refType) {
    Seg* s = xcalloc(1, sizeof(Seg));
    track(c, s, 'S');
    s->hdr.isLeaf = 1;
    s->kind = kind;
    s->refType = refType;
    /* BaseSegment field initialisers (mergeTree.ts:432-433) */
    s->clientId = LocalClientId;
    s->seq = UniversalSequenceNumber;
    if (kind == MT_SEG_TEXT || kind == MT_SEG_RUN) { /* SubSequence(items): cachedLength = items.length */
        s->tcap = len > 0 ? len : 1;
        s->text = xmalloc(sizeof(uint16_t) * s->tcap);
        if (len) memcpy(s->text, text, sizeof(uint16_t) * len);
        s->hdr.cachedLength = len; /* textSegment.ts:43-46 */
    } else if (kind == MT_SEG_PERM) {
        /* PermutationSegment(length, start = Handle.unallocated) (permutationvector.ts:47-51) */
        s->hdr.cachedLength = len;
    } else {
        s->hdr.cachedLength = 1; /* Marker constructor (mergeTree.ts:685-688) */
    }
    return s;
}

/* ------------------------------------------------------------------------------------------
 * PartialSequenceLengths (partialLengths.ts)
 * ---------------------------------------------------------------------------------------- */
static void pl_free(PL* p) {
    free(p->ov);
    p->ov = NULL;
    p->nov = p->ovcap = 0;
}
static void pla_free(PLArr* a) {
    for (int i = 0; i < a->n; i++) pl_free(&a->a[i]);
    free(a->a);
    a->a = NULL;
    a->n = a->cap = 0;
}
static PL* pla_push(PLArr* a, PL v) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 4;
        a->a = xrealloc(a->a, sizeof(PL) * a->cap);
    }
    a->a[a->n] = v;
    return &a->a[a->n++];
}
static void psl_free(PSL* p) {
    if (!p) return;
    pla_free(&p->partialLengths);
    for (int i = 0; i < p->ncli; i++) pla_free(&p->cli[i]);
    free(p->cli);
    free(p->cliDef);
    free(p);
}
static PSL* psl_new(int minSeq) { /* constructor (partialLengths.ts:401-402) */
    PSL* p = xcalloc(1, sizeof(PSL));
    p->minSeq = minSeq;
    return p;
}
static PLArr* psl_cli(PSL* p, int clientId, int create) {
    if (clientId < 0) {
        /* JS would use a string-keyed property; never reached on the replay path because
         * clientId -1 segments carry seq 0 <= minSeq. */
        return NULL;
    }
    if (clientId >= p->ncli) {
        if (!create) return NULL;
        int n = clientId + 1;
        p->cli = xrealloc(p->cli, sizeof(PLArr) * n);
        p->cliDef = xrealloc(p->cliDef, n);
        for (int i = p->ncli; i < n; i++) {
            memset(&p->cli[i], 0, sizeof(PLArr));
            p->cliDef[i] = 0;
        }
        p->ncli = n;
    }
    if (!p->cliDef[clientId]) {
        if (!create) return NULL;
        p->cliDef[clientId] = 1;
    }
    return &p->cli[clientId];
}

static void ov_put(PL* p, int clientId, int seglen) { /* RedBlackTree.put (replace data) */
    int i = 0;
    for (; i < p->nov; i++) {
        if (p->ov[i].clientId == clientId) {
            p->ov[i].seglen = seglen;
            return;
        }
        if (p->ov[i].clientId > clientId) break;
    }
    if (p->nov == p->ovcap) {
        p->ovcap = p->ovcap ? p->ovcap * 2 : 4;
        p->ov = xrealloc(p->ov, sizeof(OvlC) * p->ovcap);
    }
    memmove(&p->ov[i + 1], &p->ov[i], sizeof(OvlC) * (p->nov - i));
    p->ov[i].clientId = clientId;
    p->ov[i].seglen = seglen;
    p->nov++;
}
static OvlC* ov_get(PL* p, int clientId) {
    for (int i = 0; i < p->nov; i++)
        if (p->ov[i].clientId == clientId) return &p->ov[i];
    return NULL;
}
static void ov_clone_into(PL* d, const PL* s) { /* cloneOverlapRemoveClients (96-104) */
    d->hasOv = s->hasOv;
    d->nov = 0;
    d->ovcap = 0;
    d->ov = NULL;
    if (s->hasOv && s->nov) {
        d->ovcap = s->nov;
        d->ov = xmalloc(sizeof(OvlC) * s->nov);
        memcpy(d->ov, s->ov, sizeof(OvlC) * s->nov);
        d->nov = s->nov;
    }
}

/* latestLEQ (partialLengths.ts:31-47) */
static int latestLEQ(const PLArr* a, int key) {
    int best = -1, lo = 0, hi = a->n - 1;
    while (lo <= hi) {
        int mid = lo + (hi - lo) / 2;
        if (a->a[mid].seq <= key) {
            if (best < 0 || a->a[best].seq < a->a[mid].seq) best = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    return best;
}

/* addClientSeqNumber (partialLengths.ts:520-530) */
static void addClientSeqNumber(PSL* p, int clientId, int seq, int seglen) {
    PLArr* cli = psl_cli(p, clientId, 1);
    if (!cli) return;
    int pLen = seglen;
    if (cli->n > 0) pLen += cli->a[cli->n - 1].len;
    PL e = {0};
    e.seq = seq;
    e.len = pLen;
    e.seglen = seglen;
    e.clientId = 0;
    pla_push(cli, e);
}
/* addClientSeqNumberFromPartial (partialLengths.ts:533-541) */
static void addClientSeqNumberFromPartial(PSL* p, const PL* pl) {
    addClientSeqNumber(p, pl->clientId, pl->seq, pl->seglen);
    if (pl->hasOv)
        for (int i = 0; i < pl->nov; i++) addClientSeqNumber(p, pl->ov[i].clientId, pl->seq, pl->ov[i].seglen);
}

/* accumulateRemoveClientOverlap (partialLengths.ts:284-301) */
static void accumulateRemoveClientOverlap(PL* pl, const int* ids, int nids, int seglen) {
    if (pl->hasOv) {
        for (int i = 0; i < nids; i++) {
            OvlC* o = ov_get(pl, ids[i]);
            if (!o)
                ov_put(pl, ids[i], seglen);
            else
                o->seglen += seglen;
        }
    } else {
        pl->hasOv = 1; /* getOverlapClients (276-282) */
        for (int i = 0; i < nids; i++) ov_put(pl, ids[i], seglen);
    }
}

/* insertSegment (partialLengths.ts:303-359) */
static void psl_insertSegment(PSL* p, const Seg* s, int removedSeq) {
    int seq = s->seq, segmentLen = s->hdr.cachedLength, clientId = s->clientId;
    const int* ovl = NULL;
    int novl = 0;
    if (removedSeq) {
        seq = s->removedSeq;
        segmentLen = -segmentLen;
        clientId = s->removedClientId;
        if (s->nov) {
            ovl = s->ov;
            novl = s->nov;
        }
    }
    PLArr* a = &p->partialLengths;
    int idx = 0;
    for (; idx < a->n; idx++)
        if (a->a[idx].seq >= seq) break;
    if (idx < a->n && a->a[idx].seq == seq) {
        a->a[idx].seglen += segmentLen;
        if (ovl) accumulateRemoveClientOverlap(&a->a[idx], ovl, novl, segmentLen);
    } else {
        PL e = {0};
        e.seq = seq;
        e.clientId = clientId;
        e.len = 0;
        e.seglen = segmentLen;
        if (ovl) {
            e.hasOv = 1;
            for (int i = 0; i < novl; i++) ov_put(&e, ovl[i], segmentLen);
        }
        pla_push(a, e); /* grow by one, then shift (351-354) */
        if (idx < a->n - 1) {
            PL tmp = a->a[a->n - 1];
            memmove(&a->a[idx + 1], &a->a[idx], sizeof(PL) * (a->n - 1 - idx));
            a->a[idx] = tmp;
        }
    }
}

/* zamboni / copyDown (partialLengths.ts:489-518) */
static int copyDown(PLArr* a, int minSeq) {
    int mindex = latestLEQ(a, minSeq);
    int minLength = 0;
    if (mindex >= 0) {
        minLength = a->a[mindex].len;
        int seqCount = a->n;
        if (mindex <= seqCount - 1) {
            int remaining = seqCount - mindex - 1;
            for (int i = 0; i <= mindex; i++) pl_free(&a->a[i]);
            for (int i = 0; i < remaining; i++) {
                a->a[i] = a->a[i + mindex + 1];
                a->a[i].len -= minLength;
            }
            a->n = remaining;
        }
    }
    return minLength;
}
static void psl_zamboni(PSL* p, int minSeq) {
    p->minLength += copyDown(&p->partialLengths, minSeq);
    for (int i = 0; i < p->ncli; i++)
        if (p->cliDef[i]) copyDown(&p->cli[i], minSeq);
}

/* getBranchId (mergeTree.ts:1208-1216) is 0 for every client on this path: no branches. */

static int localNetLength(const Seg* s); /* fwd */
static int cliLatest(PSL* p, int clientId) { /* 623-630 */
    PLArr* a = psl_cli(p, clientId, 0);
    if (a && a->n > 0) return a->n - 1;
    return -1;
}
static int cliLatestLEQ(PSL* p, int clientId, int refSeq) { /* 614-621 */
    PLArr* a = psl_cli(p, clientId, 0);
    if (a) return latestLEQ(a, refSeq);
    return -1;
}
/* getBranchPartialLength (partialLengths.ts:456-486) */
static int psl_getPartialLength(PSL* p, int refSeq, int clientId) {
    int pLen = p->minLength;
    int seqIndex = latestLEQ(&p->partialLengths, refSeq);
    int cliLatestIndex = cliLatest(p, clientId);
    PLArr* cliSeq = psl_cli(p, clientId, 0);
    if (seqIndex >= 0) {
        pLen += p->partialLengths.a[seqIndex].len;
        if (cliLatestIndex >= 0) {
            PL* latest = &cliSeq->a[cliLatestIndex];
            if (latest->seq > refSeq) {
                pLen += latest->len;
                int prec = cliLatestLEQ(p, clientId, refSeq);
                if (prec >= 0) pLen -= cliSeq->a[prec].len;
            }
        }
    } else {
        if (cliLatestIndex >= 0) pLen += cliSeq->a[cliLatestIndex].len;
    }
    return pLen;
}

/* fromLeaves (partialLengths.ts:218-274) */
static void psl_fromLeaves(PSL* p, Block* b, int minSeq) {
    p->minLength = 0;
    p->segmentCount = b->childCount;
    for (int i = 0; i < b->childCount; i++) {
        Node* ch = b->children[i];
        if (!ch->isLeaf) continue;
        Seg* s = (Seg*)ch;
        /* segBranchId <= branchId always */
        if (s->seq != UnassignedSequenceNumber && s->seq <= minSeq) {
            p->minLength += s->hdr.cachedLength;
        } else if (s->seq != UnassignedSequenceNumber) {
            psl_insertSegment(p, s, 0);
        }
        if (s->hasRemoved && s->removedSeq != UnassignedSequenceNumber && s->removedSeq <= minSeq) {
            p->minLength -= s->hdr.cachedLength;
        } else if (s->hasRemoved && s->removedSeq != UnassignedSequenceNumber) {
            psl_insertSegment(p, s, 1);
        }
    }
    int prevLen = 0;
    for (int i = 0; i < p->partialLengths.n; i++) {
        p->partialLengths.a[i].len = prevLen + p->partialLengths.a[i].seglen;
        prevLen = p->partialLengths.a[i].len;
        addClientSeqNumberFromPartial(p, &p->partialLengths.a[i]);
    }
}

static PSL* psl_combine(mto_client* c, Block* b, int recur);

/* combineBranch (partialLengths.ts:86-216) */
static PSL* psl_combineBranch(mto_client* c, Block* b, int recur) {
    int minSeq = c->cw.minSeq;
    PSL* combined = psl_new(minSeq);
    psl_fromLeaves(combined, b, minSeq);
    PSL* childPartials[MaxNodesInBlock + 1];
    int nchild = 0;
    for (int i = 0; i < b->childCount; i++) {
        Node* ch = b->children[i];
        if (!ch->isLeaf) {
            Block* cb = (Block*)ch;
            if (recur) {
                psl_free(cb->partialLengths);
                cb->partialLengths = psl_combine(c, cb, 1);
            }
            childPartials[nchild++] = cb->partialLengths;
        }
    }
    if (nchild != 0) {
        PSL* leafPart = NULL;
        if (combined->partialLengths.n > 0) {
            leafPart = combined;
            childPartials[nchild++] = combined;
            combined = psl_new(minSeq);
        }
        int indices[MaxNodesInBlock + 1], counts[MaxNodesInBlock + 1];
        for (int i = 0; i < nchild; i++) {
            indices[i] = 0;
            counts[i] = childPartials[i]->partialLengths.n;
            combined->minLength += childPartials[i]->minLength;
            combined->segmentCount += childPartials[i]->segmentCount;
        }
        PL* prev = NULL; /* prevPartial: pointer into combined->partialLengths (index kept) */
        int prevIdx = -1;
        for (;;) {
            int outer = -1;
            PL* earliest = NULL;
            for (int k = 0; k < nchild; k++) {
                if (indices[k] < counts[k]) {
                    PL* cp = &childPartials[k]->partialLengths.a[indices[k]];
                    if (outer < 0 || cp->seq < earliest->seq) {
                        outer = k;
                        earliest = cp;
                    }
                }
            }
            if (outer < 0) break;
            /* addNext (124-148) */
            {
                int pLen = 0;
                int handled = 0;
                if (prevIdx >= 0) {
                    prev = &combined->partialLengths.a[prevIdx];
                    if (prev->seq == earliest->seq) {
                        prev->seglen += earliest->seglen;
                        prev->len += earliest->seglen;
                        /* combineOverlapClients (106-122) */
                        if (prev->hasOv) {
                            if (earliest->hasOv) {
                                for (int j = 0; j < earliest->nov; j++) {
                                    OvlC* a = ov_get(prev, earliest->ov[j].clientId);
                                    if (a)
                                        a->seglen += earliest->ov[j].seglen;
                                    else
                                        ov_put(prev, earliest->ov[j].clientId, earliest->ov[j].seglen);
                                }
                            }
                        } else {
                            ov_clone_into(prev, earliest);
                        }
                        handled = 1;
                    } else {
                        pLen = prev->len;
                        addClientSeqNumberFromPartial(combined, prev);
                    }
                }
                if (!handled) {
                    PL e = {0};
                    e.clientId = earliest->clientId;
                    e.len = pLen + earliest->seglen;
                    ov_clone_into(&e, earliest);
                    e.seglen = earliest->seglen;
                    e.seq = earliest->seq;
                    pla_push(&combined->partialLengths, e);
                    prevIdx = combined->partialLengths.n - 1;
                }
            }
            indices[outer]++;
        }
        if (prevIdx >= 0) addClientSeqNumberFromPartial(combined, &combined->partialLengths.a[prevIdx]);
        if (leafPart) psl_free(leafPart);
    }
    psl_zamboni(combined, minSeq); /* options.zamboni = true (63-66) */
    return combined;
}
/* combine (partialLengths.ts:68-78); no downstream branches */
static PSL* psl_combine(mto_client* c, Block* b, int recur) { return psl_combineBranch(c, b, recur); }

/* addSeq (partialLengths.ts:361-394) */
static void addSeq(PLArr* a, int seq, int seqSeglen, int clientId) {
    PL* seqPL = NULL;
    PL* penult = NULL;
    int leq = latestLEQ(a, seq);
    int penIdx = -1;
    if (leq >= 0) {
        if (a->a[leq].seq == seq) {
            seqPL = &a->a[leq];
            int l2 = latestLEQ(a, seq - 1);
            if (l2 >= 0) penIdx = l2;
        } else {
            penIdx = leq;
        }
    }
    if (!seqPL) {
        PL e = {0};
        e.clientId = clientId;
        e.seglen = seqSeglen;
        e.seq = seq;
        int seqIdx = a->n;
        pla_push(a, e);
        seqPL = &a->a[seqIdx];
    } else {
        seqPL->seglen = seqSeglen;
    }
    penult = penIdx >= 0 ? &a->a[penIdx] : NULL;
    if (penult)
        seqPL->len = seqPL->seglen + penult->len;
    else
        seqPL->len = seqPL->seglen;
}

/* updateBranch (partialLengths.ts:546-604) */
static void psl_update(mto_client* c, PSL* p, Block* node, int seq, int clientId) {
    int seqSeglen = 0, segCount = 0;
    for (int i = 0; i < node->childCount; i++) {
        Node* ch = node->children[i];
        if (!ch->isLeaf) {
            PSL* cp = ((Block*)ch)->partialLengths;
            int si = latestLEQ(&cp->partialLengths, seq);
            if (si >= 0 && cp->partialLengths.a[si].seq == seq) seqSeglen += cp->partialLengths.a[si].seglen;
            segCount += cp->segmentCount;
        } else {
            Seg* s = (Seg*)ch;
            int rseq = s->hasRemoved ? s->removedSeq : -0x7fffffff;
            if (s->seq == seq) {
                if (rseq != seq || !s->hasRemoved) seqSeglen += s->hdr.cachedLength;
            } else {
                if (s->hasRemoved && rseq == seq) seqSeglen -= s->hdr.cachedLength;
            }
            segCount++;
        }
    }
    p->segmentCount = segCount;
    addSeq(&p->partialLengths, seq, seqSeglen, clientId);
    PLArr* cli = psl_cli(p, clientId, 1);
    if (cli) addSeq(cli, seq, seqSeglen, 0);
    psl_zamboni(p, c->cw.minSeq);
}

/* ------------------------------------------------------------------------------------------
 * MergeTree lengths (mergeTree.ts)
 * ---------------------------------------------------------------------------------------- */
/* localNetLength (1195-1206) */
static int localNetLength(const Seg* s) { return s->hasRemoved ? 0 : s->hdr.cachedLength; }

/* nodeTotalLength (421-426) */
static int nodeTotalLength(Node* n) { return n->isLeaf ? localNetLength((Seg*)n) : n->cachedLength; }

static int sumBlockLength(mto_client* c, Block* b, int refSeq, int clientId);

/* nodeLength (1692-1732) */
static int nodeLength(mto_client* c, Node* node, int refSeq, int clientId) {
    if (!c->cw.collaborating || c->cw.clientId == clientId) {
        return node->isLeaf ? localNetLength((Seg*)node) : node->cachedLength;
    }
    if (!node->isLeaf) {
        Block* b = (Block*)node;
        int v = psl_getPartialLength(b->partialLengths, refSeq, clientId);
        if (c->verify) {
            int s = sumBlockLength(c, b, refSeq, clientId);
            if (s != v) FAIL(c, MTO_ERR_ASSERT);
        }
        return v;
    }
    Seg* s = (Seg*)node;
    if (s->clientId == clientId || (s->seq != UnassignedSequenceNumber && s->seq <= refSeq)) {
        if (s->hasRemoved) {
            int inOv = 0;
            for (int i = 0; i < s->nov; i++)
                if (s->ov[i] == clientId) inOv = 1;
            if (s->removedClientId == clientId || inOv ||
                (s->removedSeq != UnassignedSequenceNumber && s->removedSeq <= refSeq))
                return 0;
            return s->hdr.cachedLength;
        }
        return s->hdr.cachedLength;
    }
    return 0;
}

/* Σ leaf nodeLength — the quantity PartialSequenceLengths is meant to equal */
static int sumBlockLength(mto_client* c, Block* b, int refSeq, int clientId) {
    int t = 0;
    for (int i = 0; i < b->childCount; i++) {
        Node* ch = b->children[i];
        if (ch->isLeaf)
            t += nodeLength(c, ch, refSeq, clientId);
        else
            t += sumBlockLength(c, (Block*)ch, refSeq, clientId);
    }
    return t;
}

/* blockLength (1669-1675) */
static int blockLength(mto_client* c, Block* b, int refSeq, int clientId) {
    if (c->cw.collaborating && clientId != c->cw.clientId) return nodeLength(c, &b->hdr, refSeq, clientId);
    return b->hdr.cachedLength;
}

/* blockUpdate (2781-2801): cachedLength; the marker tile/range maps are not on this path */
static void blockUpdate(Block* b) {
    int len = 0;
    for (int i = 0; i < b->childCount; i++) len += nodeTotalLength(b->children[i]);
    b->hdr.cachedLength = len;
}
/* nodeUpdateLengthNewStructure (2754-2759) */
static void nodeUpdateLengthNewStructure(mto_client* c, Block* b, int recur) {
    blockUpdate(b);
    if (c->cw.collaborating) {
        PSL* old = b->partialLengths;
        b->partialLengths = psl_combine(c, b, recur);
        psl_free(old);
    }
}
/* blockUpdateLength (2814-2823) */
static void blockUpdateLength(mto_client* c, Block* b, int seq, int clientId) {
    blockUpdate(b);
    if (c->cw.collaborating && seq != UnassignedSequenceNumber && seq != TreeMaintenanceSequenceNumber) {
        if (b->partialLengths && clientId != NonCollabClient) {
            psl_update(c, b->partialLengths, b, seq, clientId);
        } else {
            psl_free(b->partialLengths);
            b->partialLengths = psl_combine(c, b, 0);
        }
    }
}
/* blockUpdatePathLengths (2803-2812) */
static void blockUpdatePathLengths(mto_client* c, Block* b, int seq, int clientId, int newStructure) {
    while (b) {
        if (newStructure)
            nodeUpdateLengthNewStructure(c, b, 0);
        else
            blockUpdateLength(c, b, seq, clientId);
        b = b->hdr.parent;
    }
}

/* assignChild (374-381); ordinals are not observable and are not kept */
static void assignChild(Block* b, Node* child, int index) {
    child->parent = b;
    child->index = index;
    b->children[index] = child;
}

/* ------------------------------------------------------------------------------------------
 * Heap (collections.ts:212-264) with LRUSegmentComparer (mergeTree.ts:957-960)
 * ---------------------------------------------------------------------------------------- */
static void heap_init(Heap* h) {
    h->cap = 16;
    h->L = xmalloc(sizeof(LRU) * h->cap);
    h->L[0].segment = NULL;
    h->L[0].maxSeq = -2;
    h->n = 1;
}
static int heap_count(const Heap* h) { return h->n - 1; }
static void heap_fixup(Heap* h, int k) {
    while (k > 1 && h->L[k >> 1].maxSeq - h->L[k].maxSeq > 0) {
        LRU t = h->L[k >> 1];
        h->L[k >> 1] = h->L[k];
        h->L[k] = t;
        k >>= 1;
    }
}
static void heap_fixdown(Heap* h, int k) {
    while ((k << 1) <= heap_count(h)) {
        int j = k << 1;
        if (j < heap_count(h) && h->L[j].maxSeq - h->L[j + 1].maxSeq > 0) j++;
        if (h->L[k].maxSeq - h->L[j].maxSeq <= 0) break;
        LRU t = h->L[k];
        h->L[k] = h->L[j];
        h->L[j] = t;
        k = j;
    }
}
static void heap_add(Heap* h, LRU x) {
    if (h->n == h->cap) {
        h->cap *= 2;
        h->L = xrealloc(h->L, sizeof(LRU) * h->cap);
    }
    h->L[h->n++] = x;
    heap_fixup(h, heap_count(h));
}
static LRU heap_get(Heap* h) {
    LRU x = h->L[1];
    h->L[1] = h->L[heap_count(h)];
    h->n--;
    heap_fixdown(h, 1);
    return x;
}

/* ------------------------------------------------------------------------------------------
 * Segments: split / append / canAppend / properties
 * ---------------------------------------------------------------------------------------- */
/* matchProperties (properties.ts:61-92) on interned values: equal key sets and equal values */
static int matchProperties(const Seg* a, const Seg* b) {
    if (a->hasProps) {
        if (!b->hasProps) return 0;
        if (a->props.n != b->props.n) return 0;
        for (int i = 0; i < a->props.n; i++)
            if (a->props.a[i].key != b->props.a[i].key || a->props.a[i].val != b->props.a[i].val) return 0;
        return 1;
    }
    return b->hasProps ? 0 : 1;
}

/* TextSegment.canAppend (textSegment.ts:63-68); Marker: false (BaseSegment.canAppend);
 * PermutationSegment.canAppend (permutationvector.ts:87-93): this.start === unallocated ?
 * other.start === unallocated : contiguous handles. Handles are never allocated on the replay
 * path (getAllocatedHandle is a SharedMatrix cell-op action), so two PermutationSegments always
 * append; a non-permutation segment has start === undefined and never matches. */
static int canAppend(const Seg* a, const Seg* b) {
    if (a->kind == MT_SEG_PERM) return b->kind == MT_SEG_PERM;
    /* SubSequence.canAppend (sequence sharedSequence.ts:57-60): SubSequence.is(segment) && (this.cachedLength <= MaxRun
     * || segment.cachedLength <= MaxRun); no newline rule */
    if (a->kind == MT_SEG_RUN)
        return b->kind == MT_SEG_RUN && (a->hdr.cachedLength <= MT_RUN_MAXRUN || b->hdr.cachedLength <= MT_RUN_MAXRUN);
    if (a->kind != MT_SEG_TEXT) return 0;
    int len = a->hdr.cachedLength;
    if (len > 0 && a->text[len - 1] == '\n') return 0;
    if (b->kind != MT_SEG_TEXT) return 0;
    return a->hdr.cachedLength <= TextSegmentGranularity || b->hdr.cachedLength <= TextSegmentGranularity;
}
/* TextSegment.append (textSegment.ts:74-85); SubSequence.append (sharedSequence.ts:66-76): items.concat */
static void segAppend(Seg* a, const Seg* b) {
    int n = a->hdr.cachedLength + b->hdr.cachedLength;
    if (a->kind == MT_SEG_PERM) { /* PermutationSegment.append (permutationvector.ts:95-101) */
        a->hdr.cachedLength = n;
        return;
    }
    if (n > a->tcap) {
        int cap = a->tcap * 2;
        if (cap < n) cap = n;
        a->text = xrealloc(a->text, sizeof(uint16_t) * cap);
        a->tcap = cap;
    }
    memcpy(a->text + a->hdr.cachedLength, b->text, sizeof(uint16_t) * b->hdr.cachedLength);
    a->hdr.cachedLength = n;
}

static void groupAddSeg(Group* g, Seg* s) {
    if (g->nseg == g->cap) {
        g->cap = g->cap ? g->cap * 2 : 4;
        g->segs = xrealloc(g->segs, sizeof(Seg*) * g->cap);
    }
    g->segs[g->nseg++] = s;
}
/* SegmentGroupCollection.enqueue (segmentGroupCollection.ts:28-31) */
static void segGroupsEnqueue(Seg* s, Group* g) {
    gq_push(&s->groups, g);
    groupAddSeg(g, s);
}

/* BaseSegment.splitAt (mergeTree.ts:523-567) + TextSegment.createSplitSegmentAt (103-111) */
static Seg* splitAt(mto_client* c, Seg* s, int pos) {
    if (!(pos > 0)) return NULL;
    if (s->kind == MT_SEG_MARKER) return NULL; /* Marker.createSplitSegmentAt -> undefined */
    int len = s->hdr.cachedLength;
    /* PermutationSegment.createSplitSegmentAt (permutationvector.ts:103-114): unallocated stays
     * unallocated */
    Seg* r;
    if (s->kind == MT_SEG_PERM) { /* new PermutationSegment(cachedLength - pos); cachedLength = pos */
        r = newSeg(c, MT_SEG_PERM, NULL, len - pos, 0);
        s->hdr.cachedLength = pos;
    } else { /* text.substring(pos) / substring(0, pos): past the end, an empty right part; SubSequence's
                items.slice(pos) / slice(0, pos) the same (sharedSequence.ts:93-101) */
        int cut = pos < len ? pos : len;
        r = newSeg(c, s->kind, s->text + cut, len - cut, 0);
        s->hdr.cachedLength = cut;
    }
    /* propertyManager.copyTo (segmentPropertiesManager.ts:113-128) */
    if (s->hasProps) {
        r->hasProps = 1;
        kv_copy(&r->props, &s->props);
        if (s->hasPM) {
            r->hasPM = 1;
            r->pendingRewriteCount = s->pendingRewriteCount;
            kv_copy(&r->pendingKeys, &s->pendingKeys);
        }
    }
    r->hdr.parent = s->hdr.parent;
    r->removedClientId = s->removedClientId;
    r->hasRemoved = s->hasRemoved;
    r->removedSeq = s->removedSeq;
    r->hasLocalRemovedSeq = s->hasLocalRemovedSeq;
    r->localRemovedSeq = s->localRemovedSeq;
    r->seq = s->seq;
    r->hasLocalSeq = s->hasLocalSeq;
    r->localSeq = s->localSeq;
    r->clientId = s->clientId;
    if (s->nov) {
        r->nov = s->nov;
        memcpy(r->ov, s->ov, sizeof(int) * s->nov);
    }
    /* segmentGroups.copyTo (segmentGroupCollection.ts:37-39) */
    for (int i = 0; i < s->groups.n; i++) segGroupsEnqueue(r, s->groups.a[s->groups.head + i]);
    return r;
}

/* SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111) for ops without a
 * combining op other than "rewrite". `collaborating`/`seq` as passed by the reference. */
static void segAddProperties(Seg* s, const mt_kv* kv, int nkv, int rewrite, int seq, int collaborating) {
    if (!s->hasPM) { /* BaseSegment.addProperties creates the manager (449-454) */
        s->hasPM = 1;
    }
    if (!s->hasProps) {
        s->pendingRewriteCount = 0;
        s->hasProps = 1;
        s->props.n = 0;
        s->pendingKeys.n = 0;
    }
    if (s->pendingRewriteCount > 0 && seq != UnassignedSequenceNumber && collaborating) return;
    /* shouldModifyKey: seq === -1 || pendingKeyUpdateCount[key] === undefined || combiningOp */
#define SHOULD_MODIFY(key) (seq == UnassignedSequenceNumber || kv_get(&s->pendingKeys, (key)) == 0)
    if (rewrite) {
        if (collaborating && seq == UnassignedSequenceNumber) s->pendingRewriteCount++;
        /* delete every current key not (truthily) present in newProps */
        for (int i = 0; i < s->props.n;) {
            int key = s->props.a[i].key;
            int inNew = 0;
            for (int j = 0; j < nkv; j++)
                if (kv[j].key == key && kv[j].value != 0 && !(kv[j].value & MT_VALUE_FALSY)) inNew = 1;
            /* `!newProps[key]`: JSON null (value 0) and falsy JSON values (0, "", false: ids
             * carrying MT_VALUE_FALSY) are falsy */
            if (!inNew && SHOULD_MODIFY(key)) {
                kv_del(&s->props, key);
                continue;
            }
            i++;
        }
    }
    for (int j = 0; j < nkv; j++) {
        int key = kv[j].key;
        if (collaborating) {
            if (seq == UnassignedSequenceNumber) {
                kv_set(&s->pendingKeys, key, kv_get(&s->pendingKeys, key) + 1);
            } else if (!SHOULD_MODIFY(key)) {
                continue;
            }
        }
        if (kv[j].value == 0)
            kv_del(&s->props, key);
        else
            kv_set(&s->props, key, kv[j].value);
    }
#undef SHOULD_MODIFY
}
/* ackPendingProperties (segmentPropertiesManager.ts:19-33) */
static void segAckPendingProperties(mto_client* c, Seg* s, const mt_kv* kv, int nkv, int rewrite) {
    if (rewrite) s->pendingRewriteCount--;
    for (int j = 0; j < nkv; j++) {
        int cnt = kv_get(&s->pendingKeys, kv[j].key);
        if (cnt) {
            if (!(cnt > 0)) FAIL(c, MTO_ERR_ASSERT);
            cnt--;
            if (cnt == 0)
                kv_del(&s->pendingKeys, kv[j].key);
            else
                kv_set(&s->pendingKeys, kv[j].key, cnt);
        }
    }
}

/* ------------------------------------------------------------------------------------------
 * zamboni (mergeTree.ts:1306-1511)
 * ---------------------------------------------------------------------------------------- */
/* addToLRUSet (1306-1316) */
static void addToLRUSet(mto_client* c, Seg* s, int seq) {
    if (s->hdr.parent->needsScour != 1 && seq > c->cw.currentSeq) {
        s->hdr.parent->needsScour = 1;
        LRU x = {s, seq};
        heap_add(&c->scour, x);
    }
}
static int underflow(Block* b) { return b->childCount < MaxNodesInBlock / 2; } /* 1318-1320 */

typedef struct NodeList {
    int n, cap;
    Node** a;
} NodeList;
static void nl_push(NodeList* l, Node* n) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 16;
        l->a = xrealloc(l->a, sizeof(Node*) * l->cap);
    }
    l->a[l->n++] = n;
}

/* scourNode (1322-1398) */
static void scourNode(mto_client* c, Block* node, NodeList* hold) {
    Seg* prev = NULL;
    for (int k = 0; k < node->childCount; k++) {
        Node* ch = node->children[k];
        if (ch->isLeaf) {
            Seg* s = (Seg*)ch;
            if (s->groups.n == 0) {
                if (s->hasRemoved) {
                    /* removeBrid !== createBrid is always false (branch ids are 0) */
                    if (s->removedSeq > c->cw.minSeq) {
                        nl_push(hold, ch);
                    } else {
                        /* trackingCollection is always empty on this path */
                        s->hdr.parent = NULL; /* unlink */
                    }
                    prev = NULL;
                } else {
                    if (s->seq <= c->cw.minSeq) {
                        int ok = prev && canAppend(prev, s) && matchProperties(prev, s) &&
                                 localNetLength(s) > 0;
                        if (ok) {
                            segAppend(prev, s);
                            s->hdr.parent = NULL;
                        } else {
                            nl_push(hold, ch);
                            prev = localNetLength(s) > 0 ? s : NULL;
                        }
                    } else {
                        nl_push(hold, ch);
                        prev = NULL;
                    }
                }
            } else {
                nl_push(hold, ch);
                prev = NULL;
            }
        } else {
            nl_push(hold, ch);
            prev = NULL;
        }
    }
}

/* pack (1401-1453) */
static void pack(mto_client* c, Block* block) {
    Block* parent = block->hdr.parent;
    NodeList hold = {0};
    for (int ci = 0; ci < parent->childCount; ci++) {
        Block* cb = (Block*)parent->children[ci];
        scourNode(c, cb, &hold);
        cb->hdr.parent = NULL;
    }
    int total = hold.n;
    int half = MaxNodesInBlock / 2;
    int childCount = total / half;
    if (childCount > MaxNodesInBlock - 1) childCount = MaxNodesInBlock - 1;
    if (childCount < 1) childCount = 1;
    int base = total / childCount;
    int extra = total % childCount;
    Block* packed[MaxNodesInBlock];
    int read = 0;
    for (int ni = 0; ni < childCount; ni++) {
        int cnt = base;
        if (extra > 0) {
            cnt++;
            extra--;
        }
        Block* pb = makeBlock(c, cnt);
        for (int pi = 0; pi < cnt; pi++) assignChild(pb, hold.a[read++], pi);
        pb->hdr.parent = parent;
        packed[ni] = pb;
        nodeUpdateLengthNewStructure(c, pb, 0);
    }
    free(hold.a);
    for (int j = 0; j < MaxNodesInBlock; j++) parent->children[j] = NULL;
    for (int j = 0; j < childCount; j++) assignChild(parent, &packed[j]->hdr, j);
    parent->childCount = childCount;
    if (underflow(parent) && parent->hdr.parent) {
        pack(c, parent);
    } else {
        blockUpdatePathLengths(c, parent, UnassignedSequenceNumber, -1, 1);
    }
}

/* zamboniSegments (1455-1511) */
static void zamboniSegments(mto_client* c) {
    if (!c->cw.collaborating) return;
    for (int i = 0; i < zamboniSegmentsMaxCount; i++) {
        if (heap_count(&c->scour) < 1) break; /* peek() === undefined */
        LRU top = c->scour.L[1];
        if (top.maxSeq > c->cw.minSeq) break;
        top = heap_get(&c->scour);
        Block* block = top.segment->hdr.parent;
        if (block && block->needsScour != 0) {
            NodeList copy = {0};
            scourNode(c, block, &copy);
            block->needsScour = 0;
            int newCount = copy.n;
            if (newCount < block->childCount) {
                block->childCount = newCount;
                for (int j = 0; j < MaxNodesInBlock; j++) block->children[j] = NULL;
                for (int j = 0; j < newCount; j++) assignChild(block, copy.a[j], j);
                if (underflow(block) && block->hdr.parent) {
                    pack(c, block);
                } else {
                    blockUpdatePathLengths(c, block, UnassignedSequenceNumber, -1, 1);
                }
            }
            free(copy.a);
        }
    }
}

/* setMinSeq (1751-1769) */
static void setMinSeq(mto_client* c, int minSeq) {
    if (!(minSeq <= c->cw.currentSeq)) FAIL(c, MTO_ERR_ASSERT);
    if (!(c->cw.minSeq <= minSeq)) FAIL(c, MTO_ERR_ASSERT);
    if (minSeq > c->cw.minSeq) {
        c->cw.minSeq = minSeq;
        zamboniSegments(c);
    }
}

/* ------------------------------------------------------------------------------------------
 * insertingWalk & friends (mergeTree.ts:2174-2522)
 * ---------------------------------------------------------------------------------------- */
enum { WALK_SPLIT = 0, WALK_INSERT = 1 };
typedef struct InsertCtx {
    int mode;
    Seg* candidate;
    int hasContinue;
} InsertCtx;

static Block UNFINISHED_NODE; /* MergeTree.theUnfinishedNode (1113) */

/* split (2509-2522) */
static Block* splitBlock(mto_client* c, Block* node) {
    int half = MaxNodesInBlock / 2;
    Block* nn = makeBlock(c, half);
    node->childCount = half;
    for (int i = 0; i < half; i++) {
        assignChild(nn, node->children[half + i], i);
        node->children[half + i] = NULL;
    }
    nodeUpdateLengthNewStructure(c, node, 0);
    nodeUpdateLengthNewStructure(c, nn, 0);
    return nn;
}

/* updateRoot (1909-1920) */
static void updateRoot(mto_client* c, Block* splitNode) {
    if (splitNode) {
        Block* nr = makeBlock(c, 2);
        nr->hdr.index = 0;
        assignChild(nr, &c->root->hdr, 0);
        assignChild(nr, &splitNode->hdr, 1);
        c->root = nr;
        nodeUpdateLengthNewStructure(c, c->root, 0);
    }
}

/* breakTie (2281-2310) */
static int breakTie(mto_client* c, int pos, Node* node, int refSeq, int clientId) {
    if (node->isLeaf) {
        if (pos == 0) {
            Seg* s = (Seg*)node;
            /* `removalInfo.removedSeq && ...`: 0 is falsy */
            if (s->hasRemoved && s->removedSeq != 0 && s->removedSeq <= refSeq &&
                s->removedSeq != UnassignedSequenceNumber)
                return 0;
            if (clientId == c->cw.clientId) return 1;
            if (s->seq != UnassignedSequenceNumber) return 1;
        }
        return 0;
    }
    return 1;
}

/* nodeMap (2936-2998) restricted to the leaf actions used on this path */
typedef int (*LeafFn)(mto_client* c, Seg* s, int pos, int refSeq, int clientId, int start, int end, void* ud);
typedef int (*PostFn)(mto_client* c, Block* b, void* ud);
static int nodeMap(mto_client* c, Block* node, LeafFn leaf, PostFn post, int pos, int refSeq, int clientId,
                   int start, int end, void* ud) {
    int go = 1;
    for (int ci = 0; ci < node->childCount; ci++) {
        Node* ch = node->children[ci];
        int len = nodeLength(c, ch, refSeq, clientId);
        if (go && end > 0 && len > 0 && start < len) {
            if (!ch->isLeaf) {
                if (go) go = nodeMap(c, (Block*)ch, leaf, post, pos, refSeq, clientId, start, end, ud);
            } else {
                go = leaf(c, (Seg*)ch, pos, refSeq, clientId, start, end, ud);
            }
        }
        if (!go) break;
        pos += len;
        start -= len;
        end -= len;
    }
    if (go && post) go = post(c, node, ud);
    return go;
}

/* checkSegmentIsLocal (2176-2185) */
static int checkSegmentIsLocal(mto_client* c, Seg* s, int pos, int refSeq, int clientId, int start, int end,
                               void* ud) {
    (void)c, (void)pos, (void)refSeq, (void)clientId, (void)start, (void)end;
    if (s->seq == UnassignedSequenceNumber) *(int*)ud = 1;
    return 0;
}
/* rightExcursion (2346-2376) with checkSegmentIsLocal; continueFrom (2187-2194) */
static int continueFrom(mto_client* c, Block* node) {
    int segIsLocal = 0;
    Node* startNode = &node->hdr;
    Block* parent = startNode->parent;
    while (parent) {
        int matched = 0;
        for (int ci = 0; ci < parent->childCount; ci++) {
            Node* n = parent->children[ci];
            if (matched) {
                int go;
                if (!n->isLeaf) {
                    go = nodeMap(c, (Block*)n, checkSegmentIsLocal, NULL, 0, UniversalSequenceNumber, c->cw.clientId,
                                 0, blockLength(c, (Block*)n, UniversalSequenceNumber, c->cw.clientId), &segIsLocal);
                } else {
                    go = checkSegmentIsLocal(c, (Seg*)n, 0, UniversalSequenceNumber, c->cw.clientId, 0, 0,
                                             &segIsLocal);
                }
                if (!go) return segIsLocal;
            } else {
                matched = (startNode == n);
            }
        }
        startNode = &parent->hdr;
        parent = parent->hdr.parent;
    }
    return segIsLocal;
}

/* insertingWalk (2378-2507) */
static Block* insertingWalk(mto_client* c, Block* block, int pos, int refSeq, int clientId, int seq,
                            InsertCtx* ctx) {
    int ci;
    Node* newNode = NULL;
    Block* fromSplit = NULL;
    for (ci = 0; ci < block->childCount; ci++) {
        Node* child = block->children[ci];
        int len = nodeLength(c, child, refSeq, clientId);
        if (pos < len || (pos == len && breakTie(c, pos, child, refSeq, clientId))) {
            if (!child->isLeaf) {
                Block* splitNode = insertingWalk(c, (Block*)child, pos, refSeq, clientId, seq, ctx);
                if (splitNode == NULL) {
                    blockUpdateLength(c, block, seq, clientId);
                    return NULL;
                } else if (splitNode == &UNFINISHED_NODE) {
                    pos -= len;
                    continue;
                } else {
                    newNode = &splitNode->hdr;
                    fromSplit = splitNode;
                    ci++;
                }
            } else {
                Seg* seg = (Seg*)child;
                if (ctx->mode == WALK_SPLIT) {
                    /* splitLeafSegment (2258-2272) */
                    Seg* next = NULL;
                    if (pos > 0) next = splitAt(c, seg, pos);
                    if (next) {
                        newNode = &next->hdr;
                        ci++;
                    } else {
                        return NULL;
                    }
                } else {
                    /* onLeaf (2213-2223): candidate replaces current, current moves after */
                    assignChild(block, &ctx->candidate->hdr, ci);
                    newNode = &seg->hdr;
                    ci++;
                }
            }
            break;
        } else {
            pos -= len;
        }
    }
    if (!newNode) {
        if (pos == 0) {
            if (seq != UnassignedSequenceNumber && ctx->hasContinue && continueFrom(c, block)) {
                return &UNFINISHED_NODE;
            } else {
                if (ctx->mode == WALK_INSERT) newNode = &ctx->candidate->hdr;
            }
        }
    }
    if (newNode) {
        for (int i = block->childCount; i > ci; i--) {
            block->children[i] = block->children[i - 1];
            block->children[i]->index = i;
        }
        assignChild(block, newNode, ci);
        block->childCount++;
        if (block->childCount < MaxNodesInBlock) {
            (void)fromSplit;
            blockUpdateLength(c, block, seq, clientId);
            return NULL;
        } else {
            return splitBlock(c, block);
        }
    }
    return NULL;
}

/* ensureIntervalBoundary (2274-2278) */
static void ensureIntervalBoundary(mto_client* c, int pos, int refSeq, int clientId) {
    InsertCtx ctx = {WALK_SPLIT, NULL, 0};
    Block* sp = insertingWalk(c, c->root, pos, refSeq, clientId, TreeMaintenanceSequenceNumber, &ctx);
    if (sp == &UNFINISHED_NODE) sp = NULL;
    updateRoot(c, sp);
}

static Group* newGroup(mto_client* c, int localSeq) {
    Group* g = xcalloc(1, sizeof(Group));
    track(c, g, 'G');
    g->localSeq = localSeq;
    return g;
}
/* addToPendingList (1955-1962) */
static Group* addToPendingList(mto_client* c, Seg* s, Group* g, int localSeq) {
    if (!g) {
        g = newGroup(c, localSeq);
        gq_push(&c->pending, g);
    }
    segGroupsEnqueue(s, g);
    return g;
}

/* blockInsert (2174-2257) of a single new segment */
static void blockInsert(mto_client* c, int pos, Seg* seg, int refSeq, int clientId, int seq, int hasLocalSeq,
                        int localSeq) {
    if (seg->hdr.cachedLength > 0) {
        seg->seq = seq;
        seg->hasLocalSeq = hasLocalSeq;
        seg->localSeq = localSeq;
        seg->clientId = clientId;
        InsertCtx ctx = {WALK_INSERT, seg, 1};
        Block* sp = insertingWalk(c, c->root, pos, refSeq, clientId, seq, &ctx);
        if (sp == &UNFINISHED_NODE) sp = NULL;
        if (seg->hdr.parent == NULL) {
            FAIL(c, MTO_ERR_INSERT_FAILED);
            return;
        }
        updateRoot(c, sp);
        /* saveIfLocal (2197-2212) */
        if (c->cw.collaborating) {
            if (seg->seq == UnassignedSequenceNumber && clientId == c->cw.clientId) {
                addToPendingList(c, seg, NULL, localSeq);
            } else if (seg->seq > c->cw.minSeq) {
                addToLRUSet(c, seg, seg->seq);
            }
        }
    }
}
static void insertSegments(mto_client* c, int pos, Seg* seg, int refSeq, int clientId, int seq) {
    ensureIntervalBoundary(c, pos, refSeq, clientId);
    int hasLocalSeq = seq == UnassignedSequenceNumber;
    int localSeq = hasLocalSeq ? ++c->cw.localSeq : 0;
    blockInsert(c, pos, seg, refSeq, clientId, seq, hasLocalSeq, localSeq);
    if (c->cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments(c);
} /* insertSegments (2001-2031) of a single new segment */

/* markRangeRemoved (2640-2752) */
typedef struct RemoveCtx {
    int clientId, seq, overwrite;
    int hasLocalSeq, localSeq;
    Group* group;
} RemoveCtx;
static int markRemoved(mto_client* c, Seg* s, int pos, int refSeq, int clientId, int start, int end, void* ud) {
    (void)pos, (void)refSeq, (void)start, (void)end;
    RemoveCtx* r = (RemoveCtx*)ud;
    if (s->hasRemoved) {
        r->overwrite = 1;
        if (s->removedSeq == UnassignedSequenceNumber) {
            s->removedClientId = clientId;
            s->removedSeq = r->seq;
            s->hasLocalRemovedSeq = 0;
        } else {
            if (s->nov >= MAX_OVERLAP)
                FAIL(c, MTO_ERR_UNSUPPORTED);
            else
                s->ov[s->nov++] = clientId; /* addOverlappingClient (2577-2585) */
        }
    } else {
        s->hasRemoved = 1;
        s->removedClientId = clientId;
        s->removedSeq = r->seq;
        s->hasLocalRemovedSeq = r->hasLocalSeq;
        s->localRemovedSeq = r->localSeq;
    }
    if (c->cw.collaborating) {
        if (s->removedSeq == UnassignedSequenceNumber && clientId == c->cw.clientId) {
            r->group = addToPendingList(c, s, r->group, r->localSeq);
        } else {
            addToLRUSet(c, s, r->seq);
        }
    }
    return 1;
}
static int afterMarkRemoved(mto_client* c, Block* b, void* ud) {
    RemoveCtx* r = (RemoveCtx*)ud;
    if (r->overwrite)
        nodeUpdateLengthNewStructure(c, b, 0);
    else
        blockUpdateLength(c, b, r->seq, r->clientId);
    return 1;
}
static void markRangeRemoved(mto_client* c, int start, int end, int refSeq, int clientId, int seq) {
    ensureIntervalBoundary(c, start, refSeq, clientId);
    ensureIntervalBoundary(c, end, refSeq, clientId);
    RemoveCtx r = {clientId, seq, 0, seq == UnassignedSequenceNumber, 0, NULL};
    if (r.hasLocalSeq) r.localSeq = ++c->cw.localSeq;
    nodeMap(c, c->root, markRemoved, afterMarkRemoved, 0, refSeq, clientId, start, end, &r);
    if (c->cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments(c);
}

/* annotateRange (2598-2638) */
typedef struct AnnotCtx {
    const mt_kv* kv;
    int nkv, rewrite, seq, localSeq;
    Group* group;
} AnnotCtx;
static int annotateSegment(mto_client* c, Seg* s, int pos, int refSeq, int clientId, int start, int end,
                           void* ud) {
    (void)pos, (void)refSeq, (void)clientId, (void)start, (void)end;
    AnnotCtx* a = (AnnotCtx*)ud;
    segAddProperties(s, a->kv, a->nkv, a->rewrite, a->seq, c->cw.collaborating);
    if (c->cw.collaborating) {
        if (a->seq == UnassignedSequenceNumber)
            a->group = addToPendingList(c, s, a->group, a->localSeq);
        else
            addToLRUSet(c, s, a->seq);
    }
    return 1;
}
static void annotateRange(mto_client* c, int start, int end, const mt_kv* kv, int nkv, int rewrite, int refSeq,
                          int clientId, int seq) {
    ensureIntervalBoundary(c, start, refSeq, clientId);
    ensureIntervalBoundary(c, end, refSeq, clientId);
    AnnotCtx a = {kv, nkv, rewrite, seq, 0, NULL};
    if (seq == UnassignedSequenceNumber) a.localSeq = ++c->cw.localSeq;
    nodeMap(c, c->root, annotateSegment, NULL, 0, refSeq, clientId, start, end, &a);
    if (c->cw.collaborating && seq != UnassignedSequenceNumber) zamboniSegments(c);
}

/* ackPendingSegment (mergeTree.ts:1926-1953) + BaseSegment.ack (486-521) */
static void ackPendingSegment(mto_client* c, int opKind, const mt_kv* kv, int nkv, int rewrite, int seq) {
    Group* g = gq_pop(&c->pending);
    Block* nodes[4096];
    int nnodes = 0;
    int overwrite = 0;
    if (g) {
        for (int i = 0; i < g->nseg; i++) {
            Seg* s = g->segs[i];
            Group* cur = gq_pop(&s->groups);
            int ok = 1;
            if (cur != g) FAIL(c, MTO_ERR_ASSERT);
            switch (opKind) {
            case MT_OP_ANNOTATE:
                if (!s->hasPM) FAIL(c, MTO_ERR_ASSERT);
                segAckPendingProperties(c, s, kv, nkv, rewrite);
                break;
            case MT_OP_INSERT:
                if (s->seq != UnassignedSequenceNumber) FAIL(c, MTO_ERR_ASSERT);
                s->seq = seq;
                s->hasLocalSeq = 0;
                break;
            case MT_OP_REMOVE:
                if (!s->hasRemoved || s->removedSeq == 0) FAIL(c, MTO_ERR_ASSERT);
                s->hasLocalRemovedSeq = 0;
                if (s->removedSeq == UnassignedSequenceNumber)
                    s->removedSeq = seq;
                else
                    ok = 0;
                break;
            default:
                FAIL(c, MTO_ERR_ASSERT);
            }
            overwrite = !ok || overwrite;
            addToLRUSet(c, s, seq);
            int found = 0;
            for (int k = 0; k < nnodes; k++)
                if (nodes[k] == s->hdr.parent) found = 1;
            if (!found && nnodes < 4096) nodes[nnodes++] = s->hdr.parent;
        }
        for (int k = 0; k < nnodes; k++) blockUpdatePathLengths(c, nodes[k], seq, c->cw.clientId, overwrite);
    }
    zamboniSegments(c);
}

/* ------------------------------------------------------------------------------------------
 * Client (client.ts)
 * ---------------------------------------------------------------------------------------- */
static void addLongClientId(mto_client* c, int longId) { /* 654-661 */
    if (c->nshort == c->shortcap) {
        c->shortcap = c->shortcap ? c->shortcap * 2 : 16;
        c->shortToLong = xrealloc(c->shortToLong, sizeof(int) * c->shortcap);
    }
    if (longId >= c->longcap) {
        int n = longId + 16;
        c->longToShort = xrealloc(c->longToShort, sizeof(int) * n);
        for (int i = c->longcap; i < n; i++) c->longToShort[i] = -1;
        c->longcap = n;
    }
    c->longToShort[longId] = c->nshort;
    c->shortToLong[c->nshort++] = longId;
}
static int getOrAddShortClientId(mto_client* c, int longId) { /* 637-642 */
    if (longId >= c->longcap || c->longToShort[longId] < 0) addLongClientId(c, longId);
    return c->longToShort[longId];
}

mto_client* mto_create(void) {
    mto_client* c = xcalloc(1, sizeof(mto_client));
    c->longClientId = -1;
    c->cw.clientId = LocalClientId;
    /* initialNode (1159-1163) */
    c->root = makeBlock(c, 0);
    c->root->hdr.cachedLength = 0;
    return c;
}
void mto_set_options(mto_client* c, int verify) { c->verify = verify; }

void mto_destroy(mto_client* c) {
    if (!c) return;
    for (int i = 0; i < c->alloc.n; i++) {
        void* p = c->alloc.p[i];
        if (c->alloc.tag[i] == 'S') {
            Seg* s = (Seg*)p;
            free(s->text);
            kv_free(&s->props);
            kv_free(&s->pendingKeys);
            free(s->groups.a);
        } else if (c->alloc.tag[i] == 'B') {
            psl_free(((Block*)p)->partialLengths);
        } else {
            free(((Group*)p)->segs);
        }
        free(p);
    }
    free(c->alloc.p);
    free(c->alloc.tag);
    free(c->pending.a);
    free(c->reload);
    free(c->scour.L);
    free(c->shortToLong);
    free(c->longToShort);
    free(c);
}

int mto_start_collab(mto_client* c, int longId, int minSeq, int curSeq) { /* 1053-1073 */
    if (c->longClientId < 0 && longId >= 0) { /* longId < 0: the replica stays detached (a snapshot load) */
        c->longClientId = longId;
        addLongClientId(c, longId);
        /* startCollaboration (mergeTree.ts:1287-1304) */
        c->cw.clientId = c->longToShort[longId];
        c->cw.minSeq = minSeq;
        c->cw.collaborating = 1;
        c->cw.currentSeq = curSeq;
        heap_init(&c->scour);
        nodeUpdateLengthNewStructure(c, c->root, 1);
    }
    return c->err;
}

static Seg* specToSegment(mto_client* c, const mt_op_rec* op) { /* textSegment.ts:31-39 / Marker.make */
    Seg* s;
    int len = (op->kind & MT_OP_KIND_MASK) >= MT_OP_RELOAD ? op->pos2 : op->text_len; /* mt_oplog.h */
    if (op->seg_kind == MT_SEG_MARKER)
        s = newSeg(c, MT_SEG_MARKER, NULL, 0, op->pos2);
    else if (op->seg_kind == MT_SEG_PERM) /* PermutationVector.insert (permutationvector.ts:147-151) */
        s = newSeg(c, MT_SEG_PERM, NULL, len, 0);
    else if (op->seg_kind == MT_SEG_RUN) /* new SubSequence(items) (SharedSequence.insert, sharedSequence.ts:116-125) */
        s = newSeg(c, MT_SEG_RUN, c->textPool + op->text_off, len, 0);
    else
        s = newSeg(c, MT_SEG_TEXT, c->textPool + op->text_off, len, 0);
    if (op->props) { /* TextSegment.make(text, props) -> addProperties(props) (no collab window) */
        const mt_props_rec* pr = &c->propsPool[op->props - 1];
        segAddProperties(s, c->kvPool + pr->kv_off, pr->nkv, pr->combining == MT_COMBINE_REWRITE, 0, 0);
        /* addProperties called without seq: seq undefined !== -1, collaborating falsy */
    }
    return s;
}

static int seqNumberLocal(mto_client* c) { /* getLocalSequenceNumber (952-960) */
    return c->cw.collaborating ? UnassignedSequenceNumber : UniversalSequenceNumber;
}

/* the MergeTree call of an edit record: insertSegments (mergeTree.ts:2001-2040), markRangeRemoved
 * (2640-2752) or annotateRange (2598-2638) */
static void applyEdit(mto_client* c, const mt_op_rec* op, int clientId, int refSeq, int seq) {
    int kind = op->kind & MT_OP_KIND_MASK;
    int start = op->pos1, end = op->pos2;
    if (kind == MT_OP_INSERT) {
        insertSegments(c, start, specToSegment(c, op), refSeq, clientId, seq);
    } else if (kind == MT_OP_REMOVE) {
        markRangeRemoved(c, start, end, refSeq, clientId, seq);
    } else if (kind == MT_OP_ANNOTATE) {
        const mt_kv* kv = NULL;
        int nkv = 0, rw = 0;
        if (op->props) {
            const mt_props_rec* pr = &c->propsPool[op->props - 1];
            kv = c->kvPool + pr->kv_off;
            nkv = pr->nkv;
            rw = pr->combining == MT_COMBINE_REWRITE;
        }
        annotateRange(c, start, end, kv, nkv, rw, refSeq, clientId, seq);
    }
}
/* applyInsertOp / applyRemoveRangeOp / applyAnnotateRangeOp (client.ts:321-442) */
static void applyOp(mto_client* c, const mt_op_rec* op, int isLocal, int clientId, int refSeq, int seq) {
    int kind = op->kind & MT_OP_KIND_MASK;
    int start = op->pos1, end = op->pos2;
    if (isLocal) { /* getValidOpRange (486-548) */
        int length = c->root->hdr.cachedLength;
        int bad = start < 0 || start > length || (start == length && kind != MT_OP_INSERT);
        if (kind != MT_OP_INSERT && end <= start) bad = 1;
        if (bad) return; /* logs InvalidOpRange and returns undefined: the op has no effect */
        /* insertSegmentLocal (202-205): an empty segment is not inserted */
        if (kind == MT_OP_INSERT && op->seg_kind != MT_SEG_MARKER && op->text_len <= 0) return;
    }
    applyEdit(c, op, clientId, refSeq, seq);
    if (!isLocal) { /* completeAndLogOp asserts (462-465) */
        if (!(c->cw.currentSeq < seq)) FAIL(c, MTO_ERR_ASSERT);
        if (!(c->cw.minSeq <= op->min_seq)) FAIL(c, MTO_ERR_ASSERT);
    }
}

/* SnapshotLoader.specToSegment (snapshotLoader.ts:96-126) for a RELOAD / APPEND record */
static Seg* loaderSegment(mto_client* c, const mt_op_rec* op) {
    Seg* s = specToSegment(c, op);
    s->clientId = op->client == MT_CLIENT_NONCOLLAB ? NonCollabClient : getOrAddShortClientId(c, op->client);
    s->seq = op->seq;
    if (op->ref_seq > 0) {
        s->hasRemoved = 1;
        s->removedSeq = op->ref_seq;
        s->removedClientId = getOrAddShortClientId(c, op->min_seq);
    }
    return s;
}
/* reloadFromSegments (mergeTree.ts:1229-1284): blocks of 7 children, built bottom-up */
static Block* buildMergeBlock(mto_client* c, Node** nodes, int n) {
    const int maxChildren = MaxNodesInBlock - 1;
    int blockCount = (n + maxChildren - 1) / maxChildren;
    Node** blocks = xmalloc(sizeof(Node*) * blockCount);
    for (int nodeIndex = 0, bi = 0; bi < blockCount; bi++) {
        Block* b = makeBlock(c, 0);
        for (int ci = 0; ci < maxChildren && nodeIndex < n; ci++, nodeIndex++) {
            int index = b->childCount++; /* addNode (1224-1227) */
            assignChild(b, nodes[nodeIndex], index);
        }
        blockUpdate(b);
        blocks[bi] = &b->hdr;
    }
    Block* r = blockCount == 1 ? (Block*)blocks[0] : buildMergeBlock(c, blocks, blockCount);
    free(blocks);
    return r;
}
static void applyLoad(mto_client* c, const mt_op_rec* op) {
    int kind = op->kind & MT_OP_KIND_MASK;
    if (kind == MT_OP_RELOAD) {
        if (c->cw.collaborating) FAIL(c, MTO_ERR_ASSERT); /* assert(!collaborating) (1231) */
        if (c->nreload == c->reloadcap) {
            c->reloadcap = c->reloadcap ? 2 * c->reloadcap : 64;
            c->reload = realloc(c->reload, sizeof(Node*) * c->reloadcap);
        }
        c->reload[c->nreload++] = &loaderSegment(c, op)->hdr;
        if (op->pos1 == 1) { /* the header's last segment: build the tree */
            c->root = buildMergeBlock(c, c->reload, c->nreload);
            c->root->hdr.parent = NULL;
            c->nreload = 0;
        }
    } else if (kind == MT_OP_COLLAB) {
        mto_start_collab(c, op->client, op->min_seq, op->seq);
    } else { /* MT_OP_APPEND: loadBody (snapshotLoader.ts:160-227) */
        Seg* s = loaderSegment(c, op);
        if (op->kind & MT_OPF_GROUPED) { /* a later member of a batch: blockInsert's insertPos (2226-2256) */
            int pos = c->loadPos;
            c->loadPos += s->hdr.cachedLength;
            blockInsert(c, pos, s, UniversalSequenceNumber, s->clientId, s->seq, 0, 0);
            /* (the batch's one zamboniSegments pass runs after its first member: with minSeq fixed
             * during a load and members never entering the LRU set, later passes find nothing) */
        } else {
            c->loadPos = c->root->hdr.cachedLength + s->hdr.cachedLength;
            insertSegments(c, c->root->hdr.cachedLength, s, UniversalSequenceNumber, s->clientId, s->seq);
        }
    }
}

int mto_apply(mto_client* c, const mt_op_rec* op, const uint16_t* text, const mt_props_rec* props,
              const mt_kv* kv) {
    if (c->err) return c->err;
    c->textPool = text;
    c->propsPool = props;
    c->kvPool = kv;
    int kind = op->kind & MT_OP_KIND_MASK;
    if (op->kind & MT_OPF_TREE) { /* a MergeTree-level call with explicit (refSeq, clientId, seq) (mt_oplog.h):
                                    * no getValidOpRange, no ack, no updateSeqNumbers */
        if (op->client == MT_CLIENT_NONCOLLAB || (op->kind & MT_OPF_LOCAL) || kind > MT_OP_ANNOTATE ||
            (kind == MT_OP_INSERT && op->seg_kind != MT_SEG_MARKER && op->text_len == 0)) {
            FAIL(c, MTO_ERR_UNSUPPORTED);
            return c->err;
        }
        int sid = op->client == MT_CLIENT_LOCAL ? LocalClientId : getOrAddShortClientId(c, op->client);
        applyEdit(c, op, sid, op->ref_seq, op->seq);
        return c->err;
    }
    if (op->kind & MT_OPF_LOCAL) {
        applyOp(c, op, 1, c->cw.clientId, c->cw.currentSeq, seqNumberLocal(c));
        return c->err;
    }
    if (kind >= MT_OP_RELOAD) {
        applyLoad(c, op);
        return c->err;
    }
    /* applyMsg (client.ts:797-819) */
    getOrAddShortClientId(c, op->client);
    if (kind != MT_OP_NOOP) {
        if ((int)op->client == c->longClientId) {
            const mt_kv* akv = NULL;
            int nkv = 0, rw = 0;
            if (op->props) {
                const mt_props_rec* pr = &c->propsPool[op->props - 1];
                akv = c->kvPool + pr->kv_off;
                nkv = pr->nkv;
                rw = pr->combining == MT_COMBINE_REWRITE;
            }
            ackPendingSegment(c, kind, akv, nkv, rw, op->seq);
        } else {
            int sid = getOrAddShortClientId(c, op->client);
            applyOp(c, op, 0, sid, op->ref_seq, op->seq);
        }
    }
    /* a group member other than the last: the message's seq update comes after its last member
     * (applyRemoteOp recursion client.ts:782-790, ackPendingSegment loop 615-622) */
    if (op->kind & MT_OPF_GROUPED) return c->err;
    /* updateSeqNumbers (821-828) */
    if (!(c->cw.currentSeq <= op->seq)) FAIL(c, MTO_ERR_ASSERT);
    c->cw.currentSeq = op->seq;
    if (!(op->min_seq <= op->seq)) FAIL(c, MTO_ERR_ASSERT);
    setMinSeq(c, op->min_seq);
    return c->err;
}

int mto_replay(mto_client* c, const mt_op_rec* ops, int64_t n, const uint16_t* text, const mt_props_rec* props,
               const mt_kv* kv) {
    for (int64_t i = 0; i < n; i++)
        if (mto_apply(c, &ops[i], text, props, kv)) return c->err;
    return c->err;
}

int mto_error(const mto_client* c) { return c->err; }
int mto_local_length(const mto_client* c) { return c->root->hdr.cachedLength; }
int mto_get_length(mto_client* c, int refSeq, int shortClient) {
    if (shortClient == -100) return c->root->hdr.cachedLength;
    return blockLength(c, c->root, refSeq, shortClient);
}
int mto_short_id(const mto_client* c, int longId) {
    if (longId < 0 || longId >= c->longcap) return -1;
    return c->longToShort[longId];
}
int mto_current_seq(const mto_client* c) { return c->cw.currentSeq; }
int mto_min_seq(const mto_client* c) { return c->cw.minSeq; }
int mto_pending_groups(const mto_client* c) { return c->pending.n; }

/* gatherText (textSegment.ts:188-275) without parallel arrays / placeholder */
typedef struct TextAcc {
    uint16_t* out;
    int64_t cap, n;
} TextAcc;
static int gatherText(mto_client* c, Seg* s, int pos, int refSeq, int clientId, int start, int end, void* ud) {
    (void)c, (void)pos, (void)refSeq, (void)clientId;
    TextAcc* a = (TextAcc*)ud;
    if (s->kind != MT_SEG_TEXT) return 1;
    int len = s->hdr.cachedLength;
    int b = 0, e = len;
    if (!(start <= 0 && end >= len)) {
        if (start < 0) start = 0;
        b = start;
        e = end >= len ? len : end;
    }
    for (int i = b; i < e; i++) {
        if (a->n < a->cap) a->out[a->n] = s->text[i];
        a->n++;
    }
    return 1;
}
int64_t mto_get_text(mto_client* c, int refSeq, int shortClient, uint16_t* out, int64_t cap) {
    int cid = shortClient == -100 ? c->cw.clientId : shortClient;
    if (shortClient == -100) refSeq = c->cw.currentSeq;
    int end = blockLength(c, c->root, refSeq, cid);
    TextAcc a = {out, cap, 0};
    nodeMap(c, c->root, gatherText, NULL, 0, refSeq, cid, 0, end, &a);
    return a.n;
}

/* ------------------------------------------------------------------------------------------
 * canonical dump (mt_oplog.h) — walkAllSegments order (mergeTree.ts:3002-3016)
 * ---------------------------------------------------------------------------------------- */
typedef struct Out {
    uint8_t* p;
    int64_t cap, n;
} Out;
static void put(Out* o, const void* src, int64_t k) {
    if (o->p && o->n + k <= o->cap) memcpy(o->p + o->n, src, k);
    o->n += k;
}
static void put32(Out* o, int32_t v) { put(o, &v, 4); }
static void put16(Out* o, uint16_t v) { put(o, &v, 2); }
static void put8(Out* o, uint8_t v) { put(o, &v, 1); }
static int isLeafBlock(Block* b) { return b->childCount == 0 || b->children[0]->isLeaf; }
static int longOf(mto_client* c, int shortId) {
    if (shortId < 0) return -1; /* getLongClientId: "original" (client.ts:646-653) */
    return c->shortToLong[shortId];
}
static void dumpWalk(mto_client* c, Block* b, Out* o, int* leafIdx, int* nsegs) {
    if (isLeafBlock(b)) {
        int li = (*leafIdx)++;
        for (int i = 0; i < b->childCount; i++) {
            Seg* s = (Seg*)b->children[i];
            (*nsegs)++;
            uint8_t flags = (s->hasProps ? MT_DF_HAS_PROPS : 0) | (s->hasRemoved ? MT_DF_REMOVED : 0) |
                            (s->hasLocalSeq ? MT_DF_LSEQ : 0) | (s->hasLocalRemovedSeq ? MT_DF_LRSEQ : 0);
            put8(o, (uint8_t)s->kind);
            put8(o, flags);
            put8(o, (uint8_t)s->nov);
            put8(o, (uint8_t)s->groups.n);
            put32(o, s->hdr.cachedLength);
            put32(o, s->seq);
            put32(o, longOf(c, s->clientId));
            put32(o, s->hasRemoved ? s->removedSeq : 0);
            put32(o, s->hasRemoved ? longOf(c, s->removedClientId) : 0);
            put32(o, s->hasLocalSeq ? s->localSeq : 0);
            put32(o, s->hasLocalRemovedSeq ? s->localRemovedSeq : 0);
            put32(o, li);
            for (int k = 0; k < s->nov; k++) put32(o, longOf(c, s->ov[k]));
            put16(o, (uint16_t)(s->hasProps ? s->props.n : 0));
            put16(o, (uint16_t)s->refType);
            if (s->hasProps)
                for (int k = 0; k < s->props.n; k++) {
                    put16(o, (uint16_t)s->props.a[k].key);
                    put16(o, (uint16_t)s->props.a[k].val);
                }
            if (s->kind == MT_SEG_TEXT || s->kind == MT_SEG_RUN) put(o, s->text, 2 * (int64_t)s->hdr.cachedLength);
        }
        return;
    }
    for (int i = 0; i < b->childCount; i++) dumpWalk(c, (Block*)b->children[i], o, leafIdx, nsegs);
}
int64_t mto_dump(mto_client* c, uint8_t* out, int64_t cap) {
    /* first pass counts segments and leaves for the header */
    Out cnt = {NULL, 0, 0};
    int nleaf = 0, nsegs = 0;
    dumpWalk(c, c->root, &cnt, &nleaf, &nsegs);
    Out o = {out, cap, 0};
    put32(&o, c->cw.currentSeq);
    put32(&o, c->cw.minSeq);
    put32(&o, c->cw.localSeq);
    put32(&o, c->root->hdr.cachedLength);
    put32(&o, nsegs);
    put32(&o, nleaf);
    int l2 = 0, s2 = 0;
    dumpWalk(c, c->root, &o, &l2, &s2);
    return o.n;
}
/* getContainingSegment (mergeTree.ts:1656-1667) through searchBlock (1830-1862) */
static Seg* searchBlock(mto_client* c, Block* b, int pos, int refSeq, int clientId, int* offOut) {
    for (int i = 0; i < b->childCount; i++) {
        Node* child = b->children[i];
        int len = nodeLength(c, child, refSeq, clientId);
        if (pos < len) {
            if (!child->isLeaf) return searchBlock(c, (Block*)child, pos, refSeq, clientId, offOut);
            *offOut = pos;
            return (Seg*)child;
        }
        pos -= len;
    }
    return NULL;
}
/* getPosition (mergeTree.ts:1619-1636) */
static int getPosition(mto_client* c, Node* node, int refSeq, int clientId) {
    int total = 0;
    Block* parent = node->parent;
    Node* prev = NULL;
    while (parent) {
        for (int i = 0; i < parent->childCount; i++) {
            Node* child = parent->children[i];
            if ((prev && child == prev) || child == node) break;
            total += nodeLength(c, child, refSeq, clientId);
        }
        prev = &parent->hdr;
        parent = parent->hdr.parent;
    }
    return total;
}
int mto_get_containing(mto_client* c, int pos, int refSeq, int shortClient, int32_t* out6) {
    int cid = shortClient;
    if (shortClient == -100) { /* Client.getContainingSegment: the local view (client.ts:1006-1008) */
        cid = c->cw.clientId;
        refSeq = c->cw.currentSeq;
    }
    int off = 0;
    Seg* s = pos >= 0 ? searchBlock(c, c->root, pos, refSeq, cid, &off) : NULL;
    for (int i = 0; i < 6; i++) out6[i] = 0;
    if (!s) return 0;
    out6[0] = 1;
    out6[1] = off;
    out6[2] = s->hdr.cachedLength;
    out6[3] = s->seq;
    out6[4] = longOf(c, s->clientId);
    out6[5] = getPosition(c, &s->hdr, refSeq, cid);
    return 1;
}

uint64_t mto_digest(mto_client* c) {
    int64_t n = mto_dump(c, NULL, 0);
    uint8_t* buf = xmalloc(n);
    mto_dump(c, buf, n);
    uint64_t h = MT_FNV_OFFSET;
    for (int64_t i = 0; i < n; i++) {
        h ^= buf[i];
        h *= MT_FNV_PRIME;
    }
    free(buf);
    return h;
}

static void statsWalk(Block* b, int depth, int* nsegs, int* nleaf, int* height, int* nlive) {
    if (isLeafBlock(b)) {
        (*nleaf)++;
        if (depth > *height) *height = depth;
        for (int i = 0; i < b->childCount; i++) {
            (*nsegs)++;
            if (!((Seg*)b->children[i])->hasRemoved) (*nlive)++;
        }
        return;
    }
    for (int i = 0; i < b->childCount; i++) statsWalk((Block*)b->children[i], depth + 1, nsegs, nleaf, height, nlive);
}
void mto_stats(mto_client* c, int* nsegs, int* nleaf, int* height, int* nlive) {
    *nsegs = *nleaf = *height = *nlive = 0;
    statsWalk(c->root, 1, nsegs, nleaf, height, nlive);
}

static int checkWalk(mto_client* c, Block* b, int refSeq, int cid) {
    int bad = 0;
    if (b->partialLengths) {
        int v = psl_getPartialLength(b->partialLengths, refSeq, cid);
        int s = sumBlockLength(c, b, refSeq, cid);
        if (v != s) bad++;
    }
    if (!isLeafBlock(b))
        for (int i = 0; i < b->childCount; i++) bad += checkWalk(c, (Block*)b->children[i], refSeq, cid);
    return bad;
}
int mto_check_partials(mto_client* c, int refSeq, int shortClient) {
    if (!c->cw.collaborating) return 0;
    return checkWalk(c, c->root, refSeq, shortClient);
}

/* ------------------------------------------------------------------------------------------
 * multi-document CPU replay (bench cpu_baseline): documents round-robin over threads
 * ---------------------------------------------------------------------------------------- */
typedef struct BatchArg {
    int tid, threads, ndocs;
    const mt_op_rec* ops;
    const int64_t* op_off;
    const uint16_t* text;
    const int64_t* text_off;
    const mt_props_rec* props;
    const int64_t* props_off;
    const mt_kv* kv;
    const int64_t* kv_off;
    const int32_t* local_long_id;
    uint64_t* digests;
    int32_t* errors;
} BatchArg;
static void* batchWorker(void* p) {
    BatchArg* a = (BatchArg*)p;
    for (int d = a->tid; d < a->ndocs; d += a->threads) {
        mto_client* c = mto_create();
        mto_start_collab(c, a->local_long_id ? a->local_long_id[d] : 0, 0, 0);
        mto_replay(c, a->ops + a->op_off[d], a->op_off[d + 1] - a->op_off[d], a->text + a->text_off[d],
                   a->props + a->props_off[d], a->kv + a->kv_off[d]);
        if (a->digests) a->digests[d] = mto_digest(c);
        if (a->errors) a->errors[d] = mto_error(c);
        mto_destroy(c);
    }
    return NULL;
}
double mto_replay_batch(int ndocs, const mt_op_rec* ops, const int64_t* op_off, const uint16_t* text,
                        const int64_t* text_off, const mt_props_rec* props, const int64_t* props_off,
                        const mt_kv* kv, const int64_t* kv_off, const int32_t* local_long_id, int threads,
                        uint64_t* digests, int32_t* errors) {
    if (threads < 1) threads = 1;
    pthread_t* th = xmalloc(sizeof(pthread_t) * threads);
    BatchArg* args = xmalloc(sizeof(BatchArg) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        args[t] = (BatchArg){t, threads, ndocs, ops, op_off, text, text_off, props, props_off,
                             kv, kv_off, local_long_id, digests, errors};
        pthread_create(&th[t], NULL, batchWorker, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(args);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
