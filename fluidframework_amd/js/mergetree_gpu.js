"use strict";
/*
 * mergetree_gpu.js — JavaScript facade over the MI355X replay engine (Node-API addon mt_napi.node ->
 * libmtreplay.so, include/mt_engine.h). It keeps the part of the reference merge-tree Client surface
 * the north star names (packages/dds/merge-tree/src/client.ts:43): startOrUpdateCollaboration,
 * applyMsg (with group ops), insertTextLocal / insertMarkerLocal / removeRangeLocal /
 * annotateRangeLocal, getLength, getText, getContainingSegment, getPosition, getCurrentSeq.
 *
 * A ReplayEngine holds a batch of documents on one GPU; engine.client(doc) is that document's
 * replica. Edits and sequenced messages are queued per document in the packed record format
 * (include/mt_oplog.h) and applied by the GPU at the next read (flush = submit + run + sync), so a
 * stream of messages costs one launch per read, not one per message. Errors the engine latches for a
 * document (insert failed, assert, invalid local range; client.ts:462-465, 527-544,
 * mergeTree.ts:2243-2249) are thrown at that document's next read, as the reference throws
 * synchronously. Node 12, CommonJS, no dependencies.
 */
const path = require("path");

const addon = require(process.env.MT_NAPI_ADDON || path.join(__dirname, "..", "build", "mt_napi.node"));

const OP = { INSERT: 0, REMOVE: 1, ANNOTATE: 2, GROUP: 3, NOOP: 4 };
const OP_REF = 3; // record kind of a local reference (include/mt_oplog.h MT_OP_REF)
const REF_REMOVE = 1; // seg_kind of an MT_OP_REF record that removes the reference (MT_REF_REMOVE)
const OPF_LOCAL = 0x80;
const OPF_GROUPED = 0x40;
const OPF_ATREF = 0x08; // insertAtReferencePositionLocal
const OPF_REGEN = 0x10; // regeneratePendingOp
const OPF_TREE = 0x20; // a MergeTree-level call with explicit (refSeq, clientId, seq)
const CLIENT_LOCAL = 0xfffe; // LocalClientId in a MergeTree-level record
const LocalClientId = -1; // constants.ts
const UnassignedSequenceNumber = -1;
const ReferenceType = { Simple: 0x0, Tile: 0x1, NestBegin: 0x2, NestEnd: 0x4, SlideOnRemove: 0x40 }; // ops.ts:6-15
const NOOP_SPLIT = 1; // seg_kind of a local NOOP record: walkSegments' splitRange (mt_oplog.h MT_NOOP_SPLIT)
const TILE_LABELS_KEY = "referenceTileLabels"; // reservedTileLabelsKey (mergeTree.ts:615)
const HANDLE_UNALLOCATED = -0x80000000; // Handle.unallocated (matrix handletable.ts:11)
const SEG = { TEXT: 0, MARKER: 1, PERM: 2, RUN: 3 }; // RUN: SubSequence items (mt_oplog.h MT_SEG_RUN)
const SEG_RELPOS = 0x80; // positions relative to markers (mt_oplog.h MT_SEG_RELPOS)
const MARKER_ID_KEY = "markerId"; // reservedMarkerIdKey
const VALUE_FALSY = 0x8000;
/* values the engine derives from incr / consensus (include/mt_oplog.h MT_VALUE_DERIVED ..) */
const VALUE_DERIVED = 0x7F00, VALUE_STRCAT0 = 0x7F00, VALUE_CONS0 = 0x7F80, VALUE_NAN = 0x7FFF;
const ERRORS = { 1: "MergeTree insert failed", 2: "assertion", 3: "invalid op range", 4: "unsupported",
    5: "capacity exceeded" };

const DEFAULT_CAPS = { ncap: 192, hcap: 256, acap: 1 << 16, mcap: 1024, gcap: 1024, ccap: 64 };

function canonical(v) {
    if (v === null || typeof v !== "object") return JSON.stringify(v);
    if (Array.isArray(v)) return "[" + v.map(canonical).join(",") + "]";
    return "{" + Object.keys(v).sort().map((k) => JSON.stringify(k) + ":" + canonical(v[k])).join(",") + "}";
}

/* batch-global property key / value tables (value id 0 = null = delete, segmentPropertiesManager.ts:102-106) */
class Interner {
    constructor() { this.keys = new Map(); this.values = new Map(); this.nk = 1; this.nv = 1; this.items = new Map(); this.itemList = []; }
    /* SubSequence items (SharedObjectSequence / SharedNumberSequence) by canonical JSON: a SubSequence row's units */
    item(v) {
        const s = canonical(v);
        let i = this.items.get(s);
        if (i === undefined) {
            if (this.itemList.length > 0xffff) throw new Error("too many distinct SubSequence items");
            i = this.itemList.length;
            this.items.set(s, i);
            this.itemList.push(v);
        }
        return i;
    }
    itemObj(i) { return this.itemList[i]; }
    key(k) {
        let i = this.keys.get(k);
        if (i === undefined) { i = this.nk++; this.keys.set(k, i); }
        return i;
    }
    value(v) {
        if (v === null || v === undefined) return 0;
        const s = canonical(v);
        let i = this.values.get(s);
        if (i === undefined) {
            if (this.nv >= VALUE_DERIVED) throw new Error("too many distinct property values");
            i = this.nv++;
            this.values.set(s, i);
        }
        const falsy = typeof v !== "object" && !v;
        return i | (falsy ? VALUE_FALSY : 0);
    }
    /* include/mt_oplog.h MT_VKIND_* per value id (mt_engine_set_value_kinds): what an incr annotate makes of it */
    kinds() {
        const k = new Uint8Array(this.nv);
        for (const [sv, i] of this.values) {
            const v = JSON.parse(sv);
            k[i] = typeof v === "number" || typeof v === "boolean" ? 1 : typeof v === "string" ? 2 : 0;
        }
        return k;
    }
}

/* MergeTreeDeltaType / MergeTreeMaintenanceType names of the delta stream's op words (include/mt_oplog.h) */
const DELTA_OPS = { 0: "INSERT", 1: "REMOVE", 2: "ANNOTATE", 3: "REGEN", "-1": "APPEND", "-2": "SPLIT", "-3": "UNLINK" };

/* Decode a document's delta-stream words (include/mt_oplog.h MT_DELTA_*) into the events a SharedString
 * "sequenceDelta" (INSERT / REMOVE / ANNOTATE) or "maintenance" (APPEND / SPLIT / UNLINK) listener
 * receives (sequence.ts:136-150; SequenceDeltaEvent.ranges, sequenceDeltaEvent.ts:40-50): per event the
 * operation, the seq of the message (-1: local edit) and per delta segment its position (delta events),
 * length and propertyDeltas (annotate). */
function decodeDeltas(words, interner) {
    const END = -0x80000000; // MT_DELTA_END: no position or length takes this value
    const keyName = new Map([...interner.keys].map(([k, i]) => [i, k]));
    const valueOf = new Map([...interner.values].map(([v, i]) => [i, JSON.parse(v)]));
    const events = [];
    const n = words.length;
    const need = (k) => { if (i + k > n) throw new Error(`truncated delta stream at word ${i} of ${n}`); };
    let i = 0;
    while (i < n) {
        need(2);
        const op = words[i], seq = words[i + 1];
        i += 2;
        const deltaSegments = [];
        for (;;) {
            need(1);
            if (words[i] === END) break;
            need(3);
            const pos = words[i], length = words[i + 1], nd = words[i + 2];
            i += 3;
            const seg = { position: pos < 0 ? undefined : pos, length };
            if (op === 3) seg.opType = nd; // REGEN: the regenerated op's type
            if (op === 2) {
                if (nd < 0) {
                    seg.propertyDeltas = undefined; // addProperties was blocked by pending local rewrites
                } else {
                    seg.propertyDeltas = {};
                    need(nd);
                    for (let k = 0; k < nd; k++, i++) {
                        const w = words[i] >>> 0, v = w & 0xffff;
                        seg.propertyDeltas[keyName.get(w >>> 16)] = v === 0 ? null : valueOf.get(v & ~VALUE_FALSY);
                    }
                }
            }
            deltaSegments.push(seg);
        }
        need(2);
        if (words[i + 1] !== deltaSegments.length) throw new Error(`malformed delta stream at word ${i}`);
        i += 2;
        events.push({ operation: DELTA_OPS[op], seq, deltaSegments });
    }
    return events;
}

/* The canonical segment dump (include/mt_oplog.h) as the reference's segment objects: per segment its type,
 * cachedLength, seq / clientId (long client names; LocalClientId = -1), removedSeq / removedClientId
 * (undefined when not removed), localSeq / localRemovedSeq, properties, text / refType / start, the leaf block
 * ordinal and its index (ordinal) in walkAllSegments order. */
function decodeDump(bytes, interner, nameOf) {
    const TYPES = ["TextSegment", "Marker", "PermutationSegment", "SubSequence"];
    const dv = new DataView(bytes.buffer, bytes.byteOffset, bytes.byteLength);
    const keyName = new Map([...interner.keys].map(([k, i]) => [i, k]));
    const valueOf = new Map([...interner.values].map(([v, i]) => [i, JSON.parse(v)]));
    const hdr = [0, 1, 2, 3, 4, 5].map((k) => dv.getInt32(4 * k, true));
    let o = 24;
    const segments = [];
    for (let i = 0; i < hdr[4]; i++) {
        const kind = dv.getUint8(o), flags = dv.getUint8(o + 1), nov = dv.getUint8(o + 2);
        o += 4;
        const f = [0, 1, 2, 3, 4, 5, 6, 7].map((k) => dv.getInt32(o + 4 * k, true));
        o += 32 + 4 * nov;
        const np = dv.getUint16(o, true), refType = dv.getUint16(o + 2, true);
        o += 4;
        let properties;
        const pairs = [];
        for (let k = 0; k < np; k++) pairs.push([dv.getUint16(o + 4 * k, true), dv.getUint16(o + 4 * k + 2, true)]);
        o += 4 * np;
        if (flags & 1) {
            properties = {};
            for (const [key, raw] of pairs) {
                let val;
                if (raw === VALUE_NAN) {
                    val = NaN;
                } else if (raw === VALUE_STRCAT0 || raw === VALUE_CONS0) { // contents follow the pairs (mt_oplog.h)
                    const a = dv.getInt32(o, true), b = dv.getInt32(o + 4, true);
                    o += 8;
                    val = raw === VALUE_CONS0 ? { value: undefined, seq: a }
                        : (a === 0 ? "[object Object]" : String(valueOf.get(a & ~VALUE_FALSY))) + "undefined".repeat(b);
                } else {
                    const v = raw & ~VALUE_FALSY;
                    val = v === 0 ? null : valueOf.get(v);
                }
                properties[keyName.get(key)] = val;
            }
        }
        let start = HANDLE_UNALLOCATED;
        if (flags & 16) { start = dv.getInt32(o, true); o += 4; }
        const seg = {
            type: TYPES[kind],
            cachedLength: f[0], seq: f[1], clientId: nameOf(f[2]),
            removedSeq: flags & 2 ? f[3] : undefined, removedClientId: flags & 2 ? nameOf(f[4]) : undefined,
            localSeq: flags & 4 ? f[5] : undefined, localRemovedSeq: flags & 8 ? f[6] : undefined,
            properties, leaf: f[7], ordinal: i,
        };
        if (kind === SEG.TEXT) {
            let t = "";
            for (let j = 0; j < f[0]; j++) t += String.fromCharCode(dv.getUint16(o + 2 * j, true));
            o += 2 * f[0];
            seg.text = t;
        } else if (kind === SEG.RUN) { // SubSequence.items
            seg.items = [];
            for (let j = 0; j < f[0]; j++) seg.items.push(interner.itemObj(dv.getUint16(o + 2 * j, true)));
            o += 2 * f[0];
        } else if (kind === SEG.MARKER) {
            seg.refType = refType;
        } else {
            seg.start = start;
        }
        segments.push(seg);
    }
    return { currentSeq: hdr[0], minSeq: hdr[1], localSeq: hdr[2], length: hdr[3], nleaf: hdr[5], segments };
}

/* a marker's tile labels as Marker.hasTileLabel reads them (mergeTree.ts:620-635: Tile refType and the
 * referenceTileLabels property) */
function hasTileLabel(seg, label) {
    if (seg.type !== "Marker" || !(seg.refType & ReferenceType.Tile) || !seg.properties) return false;
    const labels = seg.properties[TILE_LABELS_KEY];
    return Array.isArray(labels) && labels.includes(label);
}

class DocQueue {
    constructor() { this.recs = []; this.text = []; this.props = []; this.kv = []; }
}

class ReplayEngine {
    constructor(ndocs, caps = DEFAULT_CAPS, device = 0) {
        this.h = addon.create(device, ndocs, caps);
        this.ndocs = ndocs;
        this.interner = new Interner();
        this.clientIds = new Map(); // long client id (string) -> engine long-client index
        this.queues = Array.from({ length: ndocs }, () => new DocQueue());
        this.localNames = new Array(ndocs).fill(undefined);
        this.collab = false;
        this.currentSeq = new Array(ndocs).fill(0);
        this.nrefs = new Array(ndocs).fill(0);   // local references created per document
        this.pending = Array.from({ length: ndocs }, () => []); // op types in flight, per pending group
        this.version = 0; // bumped by every enqueued record and every collaboration start: cached reads expire
        this.dirty = new Set(); // documents with queued records
        this.kindsSent = 0; // interner values whose kinds the engine has
    }

    longIndex(name) {
        let i = this.clientIds.get(name);
        if (i === undefined) { i = this.clientIds.size; this.clientIds.set(name, i); }
        return i;
    }

    client(doc) { return new GpuClient(this, doc); }

    /* startOrUpdateCollaboration for every document at once (client.ts:1053-1073; mt_engine_start_collab_docs):
     * minSeq / currentSeq are one number for every document or an array with one per document */
    startCollaboration(localNames, minSeq = 0, currentSeq = 0) {
        this.flush(); // edits queued before collaboration apply as non-collaborating local edits
        const ids = new Int32Array(this.ndocs);
        const per = (x) => Int32Array.from({ length: this.ndocs }, (_, d) => (Array.isArray(x) || ArrayBuffer.isView(x) ? x[d] : x));
        const mins = per(minSeq), curs = per(currentSeq);
        for (let d = 0; d < this.ndocs; d++) {
            this.localNames[d] = localNames[d];
            ids[d] = this.longIndex(localNames[d]);
            this.currentSeq[d] = curs[d];
        }
        addon.startCollab(this.h, ids, mins, curs);
        this.collab = true;
        this.version++;
    }

    enqueue(doc, kind, fields, segOrProps) {
        this.version++;
        this.dirty.add(doc);
        const q = this.queues[doc];
        const r = { kind, seg_kind: 0, client: 0, seq: 0, ref_seq: 0, min_seq: 0, pos1: 0, pos2: 0, text_off: 0,
            text_len: 0, props: 0, ...fields };
        const k = kind & 7;
        if (kind & OPF_REGEN) {
            // regeneratePendingOp: the record names only the pending op's type
        } else if (k === OP.INSERT) {
            const seg = segOrProps;
            let props;
            if (typeof seg === "string") {
                r.text_off = q.text.length; r.text_len = seg.length;
                for (let i = 0; i < seg.length; i++) q.text.push(seg.charCodeAt(i));
            } else if (Array.isArray(seg)) { // PermutationSegment [length, start] (permutationvector.ts:40-43, 75-77)
                r.seg_kind = SEG.PERM; r.text_len = seg[0];
            } else if (seg && seg.marker) {
                r.seg_kind = SEG.MARKER; r.pos2 = seg.marker.refType; props = seg.props;
            } else if (seg && typeof seg.text === "string") {
                r.text_off = q.text.length; r.text_len = seg.text.length; props = seg.props;
                for (let i = 0; i < seg.text.length; i++) q.text.push(seg.text.charCodeAt(i));
            } else if (seg && Array.isArray(seg.items)) { // SubSequence {items, props} (sharedSequence.ts:23-47)
                r.seg_kind = SEG.RUN; r.text_off = q.text.length; r.text_len = seg.items.length; props = seg.props;
                for (const v of seg.items) q.text.push(this.interner.item(v));
            } else {
                throw new Error("unsupported segment spec");
            }
            if (props) r.props = this.propsRecord(q, props, undefined);
        } else if (k === OP.ANNOTATE) {
            r.props = this.propsRecord(q, segOrProps.props, segOrProps.combiningOp);
        }
        if (fields.rel1 || fields.rel2) { // IRelativePosition(s): the spec follows the record's text (mt_oplog.h MT_SEG_RELPOS)
            delete r.rel1; delete r.rel2;
            if (!(k === OP.INSERT && (r.seg_kind === SEG.TEXT || r.seg_kind === SEG.RUN))) { r.text_off = q.text.length; r.text_len = 0; }
            q.text.push(this.interner.key(MARKER_ID_KEY), (fields.rel1 ? 1 : 0) | (fields.rel2 ? 2 : 0));
            for (const rp of [fields.rel1, fields.rel2]) {
                if (!rp) { q.text.push(0, 0, 0, 0); continue; }
                if (typeof rp.id !== "string") throw new Error("a relative position needs a marker id");
                const off = rp.offset === undefined ? 0 : rp.offset >>> 0;
                q.text.push(this.interner.value(rp.id) & 0xffff, (rp.before ? 1 : 0) | (rp.offset === undefined ? 0 : 2),
                    off & 0xffff, off >>> 16);
            }
            r.seg_kind |= SEG_RELPOS;
        }
        q.recs.push(r);
    }

    propsRecord(q, props, combiningOp) {
        const off = q.kv.length;
        const keys = Object.keys(props);
        for (const k of keys) q.kv.push([this.interner.key(k), this.interner.value(props[k])]);
        // ICombiningOp -> mt_oplog.h MT_COMBINE_*: rewrite 1, incr 2, consensus 3 (without defaultValue / minValue)
        const COMB = new Map([["rewrite", 1], ["incr", 2], ["consensus", 3]]);
        // combine() starts from any defaultValue that is not undefined (null included) and clamps only to a truthy
        // minValue (properties.ts:26-38); wire.py refuses the same ones
        if (combiningOp && (!COMB.has(combiningOp.name) ||
            (combiningOp.name !== "rewrite" && (combiningOp.defaultValue !== undefined || combiningOp.minValue)))) {
            throw new Error(`combiningOp ${combiningOp.name} unsupported`);
        }
        q.props.push([off, keys.length, combiningOp ? COMB.get(combiningOp.name) : 0]);
        return q.props.length;
    }

    /* submit the queued events of the documents that have any (mt_engine_submit_docs: the others are not staged and
     * their workgroups are not launched), replay them on the GPU, wait */
    flush() {
        const dirty = [];
        for (const d of this.dirty) if (this.queues[d].recs.length) dirty.push(d);
        this.dirty.clear();
        if (dirty.length === 0) return;
        dirty.sort((a, b) => a - b);
        let nrec = 0, ntext = 0, nprops = 0, nkv = 0;
        for (const d of dirty) {
            const q = this.queues[d];
            nrec += q.recs.length; ntext += q.text.length; nprops += q.props.length; nkv += q.kv.length;
        }
        const m = dirty.length;
        const docs = BigInt64Array.from(dirty, (d) => BigInt(d));
        const ops = new Uint8Array(32 * nrec), dv = new DataView(ops.buffer);
        const text = new Uint16Array(Math.max(ntext, 1));
        const props = new Uint8Array(8 * Math.max(nprops, 1)), pv = new DataView(props.buffer);
        const kv = new Uint8Array(4 * Math.max(nkv, 1)), kvv = new DataView(kv.buffer);
        const opOff = new BigInt64Array(m + 1), textOff = new BigInt64Array(m + 1);
        const propsOff = new BigInt64Array(m + 1), kvOff = new BigInt64Array(m + 1);
        let ro = 0, to = 0, po = 0, ko = 0;
        dirty.forEach((doc, d) => {
            const q = this.queues[doc];
            opOff[d] = BigInt(ro); textOff[d] = BigInt(to); propsOff[d] = BigInt(po); kvOff[d] = BigInt(ko);
            for (const r of q.recs) {
                const b = 32 * ro++;
                dv.setUint8(b, r.kind); dv.setUint8(b + 1, r.seg_kind); dv.setUint16(b + 2, r.client, true);
                dv.setInt32(b + 4, r.seq, true); dv.setInt32(b + 8, r.ref_seq, true); dv.setInt32(b + 12, r.min_seq, true);
                dv.setInt32(b + 16, r.pos1, true); dv.setInt32(b + 20, r.pos2, true); dv.setUint32(b + 24, r.text_off, true);
                dv.setUint16(b + 28, r.text_len, true); dv.setUint16(b + 30, r.props, true);
            }
            text.set(q.text, to); to += q.text.length;
            for (const [off, n, comb] of q.props) {
                pv.setUint32(8 * po, off, true); pv.setUint16(8 * po + 4, n, true); pv.setUint8(8 * po + 6, comb); po++;
            }
            for (const [k, v] of q.kv) { kvv.setUint16(4 * ko, k, true); kvv.setUint16(4 * ko + 2, v, true); ko++; }
            q.recs = []; q.text = []; q.props = []; q.kv = [];
        });
        opOff[m] = BigInt(ro); textOff[m] = BigInt(to);
        propsOff[m] = BigInt(po); kvOff[m] = BigInt(ko);
        if (this.interner.nv !== this.kindsSent) { // the value kinds an incr annotate needs (mt_engine_set_value_kinds)
            addon.setValueKinds(this.h, this.interner.kinds());
            this.kindsSent = this.interner.nv;
        }
        addon.submitDocs(this.h, docs, ops, opOff, text, textOff, props, propsOff, kv, kvOff);
        addon.run(this.h);
        addon.sync(this.h);
    }

    /* the document's latched error, read alone (8 bytes) */
    checkDoc(doc) {
        const [err, errOp] = addon.docError(this.h, doc);
        if (err !== 0) throw new Error(`document ${doc}: ${ERRORS[err] || err} at event ${errOp}`);
    }

    digests() { this.flush(); return addon.digests(this.h); }
}

/* The MergeTree-level calls of one replica with explicit (refSeq, clientId, seq) (mergeTree.ts:2001-2031,
 * 2598-2738; mt_oplog.h MT_OPF_TREE): what applyRemoteOp and the local edits call underneath. clientId is a
 * long client id (string) or LocalClientId; seq UnassignedSequenceNumber makes a local pending op. They do
 * not touch the collaboration window (no ack, no getValidOpRange, no updateSeqNumbers). */
class GpuMergeTree {
    constructor(client) { this.client = client; }

    fields(refSeq, clientId, seq) {
        const e = this.client.engine;
        return { ref_seq: refSeq, seq, client: clientId === LocalClientId ? CLIENT_LOCAL : e.longIndex(clientId) };
    }

    /* one segment per call: a string, {text, props} or {marker: {refType}, props} */
    insertSegments(pos, segments, refSeq, clientId, seq) {
        if (!Array.isArray(segments) || segments.length !== 1) throw new Error("insertSegments: one segment per call");
        const c = this.client;
        c.engine.enqueue(c.doc, OP.INSERT | OPF_TREE, { ...this.fields(refSeq, clientId, seq), pos1: pos }, segments[0]);
        if (seq === UnassignedSequenceNumber) c.sent(OP.INSERT);
    }

    markRangeRemoved(start, end, refSeq, clientId, seq, overwrite = false) {
        if (overwrite) throw new Error("markRangeRemoved: overwrite = true is not modelled");
        const c = this.client;
        c.engine.enqueue(c.doc, OP.REMOVE | OPF_TREE, { ...this.fields(refSeq, clientId, seq), pos1: start, pos2: end });
        if (seq === UnassignedSequenceNumber) c.sent(OP.REMOVE);
    }

    annotateRange(start, end, props, combiningOp, refSeq, clientId, seq) {
        const c = this.client;
        c.engine.enqueue(c.doc, OP.ANNOTATE | OPF_TREE, { ...this.fields(refSeq, clientId, seq), pos1: start, pos2: end },
            { props, combiningOp });
        if (seq === UnassignedSequenceNumber) c.sent(OP.ANNOTATE);
    }
}

/* one replica: the reference Client's surface (client.ts:43) */
class GpuClient {
    constructor(engine, doc) { this.engine = engine; this.doc = doc; this.mergeTree = new GpuMergeTree(this); }

    get longClientId() { return this.engine.localNames[this.doc]; }

    getCurrentSeq() { return this.engine.currentSeq[this.doc]; }

    /* Client.applyMsg (client.ts:797-819): group ops become GROUPED member records (mt_oplog.h) */
    applyMsg(msg) {
        const e = this.engine;
        const base = { client: e.longIndex(msg.clientId), seq: msg.sequenceNumber,
            ref_seq: msg.referenceSequenceNumber, min_seq: msg.minimumSequenceNumber };
        if (msg.type !== "op") {
            e.enqueue(this.doc, OP.NOOP, base);
        } else {
            const op = msg.contents;
            const members = op.type === OP.GROUP ? op.ops : [op];
            members.forEach((m, i) => {
                const flag = i < members.length - 1 ? OPF_GROUPED : 0;
                // getValidOpRange (client.ts:486-503): a relative position where the absolute one is undefined
                const rel1 = m.pos1 === undefined ? m.relativePos1 : undefined;
                const rel2 = m.pos2 === undefined ? m.relativePos2 : undefined;
                const pos = { pos1: rel1 ? 0 : m.pos1, pos2: rel2 ? 0 : m.pos2, rel1, rel2 };
                if (m.type === OP.INSERT) e.enqueue(this.doc, OP.INSERT | flag, { ...base, pos1: pos.pos1, rel1 }, m.seg);
                else if (m.type === OP.REMOVE) e.enqueue(this.doc, OP.REMOVE | flag, { ...base, ...pos });
                else if (m.type === OP.ANNOTATE) {
                    e.enqueue(this.doc, OP.ANNOTATE | flag, { ...base, ...pos }, m);
                } else throw new Error(`op type ${m.type} unsupported`);
            });
        }
        if (msg.type === "op" && msg.clientId === this.longClientId) { // an ack: its groups leave the queue
            const n = msg.contents.type === OP.GROUP ? msg.contents.ops.length : 1;
            e.pending[this.doc].splice(0, n);
        }
        e.currentSeq[this.doc] = msg.sequenceNumber;
    }

    /* local edits (client.ts:164-211): return the op to submit, as the reference does. The facade keeps
     * the type of each op in flight (one per segment group) for regeneratePendingOp; the engine rejects
     * an invalid local range as the reference does, so callers submit only ops of valid ranges. */
    insertTextLocal(pos, text, props) {
        if (text.length === 0) return undefined;
        const seg = props ? { text, props } : text;
        this.engine.enqueue(this.doc, OP.INSERT | OPF_LOCAL, { pos1: pos }, seg);
        this.sent(OP.INSERT);
        return { type: OP.INSERT, pos1: pos, seg };
    }

    sent(type) { if (this.engine.collab) this.engine.pending[this.doc].push(type); }

    insertMarkerLocal(pos, refType, props) {
        const seg = { marker: { refType } };
        if (props) seg.props = props;
        this.engine.enqueue(this.doc, OP.INSERT | OPF_LOCAL, { pos1: pos }, seg);
        this.sent(OP.INSERT);
        return { type: OP.INSERT, pos1: pos, seg };
    }

    removeRangeLocal(start, end) {
        this.engine.enqueue(this.doc, OP.REMOVE | OPF_LOCAL, { pos1: start, pos2: end });
        this.sent(OP.REMOVE);
        return { type: OP.REMOVE, pos1: start, pos2: end };
    }

    annotateRangeLocal(start, end, props, combiningOp) {
        const op = { type: OP.ANNOTATE, pos1: start, pos2: end, props };
        if (combiningOp) op.combiningOp = combiningOp;
        this.engine.enqueue(this.doc, OP.ANNOTATE | OPF_LOCAL, { pos1: start, pos2: end }, op);
        this.sent(OP.ANNOTATE);
        return op;
    }

    /* new LocalReference + Client.addLocalReference at getContainingSegment(pos) (client.ts:295,
     * localReference.ts:20-117); engines need caps.rcap > 0. Returns the reference's handle. */
    createLocalReference(pos, refType = ReferenceType.SlideOnRemove) {
        this.engine.enqueue(this.doc, OP_REF | OPF_LOCAL, { pos1: pos, pos2: refType });
        return { doc: this.doc, index: this.engine.nrefs[this.doc]++ };
    }

    /* Client.removeLocalReference (client.ts:299-301 -> LocalReferenceCollection.removeLocalRef,
     * localReference.ts:225-264): the reference leaves its segment's collection and stops following splits,
     * appends and slides; it keeps its segment and offset (localReferencePosition still answers, -1 once that
     * segment leaves the tree). A detached reference's removal throws in the reference: a no-op here. */
    removeLocalReference(ref) {
        this.engine.enqueue(this.doc, OP_REF | OPF_LOCAL, { pos1: ref.index, seg_kind: REF_REMOVE });
    }

    /* LocalReference.toPosition() (localReference.ts:62-68): -1 detached. A reference whose creation the
     * reference's Client.addLocalReference would have thrown on (its offset holds only slid references,
     * localReference.ts:195-201) throws here, at its first read, as the reference throws at creation. */
    localReferencePosition(ref) {
        const [n, pos] = addon.refPositions(this.read());
        const rcap = pos.length / this.engine.ndocs;
        const p = ref.index < n[this.doc] ? pos[this.doc * rcap + ref.index] : -1;
        if (p === -2) throw new Error("addLocalReference: the offset's reference list is undefined");
        return p;
    }

    /* Client.insertAtReferencePositionLocal (client.ts:217-245) */
    insertAtReferencePositionLocal(ref, text) {
        this.engine.enqueue(this.doc, OP.INSERT | OPF_LOCAL | OPF_ATREF, { pos1: ref.index }, text);
        this.sent(OP.INSERT);
    }

    /* Client.regeneratePendingOp for every op in flight, in order (client.ts:855-893; what a
     * SharedSegmentSequence does on reconnect). The regenerated ops come back in deltaEvents() as
     * "REGEN" events; the acks of the resubmitted messages carry one member per regenerated op. */
    regeneratePendingOps() {
        const e = this.engine;
        const q = e.pending[this.doc];
        if (q.length === 0) return [];
        const before = addon.deltas(this.read(), this.doc).length; // the events logged before these records
        for (const type of q) e.enqueue(this.doc, type | OPF_LOCAL | OPF_REGEN, {});
        const words = addon.deltas(this.read(), this.doc);
        const regen = decodeDeltas(words.subarray(before), e.interner).filter((ev) => ev.operation === "REGEN");
        if (regen.length !== q.length) throw new Error("regeneratePendingOps needs an engine with caps.dcap > 0");
        const ops = [];
        for (const ev of regen) for (const sg of ev.deltaSegments) ops.push({ type: sg.opType, pos1: sg.position, length: sg.length });
        e.pending[this.doc] = ops.map((o) => o.type);
        return ops; // per regenerated op: type, findReconnectionPostition, the segment's length
    }

    /* Client.posFromRelativePos (client.ts:308, mergeTree.ts:1976-1999) in the local view: the position
     * before / after the marker whose "markerId" is relativePos.id (+/- offset); -1 if no marker holds it */
    posFromRelativePos(relativePos) {
        const e = this.engine;
        const h = this.read();
        const off = relativePos.offset;
        return addon.posFromRelativePos(h, this.doc, e.interner.key(MARKER_ID_KEY), e.interner.value(relativePos.id) & 0xffff,
            relativePos.before ? 1 : 0, off === undefined ? 0 : 1, off === undefined ? 0 : off, 0, -1);
    }

    /* SharedString.insertTextRelative / insertMarkerRelative (sharedString.ts:86-140) */
    insertTextRelative(relativePos1, text, props) { return this.insertTextLocal(this.posFromRelativePos(relativePos1), text, props); }

    insertMarkerRelative(relativePos1, refType, props) {
        return this.insertMarkerLocal(this.posFromRelativePos(relativePos1), refType, props);
    }

    /* PermutationVector (engines created with caps.pcap > 0; permutationvector.ts:157-183, 338-363):
     * getAllocatedHandle(pos) queues the allocation (a local record) and answers the handle at the next read;
     * getMaybeHandle(pos) reads it (Handle.unallocated = -2^31 when the row has none); handleTable() is
     * HandleTable.snapshot(). Zamboni's unlinks free handles as the reference's onMaintenance does. */
    getAllocatedHandle(pos) {
        this.engine.enqueue(this.doc, OP.NOOP | OPF_LOCAL, { pos1: pos });
        return this.getMaybeHandle(pos);
    }

    getMaybeHandle(pos) { return addon.getHandle(this.read(), this.doc, pos); }

    handleTable() { return addon.handleTable(this.read(), this.doc); }

    /* reads flush the queued events first */
    read() { this.engine.flush(); this.engine.checkDoc(this.doc); return this.engine.h; }

    getLength() { return addon.getLength(this.read(), this.doc, 0, -1); }

    /* SharedString.getText(start?, end?) (sequence/src/sharedString.ts:222-225): the local view */
    getText(start, end) { return addon.getText(this.read(), this.doc, 0, -1, "", start, end); }

    /* SharedString.getTextWithPlaceholders / getTextRangeWithPlaceholders (sharedString.ts:228-236): every
     * marker (or other non-text segment) as " " */
    getTextWithPlaceholders(start, end) { return addon.getText(this.read(), this.doc, 0, -1, " ", start, end); }

    /* MergeTree.getLength / getText under (refSeq, clientId) (mergeTree.ts:1610, textSegment.ts:154) */
    getLengthAt(refSeq, longClientId) { return addon.getLength(this.read(), this.doc, refSeq, this.engine.longIndex(longClientId)); }

    /* MergeTreeTextHelper.getText(refSeq, clientId, placeholder, start, end) (textSegment.ts:154-186); the
     * placeholder "*" (Marker.toString() per marker) is not supported and throws */
    getTextAt(refSeq, longClientId, placeholder = "", start, end) {
        return addon.getText(this.read(), this.doc, refSeq, this.engine.longIndex(longClientId), placeholder, start, end);
    }

    /* Client.getContainingSegment (client.ts:1006-1008): {segment: handle | undefined, offset} */
    getContainingSegment(pos) {
        const r = addon.getContainingSegment(this.read(), this.doc, pos, 0, -1);
        return r === undefined ? { segment: undefined, offset: undefined } : { segment: r, offset: r.offset };
    }

    /* Client.getPosition (client.ts:291) of a handle from getContainingSegment */
    getPosition(segment) { return addon.getPosition(this.read(), this.doc, segment.rid, segment.gen, 0, -1); }

    /* The replica's segments in walkAllSegments order (decodeDump), each with its handle (rid, gen: getPosition
     * and getContainingSegment's handles) and its position in the local view (pos; localNetLength in len) */
    segments() {
        /* decoded once per replica state: every read of it (walkSegments, findTile, getPropertiesAtPosition,
         * getMarkerFromId, ...) reuses the decode until the next enqueued record (ADVICE r4) */
        const e = this.engine;
        if (this._seg && this._segVersion === e.version) return this._seg;
        const d = this._decodeSegments();
        this._seg = d;
        this._segVersion = e.version;
        return d;
    }

    _decodeSegments() {
        const h = this.read();
        const names = [...this.engine.clientIds.keys()];
        const d = decodeDump(addon.dump(h, this.doc), this.engine.interner, (i) => (i < 0 ? LocalClientId : names[i]));
        const ids = addon.segmentIds(h, this.doc);
        let pos = 0;
        d.segments.forEach((seg, i) => {
            seg.rid = ids[2 * i];
            seg.gen = ids[2 * i + 1];
            seg.pos = pos;
            seg.len = seg.removedSeq !== undefined ? 0 : seg.cachedLength; // localNetLength
            pos += seg.len;
        });
        d.localLength = pos;
        return d;
    }

    /* Client.walkSegments(handler, start, end, accum, splitRange) (client.ts:276-285 -> MergeTree.mapRange /
     * nodeMap, mergeTree.ts:2830-2998): handler(segment, pos, refSeq, clientId, start, end, accum) for every
     * segment of the local view with a length, inside [start, end), in order, start / end relative to the
     * segment; a falsy return stops the walk. splitRange first splits the segments at start and end (a local
     * record; engines with caps.dcap, rcap or pcap > 0). Segments are the objects segments() returns. */
    walkSegments(handler, start, end, accum, splitRange = false) {
        if (splitRange) this.engine.enqueue(this.doc, OP.NOOP | OPF_LOCAL, { seg_kind: NOOP_SPLIT, pos1: start || 0, pos2: end || 0 });
        const d = this.segments();
        let a = start === undefined ? 0 : start, b = end === undefined ? d.localLength : end;
        for (const seg of d.segments) {
            if (b > 0 && seg.len > 0 && a < seg.len) {
                if (!handler(seg, seg.pos, d.currentSeq, this.longClientId, a, b, accum)) break;
            }
            a -= seg.len;
            b -= seg.len;
        }
    }

    /* Client.getPropertiesAtPosition (client.ts:1011-1025): the properties of the segment at pos (local view) */
    getPropertiesAtPosition(pos) {
        const r = addon.getContainingSegment(this.read(), this.doc, pos, 0, -1);
        if (r === undefined) return undefined;
        return this.segments().segments[r.ordinal].properties;
    }

    /* Client.getRangeExtentsOfPosition (client.ts:1026-1044): {posStart, posAfterEnd} of the segment at pos */
    getRangeExtentsOfPosition(pos) {
        const { segment } = this.getContainingSegment(pos);
        if (segment === undefined) return { posStart: undefined, posAfterEnd: undefined };
        const posStart = this.getPosition(segment);
        return { posStart, posAfterEnd: posStart + segment.length };
    }

    /* MergeTree.resolveRemoteClientPosition (mergeTree.ts:2140-2160; SharedSegmentSequence.resolveRemoteClientPosition,
     * sequence.ts:314): where a remote client's position (under its refSeq) is in the local view; undefined if
     * nothing there. A perspective the engine does not answer (mt_engine.h) throws "unsupported". */
    resolveRemoteClientPosition(remoteClientPosition, remoteClientRefSeq, remoteLongClientId) {
        return addon.resolveRemoteClientPosition(this.read(), this.doc, remoteClientPosition, remoteClientRefSeq,
            this.engine.longIndex(remoteLongClientId));
    }

    /* Client.localTransaction(groupOp) (client.ts:961-981): every member applied as a local op */
    localTransaction(groupOp) {
        for (const op of groupOp.ops) {
            if (op.pos1 === undefined || (op.type !== OP.INSERT && op.pos2 === undefined)) {
                throw new Error("localTransaction: relative positions are not modelled for local ops");
            }
            if (op.type === OP.INSERT) this.insertSegmentLocal(op.pos1, op.seg);
            else if (op.type === OP.REMOVE) this.removeRangeLocal(op.pos1, op.pos2);
            else if (op.type === OP.ANNOTATE) this.annotateRangeLocal(op.pos1, op.pos2, op.props, op.combiningOp);
        }
    }

    /* SharedSequence.insert(pos, items, props) (sequence sharedSequence.ts:116-125): a SubSequence of the items
     * (interned; a SharedObjectSequence / SharedNumberSequence document holds no TextSegment) */
    insertItemsLocal(pos, items, props) {
        if (items.length === 0) return undefined;
        const seg = props ? { items, props } : { items };
        this.engine.enqueue(this.doc, OP.INSERT | OPF_LOCAL, { pos1: pos }, seg);
        this.sent(OP.INSERT);
        return { type: OP.INSERT, pos1: pos, seg };
    }

    /* SharedSequence.getItems(start, end) (sharedSequence.ts:150-183) / getItemCount(): the local view's items of
     * [start, end) (mt_engine_get_items: the reference's splice-based cut, a marker inside the range included) */
    getItems(start, end) {
        return addon.getItems(this.read(), this.doc, start, end).map((i) => this.engine.interner.itemObj(i));
    }
    getItemCount() { return this.getLength(); }

    /* Client.insertSegmentLocal(pos, segment) (client.ts:202-211) for a segment spec: a string, {text, props},
     * {marker: {refType}, props}, {items, props} (SubSequence) or a PermutationSegment [length, start] */
    insertSegmentLocal(pos, spec) {
        if (typeof spec === "string" || (spec && typeof spec.text === "string")) {
            const text = typeof spec === "string" ? spec : spec.text;
            return this.insertTextLocal(pos, text, typeof spec === "string" ? undefined : spec.props);
        }
        if (spec && spec.marker) return this.insertMarkerLocal(pos, spec.marker.refType, spec.props);
        if (spec && Array.isArray(spec.items)) return this.insertItemsLocal(pos, spec.items, spec.props);
        if (Array.isArray(spec)) {
            this.engine.enqueue(this.doc, OP.INSERT | OPF_LOCAL, { pos1: pos }, spec);
            this.sent(OP.INSERT);
            return { type: OP.INSERT, pos1: pos, seg: spec };
        }
        throw new Error("insertSegmentLocal: unsupported segment spec");
    }

    /* Client.findTile(startPos, tileLabel, preceding) (client.ts:1075-1078 -> MergeTree.findTile, mergeTree.ts:
     * 1796-1822, search / backwardSearch with recordTileStart / tileShift, 1030-1069): the nearest marker with
     * the Tile refType and the label in its referenceTileLabels, at or before startPos (preceding) or at or after
     * it, in the local view; {tile, pos} or undefined. Blocks contribute their rightmost / leftmost tiles from
     * markers of non-zero local length (addNodeReferences 262-300), the segment the search stops at counts as it
     * is (backwardSearch from the document's end stops at its last segment, whatever its length). */
    findTile(startPos, tileLabel, preceding = true) {
        const d = this.segments();
        const segs = d.segments;
        const ok = (seg) => seg.len > 0 && hasTileLabel(seg, tileLabel);
        let stop = -1; // the segment the search reaches
        let tile;
        if (preceding) {
            if (startPos !== undefined) stop = segs.findIndex((seg) => seg.len > 0 && seg.pos <= startPos && startPos < seg.pos + seg.len);
            const shifted = stop < 0 ? segs.length : stop;
            for (let i = 0; i < shifted; i++) if (ok(segs[i])) tile = segs[i];
        } else {
            if (startPos !== undefined && startPos > d.localLength) return undefined;
            if (startPos !== undefined) {
                for (let i = segs.length - 1; i >= 0; i--) {
                    if (startPos >= segs[i].pos) { stop = i; break; } // segpos = segEnd - len <= pos
                }
            }
            for (let i = segs.length - 1; i > stop; i--) if (ok(segs[i])) tile = segs[i];
        }
        if (stop >= 0 && hasTileLabel(segs[stop], tileLabel)) tile = segs[stop];
        return tile === undefined ? undefined : { tile, pos: tile.pos };
    }

    /* Client.getMarkerFromId (client.ts:312-314; mergeTree.ts:1965-1967): the marker whose markerId is id, as a
     * segments() object; undefined if none. An id an annotate changed on a marker, or one several markers
     * hold, throws "unsupported" (mt_engine_get_marker_from_id). */
    getMarkerFromId(id) {
        const e = this.engine;
        const r = addon.getMarkerFromId(this.read(), this.doc, e.interner.key(MARKER_ID_KEY), e.interner.value(id) & 0xffff);
        return r === undefined ? undefined : this.segments().segments[r.ordinal];
    }

    /* Client.annotateMarker(marker, props, combiningOp) (client.ts:143-154; createAnnotateMarkerOp opBuilder.ts:
     * 25-38): annotates [pos, pos + 1) of the marker its markerId names, as the op's relative positions resolve
     * (getValidOpRange, client.ts:486-548); returns the op, or undefined (no id, or an invalid range) */
    annotateMarker(marker, props, combiningOp) {
        const id = marker && marker.properties ? marker.properties[MARKER_ID_KEY] : undefined;
        if (!id) return undefined;
        const m = this.getMarkerFromId(id);
        if (m === undefined) return undefined;
        const len = this.getLength();
        if (!(m.pos >= 0 && m.pos < len && m.pos + m.cachedLength <= len)) return undefined;
        const op = { combiningOp, props, relativePos1: { id, before: true }, relativePos2: { id }, type: OP.ANNOTATE };
        this.engine.enqueue(this.doc, OP.ANNOTATE | OPF_LOCAL, { pos1: m.pos, pos2: m.pos + m.cachedLength },
            { props, combiningOp });
        this.sent(OP.ANNOTATE);
        return op;
    }

    /* PermutationVector.adjustPosition(pos, fromSeq, clientId) (permutationvector.ts:185-196): a remote
     * client's row / col position in the local view, undefined when its segment is gone or removed */
    adjustPosition(pos, fromSeq, longClientId) {
        return addon.adjustPosition(this.read(), this.doc, pos, fromSeq, this.engine.longIndex(longClientId));
    }

    /* PermutationVector.handleToPosition(handle, localSeq) (permutationvector.ts:198-253): the position of a
     * handle for an op resubmitted at localSeq (default: the last local op's) */
    handleToPosition(handle, localSeq) {
        const h = this.read();
        if (localSeq === undefined) localSeq = this.segments().localSeq;
        return addon.handleToPosition(h, this.doc, handle, localSeq);
    }

    /* Every "sequenceDelta" / "maintenance" event this replica has fired since the engine was created
     * (engines created with caps.dcap > 0), decoded (decodeDeltas) */
    deltaEvents() { return decodeDeltas(addon.deltas(this.read(), this.doc), this.engine.interner); }
}

module.exports = { ReplayEngine, GpuClient, GpuMergeTree, Interner, addon, OP, DEFAULT_CAPS, decodeDeltas, decodeDump,
    ReferenceType, LocalClientId, UnassignedSequenceNumber };
