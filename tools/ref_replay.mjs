// ref_replay.mjs — replays packed op logs (include/mt_oplog.h) through the REFERENCE merge-tree
// (packages/dds/merge-tree/src, type-erased by tools/ts_erase.py into a scratch dir outside the
// repo) and writes each replica's canonical segment dump (include/mt_oplog.h, the format
// oracle/mt_oracle.c mto_dump emits). TEST INFRASTRUCTURE: golden-vector generation only
// (tools/make_ref_goldens.py); nothing in the product path runs it and it never reaches the GPU box.
//
// usage: node ref_replay.mjs <erased-dir> <batch-dir> [--time]
//   batch-dir: ops.bin op_off.bin text.bin text_off.bin props.bin props_off.bin kv.bin kv_off.bin
//              local.bin meta.json (written by make_ref_goldens.py)
//   writes batch-dir/ref_dumps.bin + ref_dump_off.bin (+ ref_err.json: per-doc thrown errors)
//   optional batch-dir/snapshots.json -> ref_snapshots.json (the emitted trees) + ref_loaded_dumps.bin /
//   ref_loaded_off.bin (dumps of the clients that loaded them and applied the rest of the log)
import fs from "fs";
import path from "path";

const [erased, dir] = process.argv.slice(2);
const timeOnly = process.argv.includes("--time");
// --deltas: also record every mergeTreeDeltaCallback / mergeTreeMaintenanceCallback the replica fires
// (the stream SharedString's "sequenceDelta" / "maintenance" listeners see, sequence.ts:136-150) in the
// word format of include/mt_oplog.h (MT_DELTA_*) -> batch-dir/ref_deltas.bin + ref_delta_off.bin
const withDeltas = process.argv.includes("--deltas");
// --handles: every replica is also a PermutationVector's HandleTable owner (matrix permutationvector.ts:
// 124-363): local NOOP records are getAllocatedHandle(pos1), zamboni's UNLINK callbacks free handles, inserted
// segments reset their start; dumps carry allocated starts (MT_DF_HANDLE) -> batch-dir/ref_handles.json
const withHandles = process.argv.includes("--handles");
const traceDoc = process.argv.includes("--trace-refs") ? Number(process.argv[process.argv.indexOf("--trace-refs") + 1]) : -1;
let Client, TextSegment, Marker, PermutationSegment, SubSequence, SnapshotV1, SnapshotLegacy, LocalReference; // bound in main() (Node 12 has no top-level await)
let HandleTable, isHandleValid;
let curHandles = null; // the HandleTable of the replica being replayed (--handles)
const handleTables = {};

const rd = (f) => fs.readFileSync(path.join(dir, f));
const meta = JSON.parse(rd("meta.json"));
const ops = rd("ops.bin"), text = rd("text.bin"), props = rd("props.bin"), kv = rd("kv.bin");
const i64 = (f) => { const b = rd(f); return Array.from({ length: b.length / 8 }, (_, i) => Number(b.readBigInt64LE(8 * i))); };
const opOff = i64("op_off.bin"), textOff = i64("text_off.bin"), propsOff = i64("props_off.bin"), kvOff = i64("kv_off.bin");
const localIds = rd("local.bin");
const keys = meta.keys, values = meta.values; // interner tables: id -> key string / canonical JSON
const keyId = new Map(keys.map((k, i) => [k, i]));
const valueId = new Map(values.map((v, i) => [v, i]));
const FALSY = 0x8000;

const name = (longId) => `c${longId}`;
const longOfName = (s) => (s === "original" ? -1 : Number(s.slice(1)));

function canonical(v) {
    if (v === null || typeof v !== "object") return JSON.stringify(v);
    if (Array.isArray(v)) return "[" + v.map(canonical).join(",") + "]";
    return "{" + Object.keys(v).sort().map((k) => JSON.stringify(k) + ":" + canonical(v[k])).join(",") + "}";
}

function propSet(doc, idx) {
    if (!idx) return undefined;
    const p = (propsOff[doc] + idx - 1) * 8;
    const off = props.readUInt32LE(p), nkv = props.readUInt16LE(p + 4), comb = props.readUInt8(p + 6);
    const set = {};
    for (let j = 0; j < nkv; j++) {
        const q = (kvOff[doc] + off + j) * 4;
        const k = kv.readUInt16LE(q), v = kv.readUInt16LE(q + 2) & ~FALSY;
        set[keys[k]] = v === 0 ? null : JSON.parse(values[v]);
    }
    return { set, combiningOp: comb === 1 ? { name: "rewrite" } : comb === 2 ? { name: "incr" } : comb === 3 ? { name: "consensus" } : undefined };
}

function textOf(doc, rec) {
    const off = textOff[doc] + rec.text_off;
    let s = "";
    for (let j = 0; j < rec.text_len; j++) s += String.fromCharCode(text.readUInt16LE(2 * (off + j)));
    return s;
}

// SubSequence items (mt_oplog.h MT_SEG_RUN: the text units are item ids): meta.items, when present, is the host's item
// interner (id -> canonical JSON); without it an item is the number its id is (a SharedNumberSequence)
const items = meta.items || null;
const itemId = items ? new Map(items.map((v, i) => [v, i])) : null;
function itemsOf(doc, rec) {
    const off = textOff[doc] + rec.text_off, out = [];
    for (let j = 0; j < rec.text_len; j++) {
        const u = text.readUInt16LE(2 * (off + j));
        out.push(items ? JSON.parse(items[u]) : u);
    }
    return out;
}
function itemUnit(v) {
    if (!items) return v;
    const id = itemId.get(canonical(v));
    if (id === undefined) throw new Error(`item not in the interner: ${canonical(v)}`);
    return id;
}
// a record's inserted segment (insertSegmentLocal / MergeTree.insertSegments): TextSegment.make, Marker.make, a
// PermutationSegment or a SubSequence, with the record's properties
function segOf(doc, rec, ps) {
    if (rec.seg_kind === 2 || rec.seg_kind === 3) {
        const seg = rec.seg_kind === 2 ? new PermutationSegment(rec.text_len) : new SubSequence(itemsOf(doc, rec));
        if (ps) seg.addProperties(ps.set);
        return seg;
    }
    return rec.seg_kind === 1 ? Marker.make(rec.pos2, ps && ps.set) : TextSegment.make(textOf(doc, rec), ps && ps.set);
}

function record(i) {
    const b = 32 * i;
    return {
        kind: ops.readUInt8(b), seg_kind: ops.readUInt8(b + 1), client: ops.readUInt16LE(b + 2),
        seq: ops.readInt32LE(b + 4), ref_seq: ops.readInt32LE(b + 8), min_seq: ops.readInt32LE(b + 12),
        pos1: ops.readInt32LE(b + 16), pos2: ops.readInt32LE(b + 20), text_off: ops.readUInt32LE(b + 24),
        text_len: ops.readUInt16LE(b + 28), props: ops.readUInt16LE(b + 30),
    };
}

// the wire op (IMergeTreeOp, ops.ts:63-102) a record stands for
function wireOp(doc, rec) {
    const op = wireOpAbs(doc, { ...rec, seg_kind: rec.seg_kind & 0x7f });
    if (rec.seg_kind & 0x80) { // MT_SEG_RELPOS: the positions are IRelativePosition objects (mt_oplog.h)
        const b = 2 * (textOff[doc] + rec.text_off + rec.text_len);
        const u = (k) => text.readUInt16LE(b + 2 * k);
        const which = u(1);
        const rel = (k) => {
            const r = { id: JSON.parse(values[u(k) & ~FALSY]) };
            if (u(k + 1) & 1) r.before = true;
            if (u(k + 1) & 2) r.offset = (u(k + 2) | (u(k + 3) << 16)) | 0;
            return r;
        };
        if (which & 1) { delete op.pos1; op.relativePos1 = rel(2); }
        if (which & 2) { delete op.pos2; op.relativePos2 = rel(6); }
    }
    return op;
}
function wireOpAbs(doc, rec) {
    const kind = rec.kind & 7;
    const ps = propSet(doc, rec.props);
    if (kind === 0) {
        let seg;
        if (rec.seg_kind === 2) return { type: 0, pos1: rec.pos1, seg: new PermutationSegment(rec.text_len).toJSONObject() };
        if (rec.seg_kind === 1) seg = { marker: { refType: rec.pos2 } };
        else if (rec.seg_kind === 3) seg = { items: itemsOf(doc, rec) }; // SubSequence.toJSONObject
        else seg = ps ? { text: textOf(doc, rec) } : textOf(doc, rec);
        if (ps) seg.props = ps.set;
        return { type: 0, pos1: rec.pos1, seg };
    }
    if (kind === 1) return { type: 1, pos1: rec.pos1, pos2: rec.pos2 };
    const op = { type: 2, pos1: rec.pos1, pos2: rec.pos2, props: ps ? ps.set : {} };
    if (ps && ps.combiningOp) op.combiningOp = ps.combiningOp;
    return op;
}

// SharedString's specToSegment; PermutationVector's (PermutationSegment.fromJSONObject) for array specs; SharedSequence's
// (SubSequence.fromJSONObject, sequenceFactory.ts) for {items} specs
const specToSegment = (spec) => (Array.isArray(spec) ? PermutationSegment.fromJSONObject(spec)
    : (spec && typeof spec === "object" && "items" in spec) ? SubSequence.fromJSONObject(spec)
        : TextSegment.fromJSONObject(spec) || Marker.fromJSONObject(spec));
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

// apply records [from, to) of `doc` to `client` (applyMsg / the local-edit entry points)
let applying = -1; // the record being applied (for error reports)
let curSeq = 0; // seq of the record being applied (-1: a local edit), the delta stream's event seq
// --combine-watch: per document, the first record after which a segment holds a value only Properties.combine
// makes as addProperties calls it (newValue undefined, properties.ts:26-59): NaN, a string ending in "undefined"
// (incr), or a {value, seq} object (consensus) -> batch-dir/ref_combine.json
const combineWatch = process.argv.includes("--combine-watch");
const combineAt = {};
function combinedValue(v) {
    return (typeof v === "number" && Number.isNaN(v)) || (typeof v === "string" && v.endsWith("undefined")) ||
        (v !== null && typeof v === "object" && "seq" in v);
}
function watchCombine(client, doc, i) {
    if (combineAt[doc] !== undefined) return;
    client.mergeTree.walkAllSegments(client.mergeTree.root, (seg) => {
        if (seg.properties) for (const k of Object.keys(seg.properties)) if (combinedValue(seg.properties[k])) combineAt[doc] = i - opOff[doc];
        return combineAt[doc] === undefined;
    });
}
function applyRange(client, doc, from, to) {
    let members = []; // members of a group message so far (records flagged GROUPED, mt_oplog.h)
    let prevComb = false; // the previous record carried an incr / consensus annotate (--combine-watch)
    for (let i = from; i <= to; i++) {
        if (prevComb) watchCombine(client, doc, i - 1);
        if (i === to) break;
        applying = i;
        const rec = record(i);
        prevComb = combineWatch && (rec.kind & 7) === 2 && rec.props > 0 && (() => {
            const ps = propSet(doc, rec.props);
            return ps && ps.combiningOp && ps.combiningOp.name !== "rewrite";
        })();
        const kind = rec.kind & 7;
        curSeq = rec.kind & 0x80 ? -1 : rec.seq;
        if ((rec.kind & 0x90) === 0x90) { // MT_OPF_REGEN: Client.regeneratePendingOp for the head pending op
            const e = pendingOps.shift();
            const newOp = client.regeneratePendingOp(e.op, e.group);
            const ops = newOp.type === 3 ? newOp.ops : [newOp];
            const w = [3, -1]; // MT_DELTA_REGEN
            for (const o of ops) {
                const len = o.type === 0 ? (typeof o.seg === "string" ? o.seg.length : o.seg.text !== undefined
                    ? o.seg.text.length : o.seg.items !== undefined ? o.seg.items.length : Array.isArray(o.seg) ? o.seg[0] : 1)
                    : o.pos2 - o.pos1;
                w.push(o.pos1, len, o.type);
            }
            w.push(END, ops.length);
            if (deltaWords[curDoc]) deltaWords[curDoc].push(...w);
            (regenWords[curDoc] = regenWords[curDoc] || []).push(...w);
            if (ops.length) {
                const groups = client.peekPendingSegmentGroups(ops.length);
                const gs = ops.length === 1 ? [groups] : groups;
                ops.forEach((o, i) => pendingOps.push({ op: o, group: gs[i] }));
            }
            continue;
        }
        if (rec.kind & 0x20) { // MT_OPF_TREE: MergeTree-level call with the record's (refSeq, clientId, seq)
            const mt = client.mergeTree;
            const cid = rec.client === 0xFFFE ? -1 : client.getOrAddShortClientId(name(rec.client));
            const opArgs = { op: wireOp(doc, rec) };
            const ps = propSet(doc, rec.props);
            if (kind === 0) {
                const seg = segOf(doc, rec, ps);
                mt.insertSegments(rec.pos1, [seg], rec.ref_seq, cid, rec.seq, opArgs);
            } else if (kind === 1) {
                mt.markRangeRemoved(rec.pos1, rec.pos2, rec.ref_seq, cid, rec.seq, false, opArgs);
            } else if (kind === 2) {
                mt.annotateRange(rec.pos1, rec.pos2, ps ? ps.set : {}, ps ? ps.combiningOp : undefined, rec.ref_seq, cid,
                    rec.seq, opArgs);
            }
            continue;
        }
        if (rec.kind & 0x80) { // local edit: insertSegmentLocal / removeRangeLocal / annotateRangeLocal
            if (kind === 4) { // PermutationVector.getAllocatedHandle(pos1) (permutationvector.ts:157-183)
                getAllocatedHandle(client, rec.pos1);
                continue;
            }
            if (kind === 0) {
                const ps = propSet(doc, rec.props);
                const seg = segOf(doc, rec, ps);
                let sent;
                if (rec.kind & 0x08) { // MT_OPF_ATREF: insertAtReferencePositionLocal at reference pos1
                    const r = curRefs[rec.pos1];
                    if (traceDoc === doc) { // debugging aid (--trace-refs DOC): where every reference sits
                        console.error(JSON.stringify(curRefs.map((x, k) => x && x.segment && {
                            k, len: x.segment.cachedLength, off: x.offset, rm: x.segment.removedSeq, seq: x.segment.seq,
                            pos: x.toPosition(), text: x.segment.text })));
                    }
                    if (r) {
                        const before = client.peekPendingSegmentGroups();
                        client.insertAtReferencePositionLocal(r, seg);
                        if (client.peekPendingSegmentGroups() !== before) sent = { type: 0, pos1: 0, seg: seg.toJSONObject() };
                    }
                } else {
                    sent = client.insertSegmentLocal(rec.pos1, seg);
                }
                if (sent && client.getCollabWindow().collaborating) pendingOps.push({ op: sent, group: client.peekPendingSegmentGroups() });
            } else if (kind === 1) {
                const sent = client.removeRangeLocal(rec.pos1, rec.pos2);
                if (sent && client.getCollabWindow().collaborating) pendingOps.push({ op: sent, group: client.peekPendingSegmentGroups() });
            } else if (kind === 2) {
                const ps = propSet(doc, rec.props);
                const sent = client.annotateRangeLocal(rec.pos1, rec.pos2, ps ? ps.set : {}, ps ? ps.combiningOp : undefined);
                if (sent && client.getCollabWindow().collaborating) pendingOps.push({ op: sent, group: client.peekPendingSegmentGroups() });
            } else if (kind === 3 && rec.seg_kind === 1) { // MT_REF_REMOVE: Client.removeLocalReference
                const r = curRefs[rec.pos1];
                if (r) {
                    try {
                        client.removeLocalReference(r);
                    } catch (e) { // a detached reference (segment undefined): the call throws, the tree is
                        removeThrew++; // untouched
                    }
                }
            } else if (kind === 3) { // a local reference (mt_oplog.h MT_OP_REF) at getContainingSegment(pos1)
                const { segment, offset } = client.getContainingSegment(rec.pos1);
                let lref = null;
                if (segment) {
                    lref = new LocalReference(client, segment, offset, rec.pos2);
                    try {
                        client.addLocalReference(lref);
                    } catch (e) { // addLocalRef at an offset holding only slid refs: refsByOffset[o].at is
                        threwRefs.add(lref); // undefined (localReference.ts:195-201); the tree is untouched
                    }
                }
                curRefs.push(lref);
            }
            continue;
        }
        if (rec.kind & 0x40) { members.push(wireOp(doc, rec)); continue; }
        let contents = kind === 4 ? undefined : wireOp(doc, rec);
        if (members.length) { contents = { type: 3, ops: [...members, contents] }; members = []; } // createGroupOp (opBuilder.ts:128-134)
        const msg = {
            clientId: name(rec.client), sequenceNumber: rec.seq, referenceSequenceNumber: rec.ref_seq,
            minimumSequenceNumber: rec.min_seq, type: kind === 4 ? "noop" : "op", contents,
        };
        // SharedString.processMergeTreeMsg (sequence.ts:579-616) when summaries are legacy: a message whose
        // refSeq is not seq - 1 is stashed rebased, its contents the ops of the sequenceDelta events it fires
        const rebase = stash !== null && kind !== 4 && msg.referenceSequenceNumber !== msg.sequenceNumber - 1;
        if (rebase) rebaseSink = [];
        client.applyMsg(msg);
        if (stash !== null && kind !== 4) {
            let st = msg;
            if (rebase) {
                st = JSON.parse(JSON.stringify(msg));
                st.referenceSequenceNumber = msg.sequenceNumber - 1;
                st.contents = rebaseSink.length !== 1 ? { ops: rebaseSink, type: 3 } : rebaseSink[0];
                rebaseSink = null;
            }
            stash.push(st);
        }
        if (kind !== 4 && name(rec.client) === client.longClientId) { // an ack: its groups leave the queue
            pendingOps.splice(0, contents.type === 3 ? contents.ops.length : 1);
        }
    }
}

// PermutationVector's handle bookkeeping around the reference Client (permutationvector.ts:124-363, restated:
// the class itself needs the container runtime), with the reference's own HandleTable (handletable.ts)
function hookHandles(client, doc, table = new HandleTable()) {
    handleTables[doc] = table;
    curHandles = table;
    const prevDelta = client.mergeTreeDeltaCallback, prevMaint = client.mergeTreeMaintenanceCallback;
    client.mergeTreeDeltaCallback = (opArgs, args) => {
        if (args.operation === 0) for (const { segment } of args.deltaSegments) segment.reset(); // onDelta INSERT (297-309)
        if (prevDelta) prevDelta(opArgs, args);
    };
    client.mergeTreeMaintenanceCallback = (args) => {
        if (prevMaint) prevMaint(args);
        if (args.operation === -3) { // onMaintenance UNLINK (338-363)
            let freed = [];
            for (const { segment } of args.deltaSegments) {
                if (isHandleValid(segment.start)) {
                    freed = freed.concat(new Array(segment.cachedLength).fill(0).map((v, i) => i + segment.start));
                }
            }
            for (const h of freed) table.free(h);
        }
    };
}
// getAllocatedHandle (157-183): getMaybeHandle is HandleCache.getHandle = the containing segment's start +
// offset (handlecache.ts:77-88); a miss allocates through walkSegments(pos, pos + 1, splitRange = true)
function getAllocatedHandle(client, pos) {
    if (!(0 <= pos && pos < client.getLength())) throw new Error(`getAllocatedHandle: position ${pos} out of range`);
    const { segment, offset } = client.getContainingSegment(pos);
    let handle = segment.start + offset;
    if (isHandleValid(handle)) return handle;
    client.walkSegments((seg) => { seg.start = handle = curHandles.allocate(); return true; }, pos, pos + 1, undefined, true);
    return handle;
}

// the delta stream (include/mt_oplog.h): per callback op, seq, per delta segment (position in the
// local view for delta events, -1 for maintenance; cachedLength; property deltas by key id), count
function valueWord(v) {
    if (v === null || v === undefined) return 0;
    const id = valueId.get(canonical(v));
    if (id === undefined) throw new Error(`property value not in the interner: ${canonical(v)}`);
    return id | (v !== null && typeof v !== "object" && !v ? FALSY : 0);
}
const END = -0x80000000; // MT_DELTA_END
function hookDeltas(client, words) {
    client.mergeTreeDeltaCallback = (opArgs, args) => {
        words.push(args.operation, curSeq);
        for (const d of args.deltaSegments) {
            words.push(client.getPosition(d.segment), d.segment.cachedLength);
            if (args.operation !== 2) { words.push(0); continue; }
            if (d.propertyDeltas === undefined) { words.push(-1); continue; }
            const pd = Object.keys(d.propertyDeltas).map((k) => [keyId.get(k), valueWord(d.propertyDeltas[k])])
                .sort((a, b) => a[0] - b[0]);
            words.push(pd.length);
            for (const [k, v] of pd) words.push(((k << 16) | v) | 0);
        }
        words.push(END, args.deltaSegments.length);
    };
    client.mergeTreeMaintenanceCallback = (args) => {
        words.push(args.operation, curSeq);
        for (const d of args.deltaSegments) words.push(-1, d.segment.cachedLength, 0);
        words.push(END, args.deltaSegments.length);
    };
}
const deltaWords = [];
// legacy summaries: SharedString's messagesSinceMSNChange of the replica being replayed (null: not kept),
// and the ops createOpsFromDelta makes of the sequenceDelta events of the message being rebased
let stash = null;
let rebaseSink = null;
// SharedSegmentSequence.createOpsFromDelta (sequence.ts:62-110), restated over one callback's delta
// segments: ranges in document order at their current position (SequenceDeltaEvent.ranges); insert ranges
// give insert ops of the segment's JSON; remove ranges extend the last op when it starts at the range's
// position, else add one; annotate ranges carry each changed key's current value (null if absent) and
// extend the last op when it ends at the range with the same props
function opsFromDelta(client, args, out) {
    const ranges = args.deltaSegments.map((d) => ({ position: client.getPosition(d.segment), segment: d.segment,
        propertyDeltas: d.propertyDeltas })).sort((a, b) => (a.segment.ordinal < b.segment.ordinal ? -1 : 1));
    for (const r of ranges) {
        const last = out[out.length - 1];
        if (args.operation === 0) {
            out.push({ pos1: r.position, seg: JSON.parse(JSON.stringify(r.segment.toJSONObject())), type: 0 });
        } else if (args.operation === 1) {
            if (last !== undefined && last.pos1 === r.position) last.pos2 += r.segment.cachedLength;
            else out.push({ pos1: r.position, pos2: r.position + r.segment.cachedLength, type: 1 });
        } else if (args.operation === 2) {
            const p = {};
            for (const k of Object.keys(r.propertyDeltas)) {
                p[k] = r.segment.properties[k] === undefined ? null : r.segment.properties[k];
            }
            if (last !== undefined && last.pos2 === r.position && MT.matchProperties(last.props, p)) {
                last.pos2 += r.segment.cachedLength;
            } else {
                out.push({ pos1: r.position, pos2: r.position + r.segment.cachedLength, props: p, type: 2 });
            }
        }
    }
}
let MT;
let curDoc = -1;
let curRefs = []; // the local references of the document being replayed, in creation order
// the replica's pending ops, one entry per pending segment group: {op, group} — what the runtime keeps
// as the message contents and localOpMetadata it hands to regeneratePendingOp on reconnect
let pendingOps = [];
const regenWords = [];
const threwRefs = new Set(); // references whose addLocalReference threw
let removeThrew = 0; // removeLocalReference calls that threw (detached references)
const refPositions = {};
const refInside = {};
const refPastEnd = {};

function replayDoc(doc, to = opOff[doc + 1], deltas = false) {
    const client = new Client(specToSegment, logger);
    curRefs = [];
    pendingOps = [];
    curDoc = doc;
    if (deltas) {
        const words = [];
        deltaWords[doc] = words;
        hookDeltas(client, words);
    }
    if (withHandles) hookHandles(client, doc);
    if (stash !== null) {
        client.mergeTreeDeltaCallback = (opArgs, args) => { if (rebaseSink !== null) opsFromDelta(client, args, rebaseSink); };
    }
    const local = localIds.readInt32LE(4 * doc);
    if (local >= 0) client.startOrUpdateCollaboration(name(local));
    applyRange(client, doc, opOff[doc], to);
    return client;
}

// ---- legacy summaries (snapshots_legacy.json: [[doc, cut, loadLong], ...]) -------------------------
// SharedString's default summary: after records [0, cut) Client.snapshot with its messagesSinceMSNChange
// (sequence.ts:566-577): the messages above the MSN, minimumSequenceNumber set to the MSN; SnapshotLegacy
// extractSync + emit (snapshotlegacy.ts:104-242). A fresh Client name(loadLong) loads the tree and applies
// the catch-up messages as SharedString's load does (sequence.ts:501-515); its dump is the "loaded" dump.
async function snapshotLegacyDoc(doc, cut, loadLong) {
    stash = [];
    let a;
    try {
        a = replayDoc(doc, opOff[doc] + cut);
    } finally {
        rebaseSink = null;
    }
    const msgs = stash;
    stash = null;
    const minSeq = a.getCollabWindow().minSeq;
    const catchUp = msgs.filter((m) => m.sequenceNumber > minSeq);
    catchUp.forEach((m) => { m.minimumSequenceNumber = minSeq; });
    const snap = new SnapshotLegacy(a.mergeTree, runtimeOf(name(loadLong)).logger);
    snap.extractSync();
    const tree = snap.emit(catchUp);
    const b = new Client(specToSegment, logger);
    try {
        const { catchupOpsP } = await b.load(runtimeOf(name(loadLong)), storageOf(tree));
        for (const m of await catchupOpsP) b.applyMsg(m);
    } catch (e) {
        return { tree, loaded: Buffer.alloc(0), loadError: String(e && e.message || e) };
    }
    if (withHandles) snapHandles[doc].final = handleTables[doc].snapshot();
    return { tree, loaded: dump(b) };
}

// ---- snapshots (snapshots.json: [[doc, cut, loadLong], ...]) --------------------------------------
// The replica after records [0, cut) is summarized (SnapshotV1.extractSync + emit, snapshotV1.ts); a
// fresh Client loads that tree (Client.load -> SnapshotLoader, snapshotLoader.ts) as client
// name(loadLong) and applies records [cut, end); its dump is the "loaded" dump.
const storageOf = (tree) => {
    const blobs = new Map(tree.entries.map((e) => [e.path, e.value.contents]));
    return {
        read: async (p) => Buffer.from(blobs.get(p), "utf8").toString("base64"),
        list: async () => [...blobs.keys()],
        contains: async (p) => blobs.has(p),
    };
};
const runtimeOf = (clientId) => ({
    options: {}, documentId: "doc", clientId, attachState: "Attached", IFluidSerializer: undefined,
    IFluidHandleContext: undefined,
    logger: { ...logger, shipAssert(cond, ev) { if (!cond) throw new Error(`shipAssert ${JSON.stringify(ev)}`); } },
});
// With --handles the replica is a PermutationVector's: its summary also holds the HandleTable blob
// (PermutationVector.snapshot, permutationvector.ts:256-268), and the loading replica installs its delta /
// maintenance hooks over HandleTable.load(blob) before Client.load, as PermutationVector's constructor and load
// do (129-145, 270-275): loadBody's inserts then reset their segments' starts (onDelta INSERT).
const snapHandles = {};
const chunkArg = process.argv.find((x) => x.startsWith("--chunk="));
const snapChunk = chunkArg ? Number(chunkArg.slice(8)) : 0; // mergeTreeSnapshotChunkSize (snapshotV1.ts:56); 0: default
async function snapshotDoc(doc, cut, loadLong) {
    const a = replayDoc(doc, opOff[doc] + cut);
    if (snapChunk > 0) a.mergeTree.options = Object.assign({}, a.mergeTree.options, { mergeTreeSnapshotChunkSize: snapChunk });
    const snap = new SnapshotV1(a.mergeTree, logger);
    snap.extractSync();
    const tree = snap.emit();
    const b = new Client(specToSegment, logger);
    let blob = null;
    if (withHandles) {
        blob = JSON.parse(JSON.stringify(handleTables[doc].snapshot()));
        hookHandles(b, doc, HandleTable.load(JSON.parse(JSON.stringify(blob))));
        snapHandles[doc] = { blob };
    }
    try {
        const { catchupOpsP } = await b.load(runtimeOf(name(loadLong)), storageOf(tree));
        await catchupOpsP;
    } catch (e) { // the reference cannot load its own snapshot (e.g. loadBody's insert fails)
        return { tree, loaded: Buffer.alloc(0), loadError: String(e && e.message || e) };
    }
    try {
        applyRange(b, doc, opOff[doc] + cut, opOff[doc + 1]);
    } catch (e) { // the loaded replica cannot apply the rest of the log: report where (tail-relative)
        return { tree, loaded: Buffer.alloc(0), tailError: [applying - opOff[doc] - cut, String(e && e.message || e)] };
    }
    if (withHandles) snapHandles[doc].final = handleTables[doc].snapshot();
    return { tree, loaded: dump(b) };
}

// ---- derived values (include/mt_oplog.h MT_VALUE_DERIVED): what Properties.combine makes with newValue undefined
// (properties.ts:26-59): NaN; a {value: undefined, seq} consensus object; base + "undefined" x k, base an interned
// string or a consensus object ("[object Object]", base 0; the engine refuses an incr over an interned object or array,
// whose String() could equal a string's). [kind marker, a, b] as the canonical dump writes them.
const VALUE_STRCAT0 = 0x7F00, VALUE_CONS0 = 0x7F80, VALUE_NAN = 0x7FFF;
const jsStringOf = new Map(); // each interned string -> its id (with the falsy bit)
values.forEach((sv, i) => {
    if (i === 0) return;
    const v = JSON.parse(sv);
    if (typeof v === "string") jsStringOf.set(v, i | (v === "" ? FALSY : 0));
});
function derivedOf(v) {
    if (typeof v === "number" && Number.isNaN(v)) return [VALUE_NAN];
    if (v !== null && typeof v === "object" && !Array.isArray(v) && v.value === undefined && typeof v.seq === "number" &&
        Object.keys(v).every((k) => k === "value" || k === "seq")) return [VALUE_CONS0, v.seq, 0];
    if (typeof v === "string") {
        let s = v, k = 0;
        while (s.endsWith("undefined")) {
            s = s.slice(0, -9);
            k++;
            if (jsStringOf.has(s)) return [VALUE_STRCAT0, jsStringOf.get(s), k];
            if (s === "[object Object]") return [VALUE_STRCAT0, 0, k];
        }
    }
    return null;
}

// ---- canonical dump (include/mt_oplog.h; the order and fields of oracle/mt_oracle.c mto_dump) ----
class Out {
    constructor() { this.parts = []; }
    i32(v) { const b = Buffer.alloc(4); b.writeInt32LE(v); this.parts.push(b); }
    u16(v) { const b = Buffer.alloc(2); b.writeUInt16LE(v); this.parts.push(b); }
    u8(v) { this.parts.push(Buffer.from([v])); }
    buf() { return Buffer.concat(this.parts); }
}

function dump(client) {
    const mt = client.mergeTree;
    const longOf = (shortId) => (shortId < 0 ? -1 : longOfName(client.getLongClientId(shortId)));
    const leaves = [];
    const walk = (b) => {
        if (b.childCount === 0 || b.children[0].isLeaf()) { leaves.push(b); return; }
        for (let i = 0; i < b.childCount; i++) walk(b.children[i]);
    };
    walk(mt.root);
    let nsegs = 0;
    for (const b of leaves) nsegs += b.childCount;
    const o = new Out();
    const cw = mt.collabWindow;
    o.i32(cw.currentSeq); o.i32(cw.minSeq); o.i32(cw.localSeq); o.i32(mt.root.cachedLength);
    o.i32(nsegs); o.i32(leaves.length);
    leaves.forEach((b, li) => {
        for (let i = 0; i < b.childCount; i++) {
            const s = b.children[i];
            const isText = s.type === "TextSegment", isMarker = s.type === "Marker", isRun = s.type === "SubSequence";
            const kind = isText ? 0 : isMarker ? 1 : isRun ? 3 : 2;
            const hasProps = s.properties !== undefined;
            const hnd = s.type === "PermutationSegment" && s.start >= 1; // an allocated start
            const removed = s.removedSeq !== undefined;
            const ov = s.removedClientOverlap || [];
            o.u8(kind);
            o.u8((hasProps ? 1 : 0) | (removed ? 2 : 0) | (s.localSeq !== undefined ? 4 : 0) | (s.localRemovedSeq !== undefined ? 8 : 0) |
                (hnd ? 16 : 0));
            o.u8(ov.length);
            o.u8(s.segmentGroups.size);
            o.i32(s.cachedLength); o.i32(s.seq); o.i32(longOf(s.clientId));
            o.i32(removed ? s.removedSeq : 0); o.i32(removed ? longOf(s.removedClientId) : 0);
            o.i32(s.localSeq !== undefined ? s.localSeq : 0);
            o.i32(s.localRemovedSeq !== undefined ? s.localRemovedSeq : 0);
            o.i32(li);
            for (const c of ov) o.i32(longOf(c));
            const pk = hasProps ? Object.keys(s.properties).map((k) => [keyId.get(k), s.properties[k]]).sort((a, b) => a[0] - b[0]) : [];
            o.u16(pk.length);
            o.u16(isMarker ? s.refType : 0);
            const extra = [];
            for (const [k, v] of pk) {
                // NaN first: canonical(NaN) is JSON's "null", the interner's id 0
                const id = typeof v === "number" && Number.isNaN(v) ? undefined : valueId.get(canonical(v));
                if (k === undefined) throw new Error(`property key not in the interner: ${k}`);
                if (id === undefined) { // a value Properties.combine made (include/mt_oplog.h MT_VALUE_DERIVED)
                    const dv = derivedOf(v);
                    if (!dv) throw new Error(`property not in the interner: ${k} ${canonical(v)}`);
                    o.u16(k); o.u16(dv[0]);
                    if (dv.length > 1) extra.push(dv[1], dv[2]);
                    continue;
                }
                const falsy = v !== null && typeof v !== "object" && !v;
                o.u16(k); o.u16(id | (falsy ? FALSY : 0));
            }
            for (const x of extra) o.i32(x);
            if (hnd) o.i32(s.start); // MT_DF_HANDLE
            if (isText) for (let j = 0; j < s.text.length; j++) o.u16(s.text.charCodeAt(j));
            if (isRun) for (const v of s.items) o.u16(itemUnit(v));
        }
    });
    return o.buf();
}

async function main() {
MT = await import(path.join(erased, "index.mjs"));
({ Client, TextSegment, Marker, LocalReference } = MT);
({ PermutationSegment } = await import(path.join(erased, "permutationSegment.mjs")));
({ SubSequence } = await import(path.join(erased, "subSequence.mjs")));
({ HandleTable, isHandleValid } = await import(path.join(erased, "handletable.mjs")));
({ SnapshotV1 } = await import(path.join(erased, "snapshotV1.mjs")));
({ SnapshotLegacy } = await import(path.join(erased, "snapshotlegacy.mjs")));
const ndocs = opOff.length - 1;
// optional read queries (queries.json: [[doc, pos, refSeq, longClient | -1 = local view], ...]):
// getContainingSegment + getPosition (mergeTree.ts:1656-1667, 1619-1636) after the doc's replay
const qpath = path.join(dir, "queries.json");
const queries = fs.existsSync(qpath) ? JSON.parse(fs.readFileSync(qpath)) : [];
const answers = [];
// optional getText queries (textqueries.json: [[doc, refSeq, longClient | -1 = local view, placeholder,
// start | null, end | null], ...]): MergeTreeTextHelper.getText (textSegment.ts:154-186) -> ref_texts.json
const tqpath = path.join(dir, "textqueries.json");
const textQueries = fs.existsSync(tqpath) ? JSON.parse(fs.readFileSync(tqpath)) : [];
const texts = [];
// optional posFromRelativePos queries (relqueries.json: [[doc, markerId, before, offset | null], ...]) in the
// replica's local view (Client.posFromRelativePos, client.ts:308) -> ref_relpos.json
const rqpath = path.join(dir, "relqueries.json");
const relQueries = fs.existsSync(rqpath) ? JSON.parse(fs.readFileSync(rqpath)) : [];
const relAnswers = [];
// optional getLength queries (lenqueries.json: [[doc, refSeq, longClient | -1 = local view], ...]):
// MergeTree.getLength(refSeq, clientId) (mergeTree.ts:1610-1612: the root's PartialSequenceLengths for a
// remote perspective, cachedLength for the local client) -> ref_lengths.json
const lqpath = path.join(dir, "lenqueries.json");
const lenQueries = fs.existsSync(lqpath) ? JSON.parse(fs.readFileSync(lqpath)) : [];
const lengths = [];
// optional getItems queries (itemqueries.json: [[doc, start, end | null], ...]): SharedSequence.getItems (sequence
// sharedSequence.ts:150-183, restated below over the reference Client, as SharedSegmentSequence's walkSegments and
// getPosition forward to it) after the doc's replay -> ref_items.json (item ids, itemUnit)
const iqpath = path.join(dir, "itemqueries.json");
const itemQueries = fs.existsSync(iqpath) ? JSON.parse(fs.readFileSync(iqpath)) : [];
const itemAnswers = [];
function getItems(client, start, end) {
    const out = [];
    let firstSegment;
    if (end !== undefined && end <= start) return out;
    client.walkSegments((segment) => {
        if (SubSequence.is(segment)) {
            if (firstSegment === undefined) firstSegment = segment;
            out.push(...segment.items);
        }
        return true;
    }, start, end);
    if (firstSegment !== undefined) out.splice(0, start - client.getPosition(firstSegment));
    if (end !== undefined) out.splice(end - start);
    return out;
}
const t0 = process.hrtime.bigint();
const dumps = [], errs = {};
for (let d = 0; d < ndocs; d++) {
    try {
        const c = replayDoc(d, opOff[d + 1], withDeltas);
        // LocalReference.toPosition (localReference.ts:62-68) of every reference, -1 when detached
        if (curRefs.length) {
            refPositions[d] = curRefs.map((r) => (threwRefs.has(r) ? -2 : r ? r.toPosition() : -1));
            // a reference an insert can target: an offset inside its segment, or past the end of a text
            // segment (an append can leave one there: refsByOffset.length is not the segment's length,
            // localReference.ts:211-223; inserting there splits off an empty segment). Past the end of a
            // PermutationSegment the split makes a negative length, and a Marker does not split (the
            // insert throws, mergeTree.ts:2082-2083).
            refInside[d] = curRefs.map((r) => !!(r && r.segment && (r.offset < r.segment.cachedLength ||
                TextSegment.is(r.segment))));
            refPastEnd[d] = curRefs.map((r) => !!(r && r.segment && r.offset >= r.segment.cachedLength));
        }
        for (const [qd, pos, ref, cl] of queries) {
            if (qd !== d) continue;
            const mt = c.mergeTree;
            const local = cl < 0;
            const refSeq = local ? mt.collabWindow.currentSeq : ref;
            const cid = local ? mt.collabWindow.clientId : c.getOrAddShortClientId(name(cl));
            const { segment, offset } = mt.getContainingSegment(pos, refSeq, cid);
            answers.push(segment === undefined ? [0, 0, 0, 0, 0, 0] : [1, offset, segment.cachedLength, segment.seq,
                segment.clientId < 0 ? -1 : longOfName(c.getLongClientId(segment.clientId)), mt.getPosition(segment, refSeq, cid)]);
        }
        for (const [qd, ref, cl, ph, st, en] of textQueries) {
            if (qd !== d) continue;
            const mt = c.mergeTree;
            const local = cl < 0;
            const refSeq = local ? mt.collabWindow.currentSeq : ref;
            const cid = local ? mt.collabWindow.clientId : c.getOrAddShortClientId(name(cl));
            const helper = new MT.MergeTreeTextHelper(mt);
            texts.push(helper.getText(refSeq, cid, ph, st === null ? undefined : st, en === null ? undefined : en));
        }
        for (const [qd, ref, cl] of lenQueries) {
            if (qd !== d) continue;
            const mt = c.mergeTree;
            const local = cl < 0;
            const refSeq = local ? mt.collabWindow.currentSeq : ref;
            const cid = local ? mt.collabWindow.clientId : c.getOrAddShortClientId(name(cl));
            lengths.push(mt.getLength(refSeq, cid));
        }
        for (const [qd, st, en] of itemQueries) {
            if (qd !== d) continue;
            itemAnswers.push(getItems(c, st, en === null ? undefined : en).map(itemUnit));
        }
        for (const [qd, id, before, offset] of relQueries) {
            if (qd !== d) continue;
            const r = { id };
            if (before) r.before = true;
            if (offset !== null) r.offset = offset;
            relAnswers.push(c.posFromRelativePos(r));
        }
        // a replica holding a value only combine makes (NaN, a {value, seq} object) has no canonical dump
        dumps.push(timeOnly || (combineWatch && combineAt[d] !== undefined) ? Buffer.alloc(0) : dump(c));
    } catch (e) {
        errs[d] = String(e && e.message || e);
        dumps.push(Buffer.alloc(0));
    }
}
const secs = Number(process.hrtime.bigint() - t0) / 1e9;
const spath = path.join(dir, "snapshots.json");
if (fs.existsSync(spath)) {
    const trees = {}, loaded = [], serr = {}, tailErrors = {}, loadErrors = {};
    for (const [d, cut, loadLong] of JSON.parse(fs.readFileSync(spath))) {
        try {
            const r = await snapshotDoc(d, cut, loadLong);
            trees[d] = r.tree;
            loaded.push(r.loaded);
            if (r.tailError) tailErrors[d] = r.tailError;
            if (r.loadError) loadErrors[d] = r.loadError;
        } catch (e) {
            serr[d] = String(e && e.stack || e);
            loaded.push(Buffer.alloc(0));
        }
    }
    const off = Buffer.alloc(8 * (loaded.length + 1));
    let acc = 0;
    loaded.forEach((b, i) => { off.writeBigInt64LE(BigInt(acc), 8 * i); acc += b.length; });
    off.writeBigInt64LE(BigInt(acc), 8 * loaded.length);
    fs.writeFileSync(path.join(dir, "ref_loaded_dumps.bin"), Buffer.concat(loaded));
    fs.writeFileSync(path.join(dir, "ref_loaded_off.bin"), off);
    fs.writeFileSync(path.join(dir, "ref_snapshots.json"), JSON.stringify({ trees, errors: serr, tailErrors, loadErrors }));
    if (withHandles) fs.writeFileSync(path.join(dir, "ref_snap_handles.json"), JSON.stringify(snapHandles));
}
const lpath = path.join(dir, "snapshots_legacy.json");
if (fs.existsSync(lpath)) {
    const trees = {}, loaded = [], serr = {}, loadErrors = {};
    for (const [d, cut, loadLong] of JSON.parse(fs.readFileSync(lpath))) {
        try {
            const r = await snapshotLegacyDoc(d, cut, loadLong);
            trees[d] = r.tree;
            loaded.push(r.loaded);
            if (r.loadError) loadErrors[d] = r.loadError;
        } catch (e) { // the summarizing SharedString itself throws (e.g. createOpsFromDelta)
            serr[d] = String(e && e.message || e);
            loaded.push(Buffer.alloc(0));
        }
    }
    const off = Buffer.alloc(8 * (loaded.length + 1));
    let acc = 0;
    loaded.forEach((b, i) => { off.writeBigInt64LE(BigInt(acc), 8 * i); acc += b.length; });
    off.writeBigInt64LE(BigInt(acc), 8 * loaded.length);
    fs.writeFileSync(path.join(dir, "ref_legacy_loaded_dumps.bin"), Buffer.concat(loaded));
    fs.writeFileSync(path.join(dir, "ref_legacy_loaded_off.bin"), off);
    fs.writeFileSync(path.join(dir, "ref_snapshots_legacy.json"), JSON.stringify({ trees, errors: serr, loadErrors }));
}
if (!timeOnly) {
    const off = Buffer.alloc(8 * (ndocs + 1));
    let acc = 0;
    dumps.forEach((b, d) => { off.writeBigInt64LE(BigInt(acc), 8 * d); acc += b.length; });
    off.writeBigInt64LE(BigInt(acc), 8 * ndocs);
    fs.writeFileSync(path.join(dir, "ref_dumps.bin"), Buffer.concat(dumps));
    fs.writeFileSync(path.join(dir, "ref_dump_off.bin"), off);
}
if (withDeltas) {
    const off = Buffer.alloc(8 * (ndocs + 1));
    const parts = [];
    let acc = 0;
    for (let d = 0; d < ndocs; d++) {
        const w = deltaWords[d] || [];
        const b = Buffer.alloc(4 * w.length);
        w.forEach((x, i) => b.writeInt32LE(x, 4 * i));
        parts.push(b);
        off.writeBigInt64LE(BigInt(acc), 8 * d);
        acc += w.length;
    }
    off.writeBigInt64LE(BigInt(acc), 8 * ndocs);
    fs.writeFileSync(path.join(dir, "ref_deltas.bin"), Buffer.concat(parts));
    fs.writeFileSync(path.join(dir, "ref_delta_off.bin"), off);
}
if (regenWords.some((x) => x)) {
    const out = {};
    regenWords.forEach((w, d) => { if (w) out[d] = w; });
    fs.writeFileSync(path.join(dir, "ref_regen.json"), JSON.stringify(out));
}
if (Object.keys(refPositions).length) {
    fs.writeFileSync(path.join(dir, "ref_refpos.json"), JSON.stringify(refPositions));
    fs.writeFileSync(path.join(dir, "ref_refinside.json"), JSON.stringify(refInside));
    fs.writeFileSync(path.join(dir, "ref_refpastend.json"), JSON.stringify(refPastEnd));
}
fs.writeFileSync(path.join(dir, "ref_err.json"), JSON.stringify({ errors: errs, seconds: secs }));
if (queries.length) fs.writeFileSync(path.join(dir, "ref_answers.json"), JSON.stringify(answers));
if (textQueries.length) fs.writeFileSync(path.join(dir, "ref_texts.json"), JSON.stringify(texts));
if (itemQueries.length) fs.writeFileSync(path.join(dir, "ref_items.json"), JSON.stringify(itemAnswers));
if (lenQueries.length) fs.writeFileSync(path.join(dir, "ref_lengths.json"), JSON.stringify(lengths));
if (withHandles) {
    const snap = {};
    for (const d of Object.keys(handleTables)) snap[d] = handleTables[d].snapshot();
    fs.writeFileSync(path.join(dir, "ref_handles.json"), JSON.stringify(snap));
}
if (relQueries.length) fs.writeFileSync(path.join(dir, "ref_relpos.json"), JSON.stringify(relAnswers));
if (combineWatch) fs.writeFileSync(path.join(dir, "ref_combine.json"), JSON.stringify(combineAt));
console.log(JSON.stringify({ ndocs, errors: Object.keys(errs).length, seconds: secs, removeThrew }));
}
main().catch((e) => { console.error(e); process.exit(1); });
