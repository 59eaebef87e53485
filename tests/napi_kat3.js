"use strict";
// The steps of tests/golden/napi_kat3_steps.json through the facade (fluidframework_amd/js/mergetree_gpu.js) ->
// Node-API addon -> libmtreplay.so on the GPU: walkSegments (with splitRange), getPropertiesAtPosition,
// getRangeExtentsOfPosition, resolveRemoteClientPosition, localTransaction, insertSegmentLocal, findTile,
// getMarkerFromId, annotateMarker, removeLocalReference, PermutationVector adjustPosition / handleToPosition.
// Prints the answers as one JSON line; tests/test_napi.py compares them with the reference's
// (tests/golden/napi_kat3_expected.json, tools/make_napi_kat3.mjs).
const fs = require("fs");
const path = require("path");
const { ReplayEngine, DEFAULT_CAPS } = require("../fluidframework_amd/js/mergetree_gpu.js");

function canonical(v) {
    if (v === undefined) return null;
    if (v === null || typeof v !== "object") return JSON.stringify(v);
    if (Array.isArray(v)) return "[" + v.map(canonical).join(",") + "]";
    return "{" + Object.keys(v).filter((k) => v[k] !== undefined).sort()
        .map((k) => JSON.stringify(k) + ":" + canonical(v[k])).join(",") + "}";
}
const segOut = (seg) => [seg.type, seg.cachedLength, seg.seq,
    seg.type === "TextSegment" ? seg.text : seg.type === "Marker" ? seg.refType : seg.start,
    canonical(seg.properties), seg.removedSeq === undefined ? null : seg.removedSeq];

const steps = JSON.parse(fs.readFileSync(path.join(__dirname, "golden", "napi_kat3_steps.json")));
let eng, clients, refs;
const out = [];
for (const st of steps) {
    const [op] = st;
    if (op === "collab") {
        const [, names, mins, curs] = st;
        eng = new ReplayEngine(names.length, { ...DEFAULT_CAPS, dcap: 1024, rcap: 16, pcap: 256 });
        clients = names.map((_, d) => eng.client(d));
        refs = names.map(() => []);
        eng.startCollaboration(names, mins, curs);
        continue;
    }
    const c = clients[st[1]];
    if (op === "msg") {
        const [, , clientId, seq, ref, min, contents] = st;
        c.applyMsg({ clientId, sequenceNumber: seq, referenceSequenceNumber: ref, minimumSequenceNumber: min,
            type: contents ? "op" : "noop", contents: contents || undefined });
    } else if (op === "text") {
        out.push(c.getText());
    } else if (op === "length") {
        out.push(c.getLength());
    } else if (op === "walk") {
        const [, , a, b, split] = st;
        const seen = [];
        c.walkSegments((seg, pos, refSeq, clientId, s, e) => { seen.push([pos, s, e, ...segOut(seg)]); return true; },
            a === null ? undefined : a, b === null ? undefined : b, undefined, split);
        out.push(seen);
    } else if (op === "props_at") {
        out.push(canonical(c.getPropertiesAtPosition(st[2])));
    } else if (op === "extents") {
        const { posStart, posAfterEnd } = c.getRangeExtentsOfPosition(st[2]);
        out.push([posStart === undefined ? null : posStart, posAfterEnd === undefined ? null : posAfterEnd]);
    } else if (op === "tile") {
        const [, , pos, label, preceding] = st;
        const r = c.findTile(pos === null ? undefined : pos, label, preceding);
        out.push(r === undefined ? null : [r.pos, r.tile.refType, (r.tile.properties && r.tile.properties.markerId) || null]);
    } else if (op === "marker") {
        const m = c.getMarkerFromId(st[2]);
        out.push(m === undefined ? null : [m.pos, m.refType, canonical(m.properties)]);
    } else if (op === "resolve") {
        const [, , pos, ref, client] = st;
        const r = c.resolveRemoteClientPosition(pos, ref, client);
        out.push(r === undefined ? null : r);
    } else if (op === "ins_local") {
        c.insertSegmentLocal(st[2], st[3]);
    } else if (op === "txn") {
        c.localTransaction(st[2]);
    } else if (op === "annotate_marker") {
        const m = c.getMarkerFromId(st[2]);
        const r = m === undefined ? undefined : c.annotateMarker(m, st[3], undefined);
        out.push(r === undefined ? null : canonical(r));
    } else if (op === "ref_create") {
        refs[st[1]].push(c.createLocalReference(st[2], st[3]));
    } else if (op === "ref_remove") {
        c.removeLocalReference(refs[st[1]][st[2]]);
    } else if (op === "ref_pos") {
        out.push(c.localReferencePosition(refs[st[1]][st[2]]));
    } else if (op === "alloc") {
        out.push(c.getAllocatedHandle(st[2]));
    } else if (op === "adjust") {
        const [, , pos, fromSeq, client] = st;
        const r = c.adjustPosition(pos, fromSeq, client);
        out.push(r === undefined ? null : r);
    } else if (op === "h2p") {
        out.push(c.handleToPosition(st[2], st[3] === null ? undefined : st[3]));
    } else {
        throw new Error(`unknown step ${op}`);
    }
}
// a perspective the engine does not answer (refSeq below a refSeq client C has sent an op under) throws
let refused = false;
try { clients[0].resolveRemoteClientPosition(2, 1, "C"); } catch (e) { refused = /unsupported|status 4/i.test(String(e.message)); }
console.log(JSON.stringify({ answers: out, refused }));
