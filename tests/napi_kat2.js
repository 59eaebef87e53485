"use strict";
// The steps of tests/golden/napi_kat2_steps.json through the facade (fluidframework_amd/js/mergetree_gpu.js)
// -> Node-API addon -> libmtreplay.so on the GPU: MergeTree-level insertSegments / markRangeRemoved /
// annotateRange with explicit (refSeq, clientId, seq), startCollaboration with per-document minSeq /
// currentSeq, getText / getTextWithPlaceholders / getTextAt with placeholder, start and end, ops with relative
// positions and posFromRelativePos, PermutationVector getAllocatedHandle / getMaybeHandle / handleTable. Prints the
// answers as one JSON line; tests/test_napi.py compares them with the reference's
// (tests/golden/napi_kat2_expected.json, tools/make_napi_kat2.mjs).
const fs = require("fs");
const path = require("path");
const { ReplayEngine, addon, DEFAULT_CAPS } = require("../fluidframework_amd/js/mergetree_gpu.js");

const steps = JSON.parse(fs.readFileSync(path.join(__dirname, "golden", "napi_kat2_steps.json")));
let eng, clients;
const out = [];
for (const st of steps) {
    const [op] = st;
    if (op === "collab") {
        const [, names, mins, curs] = st;
        // client-feature build: relative positions, PermutationVector handles
        eng = new ReplayEngine(names.length, { ...DEFAULT_CAPS, dcap: 1024, pcap: 256 });
        clients = names.map((_, d) => eng.client(d));
        eng.startCollaboration(names, mins, curs);
        continue;
    }
    const c = clients[st[1]];
    if (op === "msg") {
        const [, , clientId, seq, ref, min, contents] = st;
        c.applyMsg({ clientId, sequenceNumber: seq, referenceSequenceNumber: ref, minimumSequenceNumber: min,
            type: contents ? "op" : "noop", contents: contents || undefined });
    } else if (op === "tree_insert") {
        const [, , pos, seg, ref, client, seq] = st;
        c.mergeTree.insertSegments(pos, [seg], ref, client, seq);
    } else if (op === "tree_remove") {
        const [, , a, b, ref, client, seq] = st;
        c.mergeTree.markRangeRemoved(a, b, ref, client, seq);
    } else if (op === "tree_annotate") {
        const [, , a, b, props, ref, client, seq] = st;
        c.mergeTree.annotateRange(a, b, props, undefined, ref, client, seq);
    } else if (op === "text") {
        const [, , ph, a, b] = st;
        const s = a === null ? undefined : a, e = b === null ? undefined : b;
        if (ph === "") out.push(c.getText(s, e));
        else if (ph === " ") out.push(c.getTextWithPlaceholders(s, e));
        else out.push(addon.getText(c.read(), c.doc, 0, -1, ph, s, e));
    } else if (op === "text_at") {
        const [, , ref, client, ph, a, b] = st;
        out.push(c.getTextAt(ref, client, ph, a === null ? undefined : a, b === null ? undefined : b));
    } else if (op === "alloc") {
        out.push(c.getAllocatedHandle(st[2]));
    } else if (op === "handle") {
        out.push(c.getMaybeHandle(st[2]));
    } else if (op === "handles") {
        out.push(Array.from(c.handleTable()));
    } else if (op === "relpos") {
        out.push(c.posFromRelativePos(st[2]));
    } else if (op === "length") {
        out.push(c.getLength());
    } else if (op === "seg") {
        const { segment, offset } = c.getContainingSegment(st[2]);
        out.push([segment.seq, segment.length, offset]);
    } else {
        throw new Error(`unknown step ${op}`);
    }
}
let unsupported = false;
try { clients[0].getTextAt(0, "B", "*"); } catch (e) { unsupported = /unsupported|status 4/i.test(String(e.message)); }
console.log(JSON.stringify({ answers: out, starUnsupported: unsupported }));
