"use strict";
// A SharedObjectSequence replica driven from JavaScript through the facade (fluidframework_amd/js/mergetree_gpu.js:
// insertItemsLocal, applyMsg with {items} specs, getItems / getItemCount, getText, segments) -> Node-API addon ->
// libmtreplay.so on the GPU: the steps of tests/golden/napi_subseq_steps.json, whose answers on the type-erased
// reference are tests/golden/napi_subseq_expected.json (tools/make_napi_subseq.mjs). Run by tests/test_napi.py (GPU
// tier); prints one JSON line.
const fs = require("fs");
const path = require("path");
const { ReplayEngine } = require("../fluidframework_amd/js/mergetree_gpu.js");

const steps = JSON.parse(fs.readFileSync(path.join(__dirname, "golden", "napi_subseq_steps.json")));
const eng = new ReplayEngine(1);
const c = eng.client(0);
const answers = [];
let sent;
for (const st of steps) {
    const k = st[0];
    if (k === "local") sent = c.insertItemsLocal(st[1], st[2].items, st[2].props);
    else if (k === "collab") eng.startCollaboration([st[1]]);
    else if (k === "msg") c.applyMsg(JSON.parse(JSON.stringify(st[1])));
    else if (k === "ack") {
        c.applyMsg({ clientId: "A", sequenceNumber: st[1], referenceSequenceNumber: st[2], minimumSequenceNumber: 0,
            type: "op", contents: sent });
    } else if (k === "items") answers.push(c.getItems(st[1], st[2] === null ? undefined : st[2]));
    else if (k === "count") answers.push(c.getItemCount());
    else if (k === "text") answers.push(c.getText());
    else if (k === "textph") answers.push(c.getTextAt(eng.currentSeq[0], "A", st[1], st[2], st[3])); // the local view
    else if (k === "segs") answers.push(c.segments().segments.map((s) => [s.type, s.cachedLength]));
}
console.log(JSON.stringify({ answers }));
