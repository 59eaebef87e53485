"use strict";
// Per-read latency of the interactive facade (fluidframework_amd/js/mergetree_gpu.js) on a large engine: each read
// flushes only the documents with queued records (mt_engine_submit_docs: one launch of that many workgroups) and
// checks the one document's error (mt_engine_doc_error). Prints one JSON line.
//   node tools/facade_latency.js [ndocs=65536] [iterations=200]
// Cycles timed (process.hrtime, wall clock around the JS calls):
//   edit+getText: insertTextLocal on one document, then getText of it (flush of 1 document + the read kernel)
//   getLength:    a read with nothing queued (no flush: the read kernel alone)
//   remote+getLength: a sequenced remote insert (applyMsg) then getLength
//   64 edits+getText: one edit on each of 64 documents, then one read (a flush of 64 documents in one launch)
// Every answer is checked against the text the script expects.
const { ReplayEngine } = require("../fluidframework_amd/js/mergetree_gpu.js");

const ndocs = parseInt(process.argv[2] || "65536", 10);
const iters = parseInt(process.argv[3] || "200", 10);
const t0 = process.hrtime.bigint();
const eng = new ReplayEngine(ndocs);
const names = Array.from({ length: ndocs }, () => "local");
eng.startCollaboration(names);
const tCreate = Number(process.hrtime.bigint() - t0) / 1e6;
const expect = new Map(); // doc -> expected local text (lower half)
const remoteLen = new Map(); // doc -> expected length (upper half: remote inserts only)
const half = Math.max(1, ndocs >> 1);
const clients = new Map();
const client = (d) => { if (!clients.has(d)) clients.set(d, eng.client(d)); return clients.get(d); };
let rng = 12345;
const rand = (n) => { rng = (rng * 1103515245 + 12345) & 0x7fffffff; return rng % n; };
const ms = (a) => Number(process.hrtime.bigint() - a) / 1e6;
const stats = (xs) => {
    const s = xs.slice().sort((a, b) => a - b);
    return { n: s.length, p50: s[Math.floor(s.length / 2)], p90: s[Math.floor(s.length * 0.9)],
        mean: s.reduce((a, b) => a + b, 0) / s.length, max: s[s.length - 1] };
};
const check = (d, got) => {
    if (got !== (expect.get(d) || "")) throw new Error(`doc ${d}: got ${JSON.stringify(got)} want ${JSON.stringify(expect.get(d))}`);
};
const edit = (d) => {
    const cur = expect.get(d) || "";
    const pos = rand(cur.length + 1);
    const s = String.fromCharCode(97 + rand(26));
    client(d).insertTextLocal(pos, s);
    expect.set(d, cur.slice(0, pos) + s + cur.slice(pos));
};
// warm-up: the first flush / read kernels load the code objects
edit(0); check(0, client(0).getText());

const editRead = [], readOnly = [], remoteRead = [], batchRead = [];
for (let i = 0; i < iters; i++) {
    const d = rand(half); // local edits on the lower half, remote inserts on the upper half (texts checked below)
    let t = process.hrtime.bigint();
    edit(d);
    const txt = client(d).getText();
    editRead.push(ms(t));
    check(d, txt);

    t = process.hrtime.bigint();
    const len = client(d).getLength();
    readOnly.push(ms(t));
    if (len !== expect.get(d).length) throw new Error(`doc ${d}: length ${len}`);

    // a sequenced insert by another client at position 0 (refSeq = the current seq: sees everything sequenced)
    const r = half + rand(ndocs - half);
    const c = client(r);
    const cs = c.getCurrentSeq();
    t = process.hrtime.bigint();
    c.applyMsg({ clientId: "remote", sequenceNumber: cs + 1, referenceSequenceNumber: cs, minimumSequenceNumber: 0,
        type: "op", contents: { type: 0, pos1: 0, seg: "R" } });
    const l2 = c.getLength();
    remoteRead.push(ms(t));
    remoteLen.set(r, (remoteLen.get(r) || 0) + 1);
    if (l2 !== remoteLen.get(r)) throw new Error(`doc ${r}: length after remote insert ${l2}`);

    if (i % 4 === 0) {
        const docs = Array.from({ length: 64 }, () => rand(half));
        t = process.hrtime.bigint();
        for (const x of docs) edit(x);
        const t2 = client(docs[0]).getText();
        batchRead.push(ms(t));
        check(docs[0], t2);
    }
}
// every touched document's text, once more, through the whole path
for (const [d, want] of expect) check(d, client(d).getText());
console.log(JSON.stringify({
    ndocs, iterations: iters, create_and_collab_ms: tCreate, docs_touched: expect.size + remoteLen.size,
    unit: "ms", edit_then_getText: stats(editRead), getLength_nothing_queued: stats(readOnly),
    remote_applyMsg_then_getLength: stats(remoteRead), edits_on_64_docs_then_getText: stats(batchRead),
    answers_checked: true,
}));
