"use strict";
// Known-answer scenarios of the reference's own specs, driven from JavaScript through the facade
// (fluidframework_amd/js/mergetree_gpu.js) -> Node-API addon (mt_napi.node) -> libmtreplay.so on
// the GPU. Run by tests/test_napi.py (GPU tier); prints one JSON line of results.
//   client.applyMsg.spec.ts:17-21 (setup), 88-98 (insert ack), 100-110 (remove ack),
//   261-290 (intersecting insert after local delete), mergeTree.markRangeRemoved.spec.ts:25-44.
const { ReplayEngine, DEFAULT_CAPS } = require("../fluidframework_amd/js/mergetree_gpu.js");

const out = {};
const eng = new ReplayEngine(4);

// doc 0: setup "hello world" before collaboration, then a local insert and its ack
// doc 1: a local remove and its ack; doc 2: three clients, intersecting insert after local delete
// doc 3: a remote group op (replaceRange: insert + remove in one message)
const c = [0, 1, 2, 3].map((d) => eng.client(d));
c[0].insertTextLocal(0, "hello world");
c[1].insertTextLocal(0, "hello world");
c[2].insertTextLocal(0, "a");
c[3].insertTextLocal(0, "hello world");
eng.startCollaboration(["localUser", "localUser", "A", "localUser"]);

let op = c[0].insertTextLocal(0, "abc");
out.insertBeforeAck = c[0].getText();
let seg = c[0].getContainingSegment(0).segment;
out.insertSeqBeforeAck = seg.seq;
c[0].applyMsg({ clientId: "localUser", sequenceNumber: 17, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: op });
seg = c[0].getContainingSegment(0).segment;
out.insertSeqAfterAck = seg.seq;
out.positionOfSecond = c[0].getPosition(c[0].getContainingSegment(5).segment);

op = c[1].removeRangeLocal(0, 1);
out.removeBeforeAck = c[1].getText();
c[1].applyMsg({ clientId: "localUser", sequenceNumber: 17, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: op });
out.removeAfterAck = c[1].getText();

// client.applyMsg.spec.ts:261-290 from A's replica: A deletes "a" locally, B inserts "b" at 0 and
// C inserts "c" at 1 concurrently (refSeq 0); then A's delete is sequenced.
const del = c[2].removeRangeLocal(0, 1);
c[2].applyMsg({ clientId: "B", sequenceNumber: 1, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: { type: 0, pos1: 0, seg: "b" } });
c[2].applyMsg({ clientId: "C", sequenceNumber: 2, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: { type: 0, pos1: 1, seg: "c" } });
c[2].applyMsg({ clientId: "A", sequenceNumber: 3, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: del });
out.intersecting = c[2].getText();

c[3].applyMsg({ clientId: "B", sequenceNumber: 1, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: { type: 3, ops: [{ type: 0, pos1: 11, seg: "!" }, { type: 1, pos1: 5, pos2: 11 }] } });
out.groupReplace = c[3].getText();
out.groupLength = c[3].getLength();

out.digests = Array.from(eng.digests(), (x) => x.toString(16));

// delta events (include/mt_oplog.h), as a SharedString "sequenceDelta" / "maintenance" listener sees them
const deng = new ReplayEngine(1, { ...DEFAULT_CAPS, dcap: 4096 });
const dc = deng.client(0);
deng.startCollaboration(["me"]);
dc.applyMsg({ clientId: "B", sequenceNumber: 1, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: { type: 0, pos1: 0, seg: "hello world" } });
dc.applyMsg({ clientId: "B", sequenceNumber: 2, referenceSequenceNumber: 1, minimumSequenceNumber: 0,
    type: "op", contents: { type: 2, pos1: 0, pos2: 5, props: { bold: true } } });
dc.applyMsg({ clientId: "B", sequenceNumber: 3, referenceSequenceNumber: 2, minimumSequenceNumber: 0,
    type: "op", contents: { type: 1, pos1: 5, pos2: 6 } });
out.deltas = dc.deltaEvents();

// a local reference, a remove that slides it, an insert at it, then a reconnect (regeneratePendingOp)
const reng = new ReplayEngine(1, { ...DEFAULT_CAPS, dcap: 4096, rcap: 8 });
const rc = reng.client(0);
reng.startCollaboration(["me"]);
rc.applyMsg({ clientId: "B", sequenceNumber: 1, referenceSequenceNumber: 0, minimumSequenceNumber: 0,
    type: "op", contents: { type: 0, pos1: 0, seg: "hello world" } });
const ref = rc.createLocalReference(6);
out.refBefore = rc.localReferencePosition(ref);
rc.applyMsg({ clientId: "B", sequenceNumber: 2, referenceSequenceNumber: 1, minimumSequenceNumber: 0,
    type: "op", contents: { type: 1, pos1: 5, pos2: 8 } });
out.refSlid = rc.localReferencePosition(ref);
rc.insertAtReferencePositionLocal(ref, "X");
out.refText = rc.getText();
out.refAfterInsert = rc.localReferencePosition(ref);
out.regen = rc.regeneratePendingOps();
console.log(JSON.stringify(out));
