// make_napi_subseq.mjs — runs the steps of tests/golden/napi_subseq_steps.json (a SharedObjectSequence replica:
// SubSequence inserts, local and remote, an ack, a remove, an annotate, long runs either side of MaxRun) on the
// REFERENCE merge-tree Client with the sequence package's SubSequence (both type-erased by tools/ts_erase.py into a
// scratch directory) and writes the answers the facade must give (tests/golden/napi_subseq_expected.json):
// SharedSequence.getItems (sequence sharedSequence.ts:150-183, restated over the Client), getItemCount, getText,
// the segments' types and lengths. TEST INFRASTRUCTURE only.
// usage: node tools/make_napi_subseq.mjs <erased-dir>
import fs from "fs";
import path from "path";

const [erased] = process.argv.slice(2);
const root = path.dirname(path.dirname(new URL(import.meta.url).pathname));
const steps = JSON.parse(fs.readFileSync(path.join(root, "tests", "golden", "napi_subseq_steps.json")));
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

async function main() {
    const MT = await import(path.join(erased, "index.mjs"));
    const { Client, MergeTreeTextHelper } = MT;
    const { SubSequence } = await import(path.join(erased, "subSequence.mjs"));
    const client = new Client((spec) => SubSequence.fromJSONObject(spec), logger);
    const getItems = (start, end) => { // SharedSequence.getItems
        const out = [];
        let first;
        if (end !== undefined && end <= start) return out;
        client.walkSegments((s) => {
            if (SubSequence.is(s)) { if (first === undefined) first = s; out.push(...s.items); }
            return true;
        }, start, end);
        if (first !== undefined) out.splice(0, start - client.getPosition(first));
        if (end !== undefined) out.splice(end - start);
        return out;
    };
    const answers = [];
    let sent;
    for (const st of steps) {
        const [k] = st;
        if (k === "local") { // SharedSequence.insert: new SubSequence(items) + addProperties, insertSegmentLocal
            const seg = new SubSequence(st[2].items);
            if (st[2].props) seg.addProperties(st[2].props);
            sent = client.insertSegmentLocal(st[1], seg);
        } else if (k === "collab") {
            client.startOrUpdateCollaboration(st[1]);
        } else if (k === "msg") {
            client.applyMsg(JSON.parse(JSON.stringify(st[1])));
        } else if (k === "ack") {
            client.applyMsg({ clientId: client.longClientId, sequenceNumber: st[1], referenceSequenceNumber: st[2],
                minimumSequenceNumber: client.getCollabWindow().minSeq, type: "op", contents: sent });
        } else if (k === "items") {
            answers.push(getItems(st[1], st[2] === null ? undefined : st[2]));
        } else if (k === "count") {
            answers.push(client.getLength());
        } else if (k === "text") {
            answers.push(new MergeTreeTextHelper(client.mergeTree).getText(client.getCurrentSeq(), client.getClientId()));
        } else if (k === "textph") {
            answers.push(new MergeTreeTextHelper(client.mergeTree).getText(client.getCurrentSeq(), client.getClientId(),
                st[1], st[2], st[3]));
        } else if (k === "segs") {
            const segs = [];
            client.mergeTree.walkAllSegments(client.mergeTree.root, (s) => { segs.push([s.type, s.cachedLength]); return true; });
            answers.push(segs);
        }
    }
    fs.writeFileSync(path.join(root, "tests", "golden", "napi_subseq_expected.json"), JSON.stringify(answers));
    console.log(JSON.stringify({ answers: answers.length }));
}
main().catch((e) => { console.error(e); process.exit(1); });
