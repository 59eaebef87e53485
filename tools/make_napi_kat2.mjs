// make_napi_kat2.mjs — runs the steps of tests/golden/napi_kat2_steps.json on the REFERENCE merge-tree
// (type-erased by tools/ts_erase.py into a scratch directory) and writes the answers the facade must give
// (tests/golden/napi_kat2_expected.json): MergeTree.insertSegments / markRangeRemoved / annotateRange with
// explicit (refSeq, clientId, seq), startOrUpdateCollaboration with each replica's own minSeq / currentSeq,
// and MergeTreeTextHelper.getText with placeholder / start / end. TEST INFRASTRUCTURE only.
// usage: node tools/make_napi_kat2.mjs <erased-dir>
import fs from "fs";
import path from "path";

const [erased] = process.argv.slice(2);
const root = path.dirname(path.dirname(new URL(import.meta.url).pathname));
const steps = JSON.parse(fs.readFileSync(path.join(root, "tests", "golden", "napi_kat2_steps.json")));
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

async function main() {
    const MT = await import(path.join(erased, "index.mjs"));
    const { Client, TextSegment, Marker, MergeTreeTextHelper } = MT;
    const { PermutationSegment } = await import(path.join(erased, "permutationSegment.mjs"));
    const { HandleTable, isHandleValid } = await import(path.join(erased, "handletable.mjs"));
    const specToSegment = (spec) => {
        if (Array.isArray(spec)) return PermutationSegment.fromJSONObject(spec);
        const seg = TextSegment.fromJSONObject(spec) || Marker.fromJSONObject(spec);
        if (!seg) throw new Error(`bad segment spec ${JSON.stringify(spec)}`);
        return seg;
    };
    const segOf = (s) => (typeof s === "string" ? TextSegment.make(s)
        : s.marker ? Marker.make(s.marker.refType, s.props) : TextSegment.make(s.text, s.props));
    let clients = [];
    let tables = [];
    // PermutationVector's handle bookkeeping (matrix permutationvector.ts:157-183, 297-309, 338-363) around the
    // reference Client, with the reference HandleTable (as tools/ref_replay.mjs --handles)
    const hook = (c, t) => {
        c.mergeTreeDeltaCallback = (opArgs, args) => {
            if (args.operation === 0) for (const { segment } of args.deltaSegments) if (segment.reset) segment.reset();
        };
        c.mergeTreeMaintenanceCallback = (args) => {
            if (args.operation !== -3) return;
            let freed = [];
            for (const { segment } of args.deltaSegments) {
                if (isHandleValid(segment.start)) {
                    freed = freed.concat(new Array(segment.cachedLength).fill(0).map((v, i) => i + segment.start));
                }
            }
            for (const h of freed) t.free(h);
        };
    };
    const out = [];
    for (const st of steps) {
        const [op] = st;
        if (op === "collab") {
            const [, names, mins, curs] = st;
            tables = names.map(() => new HandleTable());
            clients = names.map((n, d) => {
                const c = new Client(specToSegment, logger);
                hook(c, tables[d]);
                c.startOrUpdateCollaboration(n, mins[d], curs[d]);
                return c;
            });
            continue;
        }
        const c = clients[st[1]];
        const mt = c.mergeTree;
        const cid = (x) => (x === -1 ? -1 : c.getOrAddShortClientId(x));
        if (op === "msg") {
            const [, , clientId, seq, ref, min, contents] = st;
            c.applyMsg({ clientId, sequenceNumber: seq, referenceSequenceNumber: ref, minimumSequenceNumber: min,
                type: contents ? "op" : "noop", contents: contents || undefined });
        } else if (op === "tree_insert") {
            const [, , pos, seg, ref, client, seq] = st;
            mt.insertSegments(pos, [segOf(seg)], ref, cid(client), seq, { op: { type: 0 } });
        } else if (op === "tree_remove") {
            const [, , a, b, ref, client, seq] = st;
            mt.markRangeRemoved(a, b, ref, cid(client), seq, false, { op: { type: 1 } });
        } else if (op === "tree_annotate") {
            const [, , a, b, props, ref, client, seq] = st;
            mt.annotateRange(a, b, props, undefined, ref, cid(client), seq, { op: { type: 2 } });
        } else if (op === "text" || op === "text_at") {
            const local = op === "text";
            const [ref, client, ph, a, b] = local ? [mt.collabWindow.currentSeq, null, st[2], st[3], st[4]] : st.slice(2);
            const who = local ? mt.collabWindow.clientId : cid(client);
            out.push(new MergeTreeTextHelper(mt).getText(ref, who, ph, a === null ? undefined : a, b === null ? undefined : b));
        } else if (op === "alloc") { // getAllocatedHandle
            const pos = st[2];
            const { segment, offset } = c.getContainingSegment(pos);
            let handle = segment.start + offset;
            if (!isHandleValid(handle)) {
                c.walkSegments((seg) => { seg.start = handle = tables[st[1]].allocate(); return true; }, pos, pos + 1,
                    undefined, true);
            }
            out.push(handle);
        } else if (op === "handle") { // getMaybeHandle
            const { segment, offset } = c.getContainingSegment(st[2]);
            out.push(isHandleValid(segment.start) ? segment.start + offset : -0x80000000);
        } else if (op === "handles") {
            out.push(tables[st[1]].snapshot().slice());
        } else if (op === "relpos") {
            out.push(c.posFromRelativePos(st[2]));
        } else if (op === "length") {
            out.push(c.getLength());
        } else if (op === "seg") {
            const { segment, offset } = c.getContainingSegment(st[2]);
            out.push([segment.seq, segment.cachedLength, offset]);
        } else {
            throw new Error(`unknown step ${op}`);
        }
    }
    fs.writeFileSync(path.join(root, "tests", "golden", "napi_kat2_expected.json"), JSON.stringify(out) + "\n");
    console.log(JSON.stringify(out));
}
main().catch((e) => { console.error(e); process.exit(1); });
