// ref_replay_tool.mjs — the reference merge-tree client replay tool's reconstruction
// (packages/tools/merge-tree-client-replay/src/clientReplayTool.ts:113-258), restated over the REFERENCE
// merge-tree (packages/dds/merge-tree/src, type-erased by tools/ts_erase.py into a scratch dir outside the
// repo). TEST INFRASTRUCTURE: golden-vector generation only (tools/make_ref_goldens.py --replaytool); nothing in
// the product path runs it and it never reaches the GPU box.
//
// The tool's FileDeltaStorageService, TestClient and SharedString factories need the container runtime; here
// the same steps run on the reference Client directly: chunked-op reassembly (119-142), envelope unwrapping
// (144-181), attach trees (182-189, 264-356), and per client (190-245) a Client per merge tree loaded from its
// attach snapshot as that client (TestClient.createFromSnapshot: Client.load, catch-up ops awaited, not
// applied), its own ops as Client.localTransaction(createGroupOp(op)) after the pending messages with
// seq <= its refSeq, every message applied once with applyMsg. (The tool's loop tests `!==` at line 211,
// which would apply the other clients' ops locally and then remotely and never the client's own; the
// evident intent is restated, as fluidframework_amd/replay_tool.py does.)
//
// usage: node ref_replay_tool.mjs <erased-dir> <messages.json> <out.json> [--literal]
//   --literal: run the tool's loop exactly as written instead (line 211's `!==`) and report its outcome
//   out.json: {"replicas": [[path, client, text, length(, items)], ...]} in (client, path) order; items (the
//   replica's SharedSequence.getItems(0), restated over the reference Client) for SharedObjectSequence /
//   SharedNumberSequence trees only
import fs from "fs";
import path from "path";

const [erased, msgPath, outPath] = process.argv.slice(2);
const SHARED_STRING = "https://graph.microsoft.com/types/mergeTree";
const SPARSE_MATRIX = "https://graph.microsoft.com/types/mergeTree/sparse-matrix";
const OBJECT_SEQUENCE = "https://graph.microsoft.com/types/mergeTree/object-sequence";
const NUMBER_SEQUENCE = "https://graph.microsoft.com/types/mergeTree/number-sequence";
let SubSequence; // the sequence package's segment (type-erased beside merge-tree), bound in main()
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

const storageOf = (tree) => {
    const blobs = new Map(tree.entries.filter((e) => e.type === "Blob").map((e) => [e.path, e.value.contents]));
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

function ddsTrees(attach) { // getDssTreesFromAttach (322-356)
    const out = new Map();
    if (!attach.snapshot) return out;
    const root = { value: attach.snapshot, fullPath: attach.id };
    out.set(attach.type, [root]);
    const trees = [root];
    while (trees.length > 0) {
        const tree = trees.shift();
        for (const entry of tree.value.entries || []) {
            if (entry.type === "Tree") {
                trees.push({ value: entry.value, fullPath: `${tree.fullPath}/${entry.path}` });
            } else if (entry.type === "Blob" && entry.path === ".attributes") {
                const c = JSON.parse(entry.value.contents);
                if (c && c.type) {
                    if (!out.has(c.type)) out.set(c.type, [tree]); else out.get(c.type).push(tree);
                }
            }
        }
    }
    return out;
}
// processAttachMessage (264-320): the tool's mergeTreeTypes in its order, each tree with its factory's segmentFromSpec
// (SharedStringFactory: TextSegment / Marker; the object and number sequences: SubSequence.fromJSONObject). The sparse
// matrix's RunSegment / PaddingSegment are not restated here: a log holding one is refused.
function processAttach(attach, attachTrees) {
    const trees = ddsTrees(attach);
    if (trees.has(SPARSE_MATRIX)) throw new Error("sparse matrix trees are not restated");
    for (const type of [SHARED_STRING, OBJECT_SEQUENCE, NUMBER_SEQUENCE]) {
        for (const t of trees.get(type) || []) {
            const entries = [...t.value.entries];
            let content;
            while (entries.length > 0) {
                content = entries.shift();
                if (content.path === "content") break;
            }
            attachTrees.set(t.fullPath, { tree: content.value, seq: type !== SHARED_STRING });
        }
    }
}
// SharedSequence.getItems (sequence sharedSequence.ts:150-183) over the reference Client (walkSegments + getPosition)
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

const literal = process.argv.includes("--literal");
// clientReplayTool.ts:190-256 exactly as written: `message.clientId !== clientId` (211) — every OTHER client's op is
// pushed to the pending queue, applied as this client's local transaction, and pushed again; the client's own
// ops are skipped. The first exception ends the tool (it rethrows); otherwise its final asserts compare every
// replica's length and text with the readonly replica's. Returns what happened.
async function literalRun(MT, clients, attachTrees, mtMessages, specOf) {
    const { Client, createGroupOp, MergeTreeDeltaType } = MT;
    clients = new Map(clients);
    clients.set("readonly", new Map());
    for (const clientId of clients.keys()) {
        const client = clients.get(clientId);
        for (const id of attachTrees.keys()) {
            const c = new Client(specOf(id), logger);
            const { catchupOpsP } = await c.load(runtimeOf(clientId), storageOf(attachTrees.get(id).tree));
            await catchupOpsP;
            client.set(id, c);
        }
        const pending = [];
        let step = "";
        try {
            for (const message of mtMessages) {
                if (message.clientId !== clientId) {
                    pending.push(message);
                    while (pending.length > 0 && pending[0].sequenceNumber <= message.referenceSequenceNumber) {
                        const m = pending.shift();
                        step = `applyMsg seq ${m.sequenceNumber}`;
                        client.get(m.fullPath).applyMsg(m);
                    }
                    const op = message.contents;
                    step = `localTransaction of seq ${message.sequenceNumber}`;
                    client.get(message.fullPath).localTransaction(op.type === MergeTreeDeltaType.GROUP ? op : createGroupOp(op));
                    pending.push(message);
                }
            }
            for (const m of pending) {
                step = `final applyMsg seq ${m.sequenceNumber}`;
                client.get(m.fullPath).applyMsg(m);
            }
        } catch (e) {
            return { outcome: "threw", client: clientId, step, error: String(e && e.message || e) };
        }
    }
    const ro = clients.get("readonly");
    for (const [clientId, client] of clients) {
        for (const [id, c] of client) {
            const r = ro.get(id);
            if (c.getLength() !== r.getLength() || c.getText() !== r.getText()) {
                return { outcome: "assert", client: clientId, path: id, length: c.getLength(), readonlyLength: r.getLength() };
            }
        }
    }
    return { outcome: "passed" };
}

async function main() {
    const MT = await import(path.join(erased, "index.mjs"));
    const { Client, TextSegment, Marker, createGroupOp, MergeTreeDeltaType } = MT;
    ({ SubSequence } = await import(path.join(erased, "subSequence.mjs")));
    const stringSpec = (spec) => TextSegment.fromJSONObject(spec) || Marker.fromJSONObject(spec);
    const seqSpec = (spec) => SubSequence.fromJSONObject(spec);
    const specOf = (id) => (attachTrees.get(id).seq ? seqSpec : stringSpec);
    const messages = JSON.parse(fs.readFileSync(msgPath));
    const attachTrees = new Map();
    const mtMessages = [];
    const clients = new Map();
    const chunkMap = new Map();
    for (let message of messages) {
        message = JSON.parse(JSON.stringify(message));
        if (message.type === "chunkedOp") { // 119-142
            const chunk = JSON.parse(message.contents);
            if (!chunkMap.has(message.clientId)) chunkMap.set(message.clientId, new Array(chunk.totalChunks));
            const chunks = chunkMap.get(message.clientId);
            if (chunks[chunk.chunkId - 1] !== undefined) throw new Error("Chunk already assigned");
            chunks[chunk.chunkId - 1] = chunk.contents;
            if (chunk.chunkId !== chunk.totalChunks) continue;
            for (const c of chunks) if (c === undefined) throw new Error("Chunk not assigned");
            message.contents = chunks.join("");
            message.type = chunk.originalType;
            chunkMap.delete(message.clientId);
        }
        const parts = [];
        if (message.type === "op") { // 144-181
            let contents = message.contents;
            if (contents) {
                do {
                    if (typeof contents === "string") contents = JSON.parse(contents);
                    parts.push(contents.address);
                    contents = contents.contents;
                } while (contents.contents);
                if (contents.type && contents.type === "attach") {
                    const legacy = contents.content;
                    legacy.id = [...parts, legacy.id].join("/");
                    processAttach(legacy, attachTrees);
                } else {
                    const content = contents.content;
                    const p = content ? [...parts, content.address].join("/") : undefined;
                    if (content && attachTrees.has(p)) {
                        if (!clients.has(message.clientId)) clients.set(message.clientId, new Map());
                        if (!content.contents.key) {
                            message.fullPath = p;
                            message.contents = content.contents;
                            mtMessages.push(message);
                        }
                    }
                }
            }
        } else if (message.type === "attach") {
            processAttach(message.contents, attachTrees);
        }
    }
    const out = [];
    if (literal && attachTrees.size > 0) { // the loop as written (190-256), to record what it does
        fs.writeFileSync(outPath, JSON.stringify({ literal: await literalRun(MT, clients, attachTrees, mtMessages, specOf) }));
        console.log(JSON.stringify({ literal: true, messages: mtMessages.length }));
        return;
    }
    if (attachTrees.size > 0) {
        clients.set("readonly", new Map());
        for (const clientId of clients.keys()) {
            const client = clients.get(clientId);
            for (const id of attachTrees.keys()) {
                const c = new Client(specOf(id), logger);
                const { catchupOpsP } = await c.load(runtimeOf(clientId), storageOf(attachTrees.get(id).tree));
                await catchupOpsP;
                client.set(id, c);
            }
            const pending = [];
            for (const message of mtMessages) {
                if (message.clientId !== clientId) { pending.push(message); continue; }
                while (pending.length > 0 && pending[0].sequenceNumber <= message.referenceSequenceNumber) {
                    const m = pending.shift();
                    client.get(m.fullPath).applyMsg(m);
                }
                const op = message.contents;
                client.get(message.fullPath).localTransaction(op.type === MergeTreeDeltaType.GROUP ? op : createGroupOp(op));
                pending.push(message);
            }
            for (const m of pending) client.get(m.fullPath).applyMsg(m);
            for (const [id, c] of client) {
                const row = [id, clientId, new MT.MergeTreeTextHelper(c.mergeTree).getText(c.getCurrentSeq(), c.getClientId()),
                    c.getLength()];
                if (attachTrees.get(id).seq) row.push(getItems(c, 0));
                out.push(row);
            }
        }
    }
    fs.writeFileSync(outPath, JSON.stringify({ replicas: out }));
    console.log(JSON.stringify({ replicas: out.length, messages: mtMessages.length }));
}
main().catch((e) => { console.error(e); process.exit(1); });
