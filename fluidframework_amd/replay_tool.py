"""Per-client reconstruction of a recorded op log: the host side of the reference's merge-tree client replay
tool (packages/tools/merge-tree-client-replay/src/clientReplayTool.ts), feeding the batched engine (SURVEY
§8(f) f2).

The reference tool reads a document's sequenced messages (FileDeltaStorageService: a JSON array of
ISequencedDocumentMessage, protocol.ts:132-172) and rebuilds, for every client that sent a merge-tree op plus a
"readonly" observer, the replica that client had: a TestClient per merge tree loaded from the tree's attach
snapshot, its own ops applied as local transactions at the point it made them, everyone's messages applied as
sequenced messages (its own as acks). Then every client's text and length must equal the observer's. Here each
(merge tree, client) replica becomes one document of an op-log batch (include/mt_oplog.h: snapshot-load
records, local edit records, sequenced message records), so one engine launch replays all of them.

Steps, each following the tool:
  - chunked ops (ContainerMessageType.ChunkedOp, containerRuntime.ts:142-150) are reassembled per client id
    and take the last chunk's message (clientReplayTool.ts:119-142);
  - an operation's envelopes are unwrapped, collecting the address path, down to the level without `contents`
    (144-152); a legacy attach at that level, or a container attach message (182-186), registers the merge
    trees of its snapshot (getDssTreesFromAttach / processAttachMessage, 264-356: every tree whose
    `.attributes` blob names a sequence type; its `content` subtree is the merge-tree snapshot); an op whose
    path is a registered merge tree and whose contents have no `key` (interval-collection ops) is a merge-tree
    message (153-179);
  - per client (190-245): replicas load the attach snapshots as that client (TestClient.createFromSnapshot:
    SnapshotLoader with the client's id; the catch-up ops it returns are awaited, not applied); for each of
    the client's own messages, the pending messages with seq <= its refSeq are applied, then its op as a local
    transaction (Client.localTransaction, client.ts:961-981: each member a local op) and the message joins
    the pending queue (its ack); the rest are applied at the end.

The tool as written tests `message.clientId !== clientId` (clientReplayTool.ts:211), which would apply the
OTHER clients' ops as local transactions and then again as remote messages, never the client's own, and
could not pass its own final equality asserts; this module follows the evident intent (own messages are local
transactions, every message is applied once, in order), and tools/ref_replay_tool.mjs restates the same loop
over the reference merge-tree to pin it. SharedObjectSequence / SharedNumberSequence trees (the tool's other
mergeTreeTypes, SubSequence.fromJSONObject specs: sequence sharedSequence.ts:18-101) replay as SubSequence documents
(mt_oplog.h MT_SEG_RUN) whose replicas also report their items (SharedSequence.getItems); a sparse matrix
(RunSegment / PaddingSegment, sequence sparsematrix.ts) raises.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional

from . import oplog as ol
from . import snapshot as sn
from . import wire

CHUNKED_OP = "chunkedOp"  # ContainerMessageType.ChunkedOp (containerRuntime.ts:137)
ATTACH = "attach"  # ContainerMessageType.Attach (134)
OPERATION = "op"  # MessageType.Operation (protocol.ts:16)
SHARED_STRING = "https://graph.microsoft.com/types/mergeTree"  # SharedStringFactory.Type (sequenceFactory.ts:23)
OBJECT_SEQUENCE = "https://graph.microsoft.com/types/mergeTree/object-sequence"  # SharedObjectSequenceFactory.Type
NUMBER_SEQUENCE = "https://graph.microsoft.com/types/mergeTree/number-sequence"  # SharedNumberSequenceFactory.Type
SPARSE_MATRIX = "https://graph.microsoft.com/types/mergeTree/sparse-matrix"      # SparseMatrixFactory.Type
SEQUENCE_TYPES = (OBJECT_SEQUENCE, NUMBER_SEQUENCE)
READONLY = "readonly"


def _parse(x):
    return json.loads(x) if isinstance(x, str) else x


def reassemble(messages: Iterable[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """Chunked ops joined per client id (clientReplayTool.ts:119-142); other messages pass unchanged."""
    out, chunks = [], {}
    for m in messages:
        if m.get("type") != CHUNKED_OP:
            out.append(m)
            continue
        ch = _parse(m["contents"])
        buf = chunks.setdefault(m["clientId"], [None] * ch["totalChunks"])
        i = ch["chunkId"] - 1
        if buf[i] is not None:
            raise ValueError("Chunk already assigned")
        buf[i] = ch["contents"]
        if ch["chunkId"] != ch["totalChunks"]:
            continue
        if any(c is None for c in buf):
            raise ValueError("Chunk not assigned")
        del chunks[m["clientId"]]
        m = dict(m, contents="".join(buf), type=ch["originalType"])
        out.append(m)
    return out


def dds_trees(attach: Dict[str, Any]) -> Dict[str, List[tuple]]:
    """type -> [(full path, tree)] of an attach message's snapshot (getDssTreesFromAttach, 322-356): the root
    is the attach's own type at its id; every tree whose `.attributes` blob names a type."""
    out: Dict[str, List[tuple]] = {}
    snap = attach.get("snapshot")
    if not snap:
        return out
    out.setdefault(attach["type"], []).append((attach["id"], snap))
    todo = [(attach["id"], snap)]
    while todo:
        path, tree = todo.pop(0)
        for e in tree.get("entries") or []:
            if e["type"] == "Tree":
                todo.append((f"{path}/{e['path']}", e["value"]))
            elif e["type"] == "Blob" and e["path"] == ".attributes":
                a = json.loads(e["value"]["contents"])
                if a and a.get("type"):
                    out.setdefault(a["type"], []).append((path, tree))
    return out


def merge_trees_of(attach: Dict[str, Any], types: Optional[Dict[str, str]] = None) -> Dict[str, dict]:
    """processAttachMessage (264-320): full path -> the `content` subtree of each merge tree in the snapshot, in the
    tool's mergeTreeTypes order (SharedString, then the object and number sequences); `types` gets each path's type."""
    found = {}
    trees = dds_trees(attach)
    if SPARSE_MATRIX in trees:
        raise ValueError(f"{SPARSE_MATRIX}: its RunSegment / PaddingSegment types are not modelled by the engine")
    for typ, path, tree in [(t, p, x) for t in (SHARED_STRING,) + SEQUENCE_TYPES for p, x in trees.get(t, [])]:
        entries = list(tree.get("entries") or [])
        content = None
        while entries:
            content = entries.pop(0)
            if content["path"] == "content":
                break
        if content is None or content["path"] != "content":
            raise ValueError(f"{path}: no content tree")
        found[path] = content["value"]
        if types is not None:
            types[path] = typ
    return found


@dataclass
class Log:
    """The merge-tree messages of a recorded document and the attach snapshots of its merge trees."""
    trees: Dict[str, dict] = field(default_factory=dict)  # full path -> merge-tree snapshot
    types: Dict[str, str] = field(default_factory=dict)  # full path -> its channel type
    messages: List[Dict[str, Any]] = field(default_factory=list)  # sequenced messages, contents = the op
    paths: List[str] = field(default_factory=list)  # each message's merge tree
    clients: List[str] = field(default_factory=list)  # clients that sent an op to a merge tree, first-seen order


def parse(messages: Iterable[Dict[str, Any]]) -> Log:
    """mainCycle's first loop (clientReplayTool.ts:113-189)."""
    log = Log()
    for m in reassemble(messages):
        t = m.get("type")
        if t == OPERATION:
            c = m.get("contents")
            if not c:
                continue
            parts = []
            while True:  # do { parse a string; push its address; descend } while (contents.contents)
                c = _parse(c)
                parts.append(c.get("address"))
                c = c.get("contents")
                if c is None:
                    raise ValueError("an operation envelope without contents")
                if not (isinstance(c, dict) and c.get("contents")):  # a string level ends the walk, as in JS
                    break
            if not isinstance(c, dict):
                continue
            if c.get("type") == ATTACH:  # a legacy attach inside the envelopes
                a = dict(c["content"])
                a["id"] = "/".join(str(p) for p in parts + [a["id"]])
                log.trees.update(merge_trees_of(a, log.types))
                continue
            content = c.get("content")
            if not isinstance(content, dict):
                continue
            path = "/".join(str(p) for p in parts + [content.get("address")])
            if path in log.trees:
                if m["clientId"] not in log.clients:  # clients.set, before the interval-op test (161-163)
                    log.clients.append(m["clientId"])
                if not _parse(content["contents"]).get("key"):  # interval-collection ops are not replayed
                    log.messages.append(dict(m, contents=_parse(content["contents"])))
                    log.paths.append(path)
        elif t == ATTACH:
            log.trees.update(merge_trees_of(_parse(m["contents"]), log.types))
    return log


def clients_of(log: Log) -> List[str]:
    """The clients that sent an op to a merge tree, in first-seen order, then the observer (clients.set, 161,
    190; a client whose only ops are interval-collection ops is one, with no own messages)."""
    return list(log.clients) + [READONLY] if log.trees else []


@dataclass
class Streams:
    """One document per (merge tree, client): batch.doc(i) is the replica of docs[i] = (path, client)."""
    batch: ol.Batch
    docs: List[tuple]
    names: wire.ClientNames
    interner: ol.Interner


def _local_records(doc: ol.DocLog, op: Dict[str, Any], names: wire.ClientNames) -> None:
    """Client.localTransaction(op or createGroupOp(op)) (client.ts:961-981): every member a local op."""
    members = op["ops"] if op["type"] == 3 else [op]
    before = len(doc.ops)
    for mem in members:
        wire._op_record(doc, mem["type"] | ol.OPF_LOCAL, mem, dict(client=0, seq=0, ref_seq=0, min_seq=0))
    for i in range(before, len(doc.ops)):
        r = list(doc.ops[i])
        if r[1] & ol.SEG_RELPOS:
            raise ValueError("a local op with a relative position is not modelled")


def streams(log: Log, interner: Optional[ol.Interner] = None) -> Streams:
    """Every client's replica of every merge tree as one batch (clientReplayTool.ts:190-245)."""
    interner = interner or ol.Interner()
    names = wire.ClientNames()
    clients = clients_of(log)
    for c in clients:
        names(c)
    docs, logs = [], []
    for client in clients:
        per = {}
        for path in log.trees:
            d = ol.DocLog(interner, local_long_id=names(client))
            sn.load_records(log.trees[path], d, names, local_client=client, catchup=False)
            per[path] = d
            docs.append((path, client))
            logs.append(d)
        pending: List[int] = []

        def apply(i):
            wire.add_message(per[log.paths[i]], log.messages[i], names)

        for i, m in enumerate(log.messages):
            if m["clientId"] != client:
                pending.append(i)
                continue
            while pending and log.messages[pending[0]]["sequenceNumber"] <= m["referenceSequenceNumber"]:
                apply(pending.pop(0))
            _local_records(per[log.paths[i]], m["contents"], names)
            pending.append(i)
        for i in pending:
            apply(i)
    return Streams(ol.Batch.from_logs(logs), docs, names, interner)


def replay(log: Log, device: int = 0, **caps):
    """Replay every (merge tree, client) replica of a recorded log in one engine launch on `device`; returns
    [(path, client, text, length, items)] in clientReplayTool's order (clients, then merge trees); items: a sequence
    tree's SharedSequence.getItems(0) values, None for a SharedString."""
    from .engine import Engine, default_caps
    st = streams(log)
    c = default_caps(0)
    c.update(ncap=2048, hcap=4096, acap=1 << 20, mcap=8192)  # capacity promotion covers larger replicas
    c.update(caps)
    eng = Engine(st.batch.ndocs, device=device, **c)  # no start_collab: each replica's COLLAB record starts it
    try:
        eng.replay(st.batch)
        err, err_op = eng.errors()
        bad = [i for i in range(st.batch.ndocs) if err[i]]
        if bad:
            i = bad[0]
            raise RuntimeError(f"replica {st.docs[i]} failed at record {err_op[i]}: error {err[i]}")
        return [(p, c_, eng.get_text(i), eng.get_length(i),
                 [st.interner.item_obj(u) for u in eng.get_items(i, 0)] if log.types.get(p) in SEQUENCE_TYPES else None)
                for i, (p, c_) in enumerate(st.docs)]
    finally:
        eng.close()


def main(argv=None) -> int:
    """`python -m fluidframework_amd.replay_tool --indir DIR [--to N] [--verbose]`: ReplayArgs (replayArgs.ts,
    main.ts) over DIR/messages.json (FileDeltaStorageService, fileDeltaStorageService.ts:18-20: the first N
    messages, getFromWebSocket(0, to)); every client's replica of every merge tree must equal the readonly
    observer's text and length (clientReplayTool.ts:246-257). Exit status 0 when they all do."""
    import argparse
    import os
    import sys
    ap = argparse.ArgumentParser(prog="replay_tool")
    ap.add_argument("--indir", required=True)
    ap.add_argument("--to", type=int, default=2 ** 53 - 1)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    with open(os.path.join(a.indir, "messages.json"), encoding="utf-8") as f:
        msgs = json.load(f)[: a.to]
    log = parse(msgs)
    for path in log.trees:
        print(f"MergeTree Found:\n {json.dumps({'fullPath': path, 'type': log.types.get(path, SHARED_STRING)})}")
    if a.verbose:
        for p, m in zip(log.paths, log.messages):
            print(f"MergeTree op {p}:\n {json.dumps(m['contents'])}")
    reps = replay(log)
    obs = {p: (t, n, it) for p, c, t, n, it in reps if c == READONLY}
    errors = 0
    for p, c, t, n, it in reps:  # the tool compares getLength and getText; a sequence's items are compared too
        if (t, n, it) != obs[p]:
            errors += 1
            if errors <= 5:
                print(f"{c} {p}: length {n} text differs from the readonly client's (length {obs[p][1]})",
                      file=sys.stderr)
    print(json.dumps({"merge_trees": len(log.trees), "messages": len(log.messages), "replicas": len(reps),
                      "errors": errors}))
    return 0 if errors == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
