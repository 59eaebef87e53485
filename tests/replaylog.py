"""Recorded-document op logs for the client replay tool (test infrastructure; fluidframework_amd/replay_tool.py,
tools/ref_replay_tool.mjs, tests/test_replay_tool.py).

A log is what FileDeltaStorageService reads: a JSON array of ISequencedDocumentMessage. It is built from the
sequenced messages of a generated TestClient conflict farm (config 1: 7 editing clients in rounds of 100 ops;
the observer replica's stream, turned into wire messages by wire.record_messages) on top of a SharedString
attach snapshot (a reference v1 fixture under tests/golden/sequence_snapshots_v1), with what real logs carry
around them:
  - the attach, either as a container Attach message (ContainerMessageType.Attach) or as a legacy attach
    inside an operation's envelopes;
  - each merge-tree op wrapped in the container / data-store envelopes ({address, contents: {content:
    {address, contents: op}, type}}), a few of them JSON strings;
  - long ops split into ChunkedOp messages (containerRuntime.ts:142-150);
  - noise the tool skips: non-op messages, ops of an unattached channel, interval-collection ops (`key`) on
    the string, including a client that sends nothing else."""
import json
import os

import numpy as np

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
from fluidframework_amd import replay_tool as rt
from fluidframework_amd import wire

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DS, STR = "ds", "str"


def _attach_snapshot(fixture: str) -> dict:
    """a data store's snapshot holding one SharedString: `.attributes` naming its type + the summary tree"""
    summary = json.load(open(os.path.join(GOLDEN, "sequence_snapshots_v1", fixture + ".json")))
    attrs = {"mode": "100644", "path": ".attributes", "type": "Blob",
             "value": {"contents": json.dumps({"type": rt.SHARED_STRING, "snapshotFormatVersion": "0.1"}),
                       "encoding": "utf-8"}}
    return {"entries": [{"mode": "040000", "path": STR, "type": "Tree",
                         "value": {"entries": [attrs] + summary["entries"]}}]}


def _sequence_snapshot(kind: str, seed: int) -> dict:
    """a data store's snapshot holding one SharedObjectSequence / SharedNumberSequence: `.attributes` naming its type
    + a `content` tree, the v1 summary (snapshot.emit_v1) of a few SubSequence segments of items"""
    from fluidframework_amd import snapshot as sn
    it = ol.Interner()
    rng = np.random.default_rng(1000 + seed)
    segs = []
    for k in range(6):
        items = [_item(kind, int(x)) for x in rng.integers(48, 123, int(rng.integers(1, 40)))]
        segs.append(dict(kind=ol.SEG_RUN, flags=0, ngroups=0, len=len(items), seq=0, client=-1, removedSeq=None,
                         removedClient=0, localSeq=0, localRemovedSeq=0, leaf=0, overlap=[], props=[], refType=0,
                         text="", start=None, items=[it.item(v) for v in items]))
    tree = sn.emit_v1({"minSeq": 0, "currentSeq": 0}, segs, it, lambda i: f"c{i}")
    typ = rt.OBJECT_SEQUENCE if kind == "objects" else rt.NUMBER_SEQUENCE
    attrs = {"mode": "100644", "path": ".attributes", "type": "Blob",
             "value": {"contents": json.dumps({"type": typ, "snapshotFormatVersion": "0.1"}), "encoding": "utf-8"}}
    return {"entries": [{"mode": "040000", "path": STR, "type": "Tree", "value": {"entries": [
        attrs, {"mode": "040000", "path": "content", "type": "Tree", "value": tree}]}}]}


def _item(kind: str, unit: int):
    """the item a generated text unit stands for: a number (SharedNumberSequence) or an object (SharedObjectSequence)"""
    return unit if kind == "numbers" else {"c": chr(unit), "n": unit % 7}


def _as_items(op, kind: str):
    """a SharedString insert op's text spec as a SharedSequence.insert's {items, props} spec (sharedSequence.ts:116-125)"""
    if op.get("type") == 3:
        return dict(op, ops=[_as_items(m, kind) for m in op["ops"]])
    if op.get("type") != 0:
        return op
    seg = op["seg"]
    text, props = (seg, None) if isinstance(seg, str) else (seg["text"], seg.get("props"))
    spec = {"items": [_item(kind, ord(ch)) for ch in text]}
    if props is not None:
        spec["props"] = props
    return dict(op, seg=spec)


def _envelope(op, rng):
    c = {"address": DS, "contents": {"content": {"address": STR, "contents": op}, "type": "component"}}
    return json.dumps(c) if rng.random() < 0.1 else c


def build(seed: int, nops: int = 2000, legacy_attach: bool = False, fixture: str = "headerAndBody",
          kind: str = "string"):
    """(messages, farm batch): one recorded document. kind "objects" / "numbers": the channel is a SharedObjectSequence
    / SharedNumberSequence whose inserts carry the farm's texts as items."""
    farm = gen.generate(gen.config1(nops), ids=list(range(8 * seed, 8 * seed + 8)), threads=8)
    ops, text, props, kv = farm.doc(0)  # the observer: every sequenced message in order
    it = gen.generator_interner()
    rng = np.random.default_rng(seed)
    snap = _attach_snapshot(fixture) if kind == "string" else _sequence_snapshot(kind, seed)
    out = []
    if legacy_attach:  # an attach inside an operation's envelopes (clientReplayTool.ts:153-157)
        out.append({"clientId": "c1", "sequenceNumber": 0, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                    "type": "op", "contents": {"address": "root", "contents": {
                        "content": {"id": DS, "type": "component", "snapshot": snap}, "type": "attach"}}})
    else:
        out.append({"clientId": "c1", "sequenceNumber": 0, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                    "type": "attach", "contents": {"id": DS, "type": "component", "snapshot": snap}})
    for msg, _ in wire.record_messages(ops, text, props, kv, it, lambda i: f"c{i}"):
        base = {k: msg[k] for k in ("clientId", "sequenceNumber", "referenceSequenceNumber", "minimumSequenceNumber")}
        if msg["type"] != "op":
            out.append(dict(base, type="noop", contents=None))
            continue
        env = _envelope(msg["contents"] if kind == "string" else _as_items(msg["contents"], kind), rng)
        if legacy_attach:
            env = {"address": "root", "contents": env if isinstance(env, dict) else json.loads(env)}
        r = rng.random()
        if r < 0.06:  # a ChunkedOp split of the whole contents
            s = env if isinstance(env, str) else json.dumps(env)
            n = 2 + int(rng.integers(0, 2))
            cut = [len(s) * k // n for k in range(n + 1)]
            for k in range(n):
                out.append(dict(base, type="chunkedOp", contents=json.dumps(
                    {"chunkId": k + 1, "totalChunks": n, "contents": s[cut[k]: cut[k + 1]], "originalType": "op"})))
            continue
        out.append(dict(base, type="op", contents=env))
        if r > 0.97:  # noise: an op of an unattached channel, an interval-collection op on the string
            out.append(dict(base, type="op", contents={"address": DS, "contents": {
                "content": {"address": "map", "contents": {"type": "set", "key": "k", "value": 1}}, "type": "component"}}))
            out.append(dict(base, clientId="c99", type="op", contents={"address": DS, "contents": {
                "content": {"address": STR, "contents": {"key": "intervals", "type": "act"}}, "type": "component"}}))
            out.append(dict(base, type="noop", contents=None))
    return out, farm


def documents():
    """the two recorded documents of the fixture"""
    return [build(0, legacy_attach=False, fixture="headerAndBody")[0],
            build(1, legacy_attach=True, fixture="withMarkers")[0]]


def sequence_documents():
    """two recorded documents of SubSequence channels (refreplaytool_seq.npz): a SharedObjectSequence attached by a
    container Attach message, a SharedNumberSequence by a legacy attach"""
    return [build(2, legacy_attach=False, kind="objects")[0], build(3, legacy_attach=True, kind="numbers")[0]]
