"""Wire-format ingestion: sequenced messages as the reference receives them
-> op records (include/mt_oplog.h).

A message is an `ISequencedDocumentMessage` (protocol-definitions protocol.ts:132-172) whose
`contents` is an `IMergeTreeOp` (merge-tree ops.ts:63-102): insert / remove / annotate / group.
`Client.applyMsg` (client.ts:797-819) applies it; here it becomes one record per member op (a
group's members but the last flagged MT_OPF_GROUPED), with the message's client / seq / refSeq /
minSeq. The records then go to the engine like any other batch (mt_engine_submit).

Supported segment specs: a string, `{text, props}`, `{marker: {refType}, props}` (textSegment.ts,
mergeTree.ts:690-708), `[length, start]` PermutationSegment rows (matrix permutationvector.ts:
75-77) and `{items, props}` SubSequence runs (SharedObjectSequence / SharedNumberSequence, sequence
sharedSequence.ts:18-47: the items are interned, oplog.Interner.item). `relativePos1/2` (IRelativePosition {id, before, offset}, ops.ts:56-61) become MT_SEG_RELPOS records that the
engine resolves as Client.getValidOpRange does (posFromRelativePos under the op's refSeq and client); they
need an engine with the client-feature build (caps.dcap or caps.rcap > 0). Combining ops other than
`rewrite` raise ValueError.
"""
from __future__ import annotations

import json
from typing import Any, Callable, Dict, Iterable, Optional, Union

from . import oplog as ol

MSG_OP = "op"  # MessageType.Operation (protocol-definitions protocol.ts:16)


def _rel(r: Optional[Dict[str, Any]]) -> Optional[tuple]:
    if r is None:
        return None
    if not isinstance(r.get("id"), str):
        raise ValueError("a relative position needs a marker id")
    return (r["id"], bool(r.get("before")), r.get("offset"))


def _op_record(log: ol.DocLog, kind: int, op: Dict[str, Any], common: Dict[str, int]) -> None:
    t = op["type"]
    # getValidOpRange (client.ts:486-503): an absolute position wins over a relative one
    r1 = _rel(op.get("relativePos1")) if op.get("pos1") is None else None
    r2 = _rel(op.get("relativePos2")) if op.get("pos2") is None else None
    if r1 is not None or r2 is not None:
        def add(k, **kw):
            log.add_relative(k, r1, r2, **kw)
    else:
        add = log.add
    p1 = 0 if r1 is not None else op.get("pos1")
    p2 = 0 if r2 is not None else op.get("pos2")
    if t == ol.OP_INSERT:
        seg = op["seg"]
        if isinstance(seg, str):
            add(kind, pos1=p1, text=seg, **common)
        elif isinstance(seg, list):
            add(kind, pos1=p1, perm=int(seg[0]), **common)
        elif "marker" in seg:
            add(kind, pos1=p1, marker=seg["marker"]["refType"], props=seg.get("props"), **common)
        elif "items" in seg:  # SubSequence.fromJSONObject (sharedSequence.ts:23-32)
            add(kind, pos1=p1, items=seg["items"], props=seg.get("props"), **common)
        elif "text" in seg:
            add(kind, pos1=p1, text=seg["text"], props=seg.get("props"), **common)
        else:
            raise ValueError(f"unsupported segment spec {seg!r}")
    elif t == ol.OP_REMOVE:
        add(kind, pos1=p1, pos2=p2, **common)
    elif t == ol.OP_ANNOTATE:
        add(kind, pos1=p1, pos2=p2, props=op["props"], combining=combining_kind(op.get("combiningOp")), **common)
    else:
        raise ValueError(f"unsupported merge-tree op type {t}")


def combining_kind(comb) -> int:
    """An annotate's ICombiningOp (ops.ts) as mt_oplog.h MT_COMBINE_*: "rewrite", or "incr" / "consensus", which the
    engine applies as the reference's addProperties does (combine with newValue undefined, properties.ts:26-59:
    incr's NaN and consensus's new objects latch MT_E_UNSUPPORTED). A defaultValue / minValue would change what
    combine starts from: refused, as are other names."""
    if comb is None:
        return ol.COMBINE_NONE
    name = comb.get("name")
    if name == "rewrite":
        return ol.COMBINE_REWRITE
    if name in ("incr", "consensus"):
        # combine() starts from defaultValue whenever the key is present (a JSON null included: null + undefined and
        # null.seq are not undefined's results) and clamps only to a truthy minValue (properties.ts:26-38)
        if "defaultValue" in comb or comb.get("minValue"):
            raise ValueError(f"combining op {name!r} with a defaultValue / minValue is not supported")
        return ol.COMBINE_INCR if name == "incr" else ol.COMBINE_CONSENSUS
    raise ValueError(f"combining op {name!r} is not supported")


def add_message(log: ol.DocLog, msg: Dict[str, Any], client_index: Callable[[str], int]) -> None:
    """Append one sequenced message's records (Client.applyMsg, client.ts:797-819; group ops
    client.ts:782-790 -> GROUPED member records). `client_index(clientId)` maps the long client id
    to the batch's long-client index."""
    common = dict(client=client_index(msg["clientId"]), seq=int(msg["sequenceNumber"]),
                  ref_seq=int(msg["referenceSequenceNumber"]), min_seq=int(msg["minimumSequenceNumber"]))
    if msg.get("type") != MSG_OP or msg.get("contents") is None:
        log.add(ol.OP_NOOP, **common)  # updateSeqNumbers only (client.ts:818-828)
        return
    op = msg["contents"]
    if isinstance(op, str):
        op = json.loads(op)
    members = op["ops"] if op["type"] == 3 else [op]  # MergeTreeDeltaType.GROUP (ops.ts:33)
    if not members:  # an empty group applies nothing; applyMsg still runs updateSeqNumbers
        log.add(ol.OP_NOOP, **common)
        return
    for i, m in enumerate(members):
        _op_record(log, m["type"] | (ol.OPF_GROUPED if i + 1 < len(members) else 0), m, common)


def add_messages(log: ol.DocLog, msgs: Iterable[Union[Dict[str, Any], str]],
                 client_index: Callable[[str], int]) -> None:
    for m in msgs:
        add_message(log, json.loads(m) if isinstance(m, str) else m, client_index)


UNALLOCATED = -0x80000000  # Handle.unallocated (matrix handletable.ts:11)


def _props_of(props, kv, pidx: int, interner: ol.Interner):
    """(property set with JSON nulls, combining op) of a record's props index (0: none)."""
    if not pidx:
        return None, None
    pr = props[pidx - 1]
    ps = {}
    for j in range(int(pr["nkv"])):
        e = kv[int(pr["kv_off"]) + j]
        v = int(e["value"])
        ps[interner.key_str(int(e["key"]))] = None if v == 0 else interner.value_obj(v)
    return ps, ({"name": "rewrite"} if int(pr["combining"]) == ol.COMBINE_REWRITE else None)


def _relpos_of(rec, text, interner: ol.Interner):
    """(relativePos1, relativePos2) of an MT_SEG_RELPOS record: the MT_RELPOS_UNITS spec after the
    record's text (oplog.DocLog.add_relative), None for an absolute end."""
    base = int(rec["text_off"]) + int(rec["text_len"])
    u = [int(x) for x in text[base: base + ol.RELPOS_UNITS]]
    out = []
    for i in range(2):
        if not u[1] & (1 << i):
            out.append(None)
            continue
        mid, fl, lo, hi = u[2 + 4 * i: 6 + 4 * i]
        r = {"id": interner.value_obj(mid), "before": bool(fl & 1)}
        if fl & 2:
            off = lo | (hi << 16)
            r["offset"] = off - (1 << 32) if off & 0x80000000 else off
        out.append(r)
    return out


def record_op(rec, text, props, kv, interner: ol.Interner) -> Dict[str, Any]:
    """The IMergeTreeOp (ops.ts:63-102) a (non-load) record stands for: the inverse of _op_record,
    including relativePos1/2 (MT_SEG_RELPOS records carry placeholder pos1/pos2 for a relative end)."""
    kind = int(rec["kind"]) & 7
    if int(rec["kind"]) & ol.OPF_TREE:
        raise ValueError("a MergeTree-level record (MT_OPF_TREE) is not a sequenced message")
    ps, comb = _props_of(props, kv, int(rec["props"]), interner)
    sk = int(rec["seg_kind"])
    rel = _relpos_of(rec, text, interner) if sk & ol.SEG_RELPOS else (None, None)
    op = _record_op(rec, kind, sk & 0x7F, ps, comb, text, interner)
    for i, r in enumerate(rel):
        if r is not None:
            op.pop(f"pos{i + 1}", None)
            op[f"relativePos{i + 1}"] = r
    return op


def _record_op(rec, kind, sk, ps, comb, text, interner: ol.Interner) -> Dict[str, Any]:
    if kind == ol.OP_INSERT:
        if sk == ol.SEG_PERM:
            seg = [int(rec["text_len"]), UNALLOCATED]
        elif sk == ol.SEG_RUN:  # SubSequence.toJSONObject (sharedSequence.ts:43-47)
            ids = text[int(rec["text_off"]): int(rec["text_off"]) + int(rec["text_len"])]
            seg = {"items": [interner.item_obj(int(u)) for u in ids]}
            if ps is not None:
                seg["props"] = ps
        elif sk == ol.SEG_MARKER:
            seg = {"marker": {"refType": int(rec["pos2"])}}
            if ps is not None:
                seg["props"] = ps
        else:
            t = text[int(rec["text_off"]): int(rec["text_off"]) + int(rec["text_len"])].tobytes().decode("utf-16-le")
            seg = {"text": t, "props": ps} if ps is not None else t
        return {"pos1": int(rec["pos1"]), "seg": seg, "type": ol.OP_INSERT}
    if kind == ol.OP_REMOVE:
        return {"pos1": int(rec["pos1"]), "pos2": int(rec["pos2"]), "type": ol.OP_REMOVE}
    if kind == ol.OP_ANNOTATE:
        op = {"pos1": int(rec["pos1"]), "pos2": int(rec["pos2"]), "props": ps if ps is not None else {},
              "type": ol.OP_ANNOTATE}
        if comb is not None:
            op["combiningOp"] = comb
        return op
    raise ValueError(f"record kind {kind} is not a merge-tree op")


def record_messages(ops, text, props, kv, interner: ol.Interner, long_name: Callable[[int], str]):
    """The sequenced messages (ISequencedDocumentMessage, protocol.ts:132-172) of a record stream, in
    order: one per non-local record, a group's members combined into a GROUP op (createGroupOp,
    opBuilder.ts:128-134). Returns [(message, index of its last record)]."""
    out, members = [], []
    for i, rec in enumerate(ops):
        k = int(rec["kind"])
        if k & ol.OPF_LOCAL or (k & 7) >= ol.OP_RELOAD:
            continue
        if k & ol.OPF_TREE:
            raise ValueError(f"record {i}: a MergeTree-level record (MT_OPF_TREE) is not a sequenced message")
        if k & ol.OPF_GROUPED:
            members.append(record_op(rec, text, props, kv, interner))
            continue
        msg = {"clientId": long_name(int(rec["client"])), "sequenceNumber": int(rec["seq"]),
               "referenceSequenceNumber": int(rec["ref_seq"]), "minimumSequenceNumber": int(rec["min_seq"])}
        if (k & 7) == ol.OP_NOOP:
            msg["type"] = "noop"
        else:
            msg["type"] = MSG_OP
            op = record_op(rec, text, props, kv, interner)
            msg["contents"] = {"ops": members + [op], "type": 3} if members else op
        members = []
        out.append((msg, i))
    return out


class ClientNames:
    """Long client id strings <-> dense long-client indices (one table per batch)."""

    def __init__(self, names: Optional[Iterable[str]] = None) -> None:
        self.index: Dict[str, int] = {}
        self.names: list = []
        for n in names or ():
            self(n)

    def __call__(self, name: str) -> int:
        i = self.index.get(name)
        if i is None:
            i = len(self.names)
            if i >= ol.CLIENT_NONCOLLAB:
                raise ValueError("too many distinct client ids")
            self.index[name] = i
            self.names.append(name)
        return i

    def name(self, i: int) -> str:
        return self.names[i]
