"""Wire-format ingestion: sequenced messages as the reference receives them
-> op records (include/mt_oplog.h).

A message is an `ISequencedDocumentMessage` (protocol-definitions protocol.ts:132-172) whose
`contents` is an `IMergeTreeOp` (merge-tree ops.ts:63-102): insert / remove / annotate / group.
`Client.applyMsg` (client.ts:797-819) applies it; here it becomes one record per member op (a
group's members but the last flagged MT_OPF_GROUPED), with the message's client / seq / refSeq /
minSeq. The records then go to the engine like any other batch (mt_engine_submit).

Supported segment specs: a string, `{text, props}`, `{marker: {refType}, props}` (textSegment.ts,
mergeTree.ts:690-708) and `[length, start]` PermutationSegment rows (matrix permutationvector.ts:
75-77). Positions must be absolute (`pos1`/`pos2`); `relativePos1/2` and combining ops other than
`rewrite` raise ValueError (not on the path).
"""
from __future__ import annotations

import json
from typing import Any, Callable, Dict, Iterable, Optional, Union

from . import oplog as ol

MSG_OP = "op"  # MessageType.Operation (protocol-definitions protocol.ts:16)


def _op_record(log: ol.DocLog, kind: int, op: Dict[str, Any], common: Dict[str, int]) -> None:
    t = op["type"]
    if "relativePos1" in op or "relativePos2" in op:
        raise ValueError("relative positions are not supported")
    if t == ol.OP_INSERT:
        seg = op["seg"]
        if isinstance(seg, str):
            log.add(kind, pos1=op["pos1"], text=seg, **common)
        elif isinstance(seg, list):
            log.add(kind, pos1=op["pos1"], perm=int(seg[0]), **common)
        elif "marker" in seg:
            log.add(kind, pos1=op["pos1"], marker=seg["marker"]["refType"], props=seg.get("props"), **common)
        elif "text" in seg:
            log.add(kind, pos1=op["pos1"], text=seg["text"], props=seg.get("props"), **common)
        else:
            raise ValueError(f"unsupported segment spec {seg!r}")
    elif t == ol.OP_REMOVE:
        log.add(kind, pos1=op["pos1"], pos2=op["pos2"], **common)
    elif t == ol.OP_ANNOTATE:
        comb = op.get("combiningOp")
        if comb is not None and comb.get("name") != "rewrite":
            raise ValueError(f"combining op {comb.get('name')!r} is not supported")
        log.add(kind, pos1=op["pos1"], pos2=op["pos2"], props=op["props"],
                combining=ol.COMBINE_REWRITE if comb is not None else ol.COMBINE_NONE, **common)
    else:
        raise ValueError(f"unsupported merge-tree op type {t}")


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
    for i, m in enumerate(members):
        _op_record(log, m["type"] | (ol.OPF_GROUPED if i + 1 < len(members) else 0), m, common)


def add_messages(log: ol.DocLog, msgs: Iterable[Union[Dict[str, Any], str]],
                 client_index: Callable[[str], int]) -> None:
    for m in msgs:
        add_message(log, json.loads(m) if isinstance(m, str) else m, client_index)


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
