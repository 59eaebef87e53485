"""Packed op-log format (include/mt_oplog.h) and builders.

A *document log* is one replica's arrival-ordered event stream: sequenced messages
(``Client.applyMsg``, reference ``packages/dds/merge-tree/src/client.ts:797-819``) interleaved
with the replica's own local edits (``insertSegmentLocal`` / ``removeRangeLocal`` /
``annotateRangeLocal``, client.ts:202/189/164). A *batch* is many document logs concatenated
with per-document offsets; it is what the HIP replay engine (``libmtreplay.so``) consumes.
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, NamedTuple, Optional, Sequence

import numpy as np

OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP = 0, 1, 2, 4
OP_REF = 3  # local reference (mt_oplog.h MT_OP_REF; always with OPF_LOCAL)
OP_RELOAD, OP_COLLAB, OP_APPEND = 5, 6, 7  # snapshot load records (mt_oplog.h)
OPF_LOCAL = 0x80
OPF_GROUPED = 0x40
OPF_TREE = 0x20  # MergeTree-level call (mt_oplog.h MT_OPF_TREE)
OPF_REGEN = 0x10  # regeneratePendingOp (MT_OPF_REGEN)
OPF_ATREF = 0x08  # insertAtReferencePositionLocal (MT_OPF_ATREF)
SEG_TEXT, SEG_MARKER, SEG_PERM, SEG_RUN = 0, 1, 2, 3  # SEG_RUN: SubSequence items (mt_oplog.h MT_SEG_RUN)
SEG_RELPOS = 0x80  # seg_kind flag: positions relative to markers (mt_oplog.h MT_SEG_RELPOS)
RELPOS_UNITS = 10  # MT_RELPOS_UNITS
MARKER_ID_KEY = "markerId"  # reservedMarkerIdKey (merge-tree properties / mergeTree.ts getId)
CLIENT_NONCOLLAB = 0xFFFF
_SEGMENT_KINDS = (OP_INSERT, OP_RELOAD, OP_APPEND)
COMBINE_NONE, COMBINE_REWRITE, COMBINE_INCR, COMBINE_CONSENSUS = 0, 1, 2, 3  # mt_oplog.h MT_COMBINE_*
VALUE_FALSY = 0x8000

OP_DTYPE = np.dtype(
    [
        ("kind", "u1"),
        ("seg_kind", "u1"),
        ("client", "<u2"),
        ("seq", "<i4"),
        ("ref_seq", "<i4"),
        ("min_seq", "<i4"),
        ("pos1", "<i4"),
        ("pos2", "<i4"),
        ("text_off", "<u4"),
        ("text_len", "<u2"),
        ("props", "<u2"),
    ]
)
assert OP_DTYPE.itemsize == 32
PROPS_DTYPE = np.dtype([("kv_off", "<u4"), ("nkv", "<u2"), ("combining", "u1"), ("_pad", "u1")])
KV_DTYPE = np.dtype([("key", "<u2"), ("value", "<u2")])


def canonical_json(v: Any) -> str:
    """Canonical JSON of a property value: structural equality == string equality, which is
    what ``matchProperties`` (properties.ts:61-92) tests for JSON-shaped values."""
    return json.dumps(v, sort_keys=True, separators=(",", ":"), ensure_ascii=False)


def _falsy(v: Any) -> bool:
    return v is not None and not v and not isinstance(v, (dict, list))


class Interner:
    """Batch-global key / value string tables. Value id 0 is JSON null (= delete). `items`: SubSequence items
    (mt_oplog.h MT_SEG_RUN) by canonical JSON, ids 0..65535: what a SubSequence row's units hold."""

    def __init__(self) -> None:
        self.keys: List[str] = [""]
        self.key_ids: Dict[str, int] = {}
        self.values: List[str] = ["null"]
        self.value_ids: Dict[str, int] = {}
        self.items: List[str] = []
        self.item_ids: Dict[str, int] = {}

    def item(self, v: Any) -> int:
        s = canonical_json(v)
        i = self.item_ids.get(s)
        if i is None:
            i = len(self.items)
            if i > 0xFFFF:
                raise ValueError("too many distinct SubSequence items")
            self.items.append(s)
            self.item_ids[s] = i
        return i

    def item_obj(self, i: int) -> Any:
        return json.loads(self.items[i])

    def key(self, k: str) -> int:
        i = self.key_ids.get(k)
        if i is None:
            i = len(self.keys)
            if i >= 0xFFFF:
                raise ValueError("too many distinct property keys")
            self.keys.append(k)
            self.key_ids[k] = i
        return i

    def value(self, v: Any) -> int:
        if v is None:
            return 0
        s = canonical_json(v)
        i = self.value_ids.get(s)
        if i is None:
            i = len(self.values)
            if i >= VALUE_DERIVED:  # the ids above are the engine's derived values (mt_oplog.h)
                raise ValueError("too many distinct property values")
            self.values.append(s)
            self.value_ids[s] = i
        return i | (VALUE_FALSY if _falsy(v) else 0)

    def key_str(self, i: int) -> str:
        return self.keys[i]

    def value_obj(self, i: int) -> Any:
        return json.loads(self.values[i & ~VALUE_FALSY])


def concat_records(a, b):
    """Two record streams (ops, text, props, kv) of one document as one: b's pool references are
    re-based past a's pools (e.g. a snapshot's load records followed by the ops after it)."""
    ao, at, ap, akv = a
    bo, bt, bp, bkv = b
    bo = bo.copy()
    # a PermutationSegment load record's text_off is its start handle, not a pool reference (mt_oplog.h)
    k = bo["kind"] & 7
    handle = ((k == OP_RELOAD) | (k == OP_APPEND)) & ((bo["seg_kind"] & 0x7F) == SEG_PERM)
    bo["text_off"][~handle] += np.uint32(len(at))
    has = bo["props"] != 0
    bo["props"][has] += np.uint16(len(ap))
    bp = bp.copy()
    bp["kv_off"] += np.uint32(len(akv))
    return (np.concatenate([ao, bo]), np.concatenate([at, bt]), np.concatenate([ap, bp]),
            np.concatenate([akv, bkv]))


DELTA_END = -0x80000000  # MT_DELTA_END (include/mt_oplog.h)


def decode_deltas(words):
    """A document's delta-stream words (include/mt_oplog.h MT_DELTA_*) -> [(op, seq, segments)], a segment
    being (pos, len, nd or word) and for ANNOTATE events its property deltas [(key id, value id)] or None
    (addProperties was blocked by a pending local rewrite). Raises on a truncated stream."""
    w = [int(x) for x in words]
    n, i, out = len(w), 0, []

    def need(k):
        if i + k > n:
            raise ValueError(f"truncated delta stream at word {i} of {n}")

    while i < n:
        need(2)
        op, seq = w[i], w[i + 1]
        i += 2
        segs = []
        while True:
            need(1)
            if w[i] == DELTA_END:
                break
            need(3)
            pos, ln, nd = w[i], w[i + 1], w[i + 2]
            i += 3
            pd = None
            if op == 2 and nd >= 0:
                need(nd)
                pd = [((x & 0xFFFFFFFF) >> 16, x & 0xFFFF) for x in w[i: i + nd]]
                i += nd
            segs.append((pos, ln, nd, pd))
        need(2)
        if w[i + 1] != len(segs):
            raise ValueError(f"malformed delta stream at word {i}")
        i += 2
        out.append((op, seq, segs))
    return out


# values the engine derives from incr / consensus annotates (include/mt_oplog.h MT_VALUE_DERIVED ..): host interners
# stay below VALUE_DERIVED; a dump writes each by its kind, its contents after the segment's pairs
VALUE_DERIVED, VALUE_STRCAT0, VALUE_CONS0, VALUE_NAN = 0x7F00, 0x7F00, 0x7F80, 0x7FFF
VKIND_UNKNOWN, VKIND_NUMERIC, VKIND_STRING = 0, 1, 2


class Derived(NamedTuple):
    """A property value Properties.combine made (properties.ts:26-59, newValue undefined): "nan"; "strcat": String(
    value a) + "undefined" x b (a = 0: a consensus object's "[object Object]"); "cons": {value: undefined, seq: a}."""
    kind: str
    a: int
    b: int


def derived_json(d: "Derived", interner: "Interner") -> Any:
    """The value JSON.stringify gives a derived value (SnapshotV1 serializes properties as JSON): NaN -> null, a
    consensus object -> {"seq": seq} (`value` undefined is dropped), a string as itself."""
    if d.kind == "nan":
        return None
    if d.kind == "cons":
        return {"seq": d.a}
    base = "[object Object]" if d.a == 0 else interner.value_obj(d.a)
    return base + "undefined" * d.b


def value_kinds(interner: "Interner") -> np.ndarray:
    """MT_VKIND_* per value id of an interner (mt_engine_set_value_kinds): numbers and booleans NUMERIC (incr makes
    NaN), strings STRING (incr appends "undefined"); objects and arrays stay UNKNOWN (an incr over one latches
    MT_E_UNSUPPORTED: String() of one can equal a string's, so the derived value would have no canonical base)."""
    k = np.zeros(len(interner.values), np.uint8)
    for i, sv in enumerate(interner.values):
        if i == 0:
            continue
        v = json.loads(sv)
        k[i] = VKIND_NUMERIC if isinstance(v, (bool, int, float)) else VKIND_STRING if isinstance(v, str) else 0
    return k


# canonical-dump segment flag bits (include/mt_oplog.h MT_DF_*)
DF_HAS_PROPS, DF_REMOVED, DF_LSEQ, DF_LRSEQ, DF_HANDLE = 1, 2, 4, 8, 16
HANDLE_UNALLOCATED = -0x80000000  # Handle.unallocated (matrix handletable.ts:11)


def parse_dump(b: bytes):
    """Decode the canonical dump (include/mt_oplog.h) into (header dict, [segment dicts])."""
    hdr = struct.unpack_from("<6i", b, 0)
    off = 24
    segs = []
    for _ in range(hdr[4]):
        kind, flags, nov, ngroups = struct.unpack_from("<4B", b, off)
        off += 4
        f = struct.unpack_from("<8i", b, off)
        off += 32
        ov = list(struct.unpack_from(f"<{nov}i", b, off))
        off += 4 * nov
        nprops, ref_type = struct.unpack_from("<2H", b, off)
        off += 4
        props = [struct.unpack_from("<2H", b, off + 4 * k) for k in range(nprops)]
        off += 4 * nprops
        for k, (key, v) in enumerate(props):  # derived values' contents follow the pairs (mt_oplog.h)
            if v in (VALUE_STRCAT0, VALUE_CONS0):
                a, c = struct.unpack_from("<2i", b, off)
                off += 8
                props[k] = (key, Derived("strcat", a, c) if v == VALUE_STRCAT0 else Derived("cons", a, 0))
            elif v == VALUE_NAN:
                props[k] = (key, Derived("nan", 0, 0))
        start = HANDLE_UNALLOCATED
        if flags & DF_HANDLE:  # an allocated PermutationSegment start (mt_oplog.h MT_DF_HANDLE)
            (start,) = struct.unpack_from("<i", b, off)
            off += 4
        text, items = "", None
        if kind == SEG_TEXT:
            text = b[off: off + 2 * f[0]].decode("utf-16-le")
            off += 2 * f[0]
        elif kind == SEG_RUN:  # a SubSequence's item ids
            items = list(struct.unpack_from(f"<{f[0]}H", b, off))
            off += 2 * f[0]
        segs.append(dict(kind=kind, flags=flags, ngroups=ngroups, len=f[0], seq=f[1], client=f[2],
                         removedSeq=f[3] if flags & 2 else None, removedClient=f[4], localSeq=f[5],
                         localRemovedSeq=f[6], leaf=f[7], overlap=ov, props=props, refType=ref_type, text=text,
                         start=start, items=items))
    if off != len(b):
        raise ValueError("trailing bytes after the canonical dump")
    return dict(currentSeq=hdr[0], minSeq=hdr[1], localSeq=hdr[2], length=hdr[3], nsegs=hdr[4],
                nleaf=hdr[5]), segs


@dataclass
class DocLog:
    """One replica's event stream plus its text / props pools."""

    interner: Interner
    local_long_id: int = 0
    ops: List[tuple] = field(default_factory=list)
    text: List[int] = field(default_factory=list)
    props: List[tuple] = field(default_factory=list)
    kv: List[tuple] = field(default_factory=list)
    _pindex: Dict[tuple, int] = field(default_factory=dict, repr=False)

    def _props(self, props: Optional[Dict[str, Any]], combining: int = COMBINE_NONE) -> int:
        """The record index (1-based; a record's `props` field is 16 bits) of a property set: equal sets
        (same keys in the same order, same values, same combining op) share one record."""
        if props is None:
            return 0
        kvs = tuple((self.interner.key(k), self.interner.value(v)) for k, v in props.items())
        i = self._pindex.get((kvs, combining))
        if i is not None:
            return i
        if len(self.props) >= 0xFFFF:
            raise ValueError("more than 65,535 distinct property sets in one document's log")
        off = len(self.kv)
        self.kv.extend(kvs)
        self.props.append((off, len(props), combining, 0))
        self._pindex[(kvs, combining)] = len(self.props)
        return len(self.props)

    def _text(self, text: str) -> tuple:
        units = text.encode("utf-16-le")
        arr = np.frombuffer(units, dtype="<u2")
        off = len(self.text)
        self.text.extend(arr.tolist())
        return off, len(arr)

    def add(self, kind: int, *, client: int = 0, seq: int = 0, ref_seq: int = 0, min_seq: int = 0,
            pos1: int = 0, pos2: int = 0, text: Optional[str] = None, marker: Optional[int] = None,
            props: Optional[Dict[str, Any]] = None, combining: int = COMBINE_NONE,
            perm: Optional[int] = None, items: Optional[list] = None) -> None:
        """One record; `perm` = the row count of a PermutationSegment insert / loaded segment; `items` = a SubSequence
        insert / loaded segment's items (interned: the row's units are their item ids)."""
        seg_kind = SEG_TEXT
        toff = tlen = 0
        if kind & 7 in _SEGMENT_KINDS:
            if perm is not None:
                seg_kind = SEG_PERM
                tlen = perm
            elif items is not None:
                seg_kind = SEG_RUN
                toff = len(self.text)
                self.text.extend(self.interner.item(v) for v in items)
                tlen = len(items)
            elif marker is not None:
                seg_kind = SEG_MARKER
                pos2 = marker
            else:
                toff, tlen = self._text(text or "")
        if kind & 7 in (OP_RELOAD, OP_APPEND) and seg_kind != SEG_MARKER:
            pos2, tlen = tlen, 0  # load records carry the length in pos2 (mt_oplog.h)
        pidx = self._props(props, combining)
        self.ops.append((kind, seg_kind, client, seq, ref_seq, min_seq, pos1, pos2, toff, tlen, pidx))

    def add_relative(self, kind: int, rel1: Optional[tuple] = None, rel2: Optional[tuple] = None, **kw) -> None:
        """One sequenced op record whose pos1 / pos2 are IRelativePosition (ops.ts:56-61) instead: rel =
        (marker id, before, offset or None); the MT_RELPOS_UNITS spec follows the record's text in the text
        pool (mt_oplog.h MT_SEG_RELPOS)."""
        self.add(kind, **kw)
        r = list(self.ops[-1])
        if kind & 7 == OP_INSERT and r[1] in (SEG_TEXT, SEG_RUN):
            assert r[8] + r[9] == len(self.text)
        else:
            r[8], r[9] = len(self.text), 0
        u = [self.interner.key(MARKER_ID_KEY), (1 if rel1 else 0) | (2 if rel2 else 0)]
        for rel in (rel1, rel2):
            if rel is None:
                u += [0, 0, 0, 0]
                continue
            mid, before, off = rel
            o = 0 if off is None else int(off) & 0xFFFFFFFF
            u += [self.interner.value(mid) & 0xFFFF, (1 if before else 0) | (0 if off is None else 2), o & 0xFFFF,
                  o >> 16]
        self.text.extend(u)
        r[1] |= SEG_RELPOS
        self.ops[-1] = tuple(r)

    def arrays(self):
        ops = np.array(self.ops, dtype=OP_DTYPE) if self.ops else np.zeros(0, OP_DTYPE)
        text = np.array(self.text, dtype="<u2") if self.text else np.zeros(1, "<u2")
        props = np.array(self.props, dtype=PROPS_DTYPE) if self.props else np.zeros(1, PROPS_DTYPE)
        kv = np.array(self.kv, dtype=KV_DTYPE) if self.kv else np.zeros(1, KV_DTYPE)
        return ops, text, props, kv


@dataclass
class Batch:
    """Many document logs, concatenated; offsets are per-document (length ndocs+1)."""

    ops: np.ndarray
    op_off: np.ndarray
    text: np.ndarray
    text_off: np.ndarray
    props: np.ndarray
    props_off: np.ndarray
    kv: np.ndarray
    kv_off: np.ndarray
    local_long_id: np.ndarray

    @property
    def ndocs(self) -> int:
        return len(self.op_off) - 1

    @property
    def nops(self) -> int:
        return int(self.op_off[-1])

    def doc(self, d: int):
        """(ops, text, props, kv) of document d. Pools are returned as suffixes starting at the
        document's offset: documents may share one pool (offsets need not increase)."""
        return (
            self.ops[self.op_off[d]: self.op_off[d + 1]],
            self.text[self.text_off[d]:],
            self.props[self.props_off[d]:],
            self.kv[self.kv_off[d]:],
        )

    def doc_arrays(self, d: int):
        """(ops, text, props, kv) of document d with pools cut to the document's own segment (a pool
        every document shares is returned whole)."""
        def pool(arr, off):
            if np.all(off == off[0]) or off[d + 1] < off[d]:
                return arr[off[d]:]
            seg = arr[off[d]: off[d + 1]]
            return seg if len(seg) else arr[:1]
        return (self.ops[self.op_off[d]: self.op_off[d + 1]], pool(self.text, self.text_off),
                pool(self.props, self.props_off), pool(self.kv, self.kv_off))

    def subset(self, docs: Sequence[int]) -> "Batch":
        """A batch of the given documents. A pool that is one segment per document (offsets
        increasing to the pool's end) is sliced per document; a pool all documents share (equal
        offsets) stays shared."""
        docs = [int(d) for d in docs]

        def pool(arr, off):
            if len(off) and np.all(off == off[0]):
                return np.ascontiguousarray(arr[off[0]:]), np.zeros(len(docs) + 1, np.int64)
            if np.all(np.diff(off) >= 0):
                parts = [arr[off[d]: off[d + 1]] for d in docs]
                o = np.zeros(len(docs) + 1, np.int64)
                o[1:] = np.cumsum([len(x) for x in parts])
                cat = np.concatenate(parts) if parts else arr[:0]
                return (np.ascontiguousarray(cat) if len(cat) else arr[:1].copy()), o
            raise ValueError("pool offsets are neither per-document segments nor shared")

        ops = np.concatenate([self.ops[self.op_off[d]: self.op_off[d + 1]] for d in docs]) if docs else self.ops[:0]
        op_off = np.zeros(len(docs) + 1, np.int64)
        op_off[1:] = np.cumsum([self.op_off[d + 1] - self.op_off[d] for d in docs])
        text, text_off = pool(self.text, self.text_off)
        props, props_off = pool(self.props, self.props_off)
        kv, kv_off = pool(self.kv, self.kv_off)
        return Batch(np.ascontiguousarray(ops), op_off, text, text_off, props, props_off, kv, kv_off,
                     np.asarray([self.local_long_id[d] for d in docs], np.int32))

    @staticmethod
    def from_arrays(per_doc, local_ids) -> "Batch":
        def cat(idx, dt):
            parts = [p[idx] for p in per_doc]
            off = np.zeros(len(parts) + 1, np.int64)
            off[1:] = np.cumsum([len(x) for x in parts])
            arr = np.concatenate(parts) if parts else np.zeros(0, dt)
            if len(arr) == 0:
                arr = np.zeros(1, dt)
            return np.ascontiguousarray(arr), off

        ops, op_off = cat(0, OP_DTYPE)
        if op_off[-1] == 0:
            ops = np.zeros(0, OP_DTYPE)
        text, text_off = cat(1, np.dtype("<u2"))
        props, props_off = cat(2, PROPS_DTYPE)
        kv, kv_off = cat(3, KV_DTYPE)
        return Batch(ops, op_off, text, text_off, props, props_off, kv, kv_off,
                     np.asarray(local_ids, np.int32))

    @staticmethod
    def from_logs(logs: Sequence[DocLog]) -> "Batch":
        return Batch.from_arrays([lg.arrays() for lg in logs], [lg.local_long_id for lg in logs])
