"""Host facade over the MI355X replay engine (C ABI: include/mt_engine.h, libmtreplay.so).

`Engine` holds a batch of document replicas resident in one GPU's HBM. It is the batched form
of the reference ``Client`` (packages/dds/merge-tree/src/client.ts:43): `submit` + `run` apply
whole event streams (``Client.applyMsg`` for sequenced messages, the ``*Local`` edits for local
ones), and the reads mirror ``getLength`` / ``getText`` under a (refSeq, clientId) perspective.
There is no CPU fallback: if the HIP library cannot be loaded this raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import native
from . import oplog as ol

TEXT_DEFAULT = -(1 << 31)  # MT_TEXT_DEFAULT: getValidRange's default start / end (mt_engine_get_text_range)
ERRORS = {0: "ok", 1: "MergeTree insert failed", 2: "assertion", 3: "invalid op range", 4: "unsupported",
          5: "capacity exceeded"}


class EngineError(RuntimeError):
    """A failed engine call; `code` is the MT_E_* status when the call returned one."""

    def __init__(self, msg: str, code: Optional[int] = None):
        super().__init__(msg)
        self.code = code


class SegRef(ctypes.Structure):
    """mt_seg_ref: a segment handle (row id + generation) and where the position falls in it."""
    _fields_ = [(n, ctypes.c_int32) for n in ("rid", "gen", "offset", "length", "seq", "client", "removed_seq",
                                                "removed_client", "ordinal")]


class _Caps(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("ncap", "hcap", "acap", "mcap", "gcap", "ccap", "dcap", "rcap", "pcap")]


_LIB = None
MT_VAR_SMALL_WAVES, MT_VAR_TILED_WIDE, MT_VAR_CHUNK_DOCS = 1, 2, 3  # include/mt_engine.h


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.environ.get("MT_REPLAY_LIB") or native.lib_path("libmtreplay.so")
        if not os.path.exists(path):
            raise EngineError(f"HIP replay library missing: {path} (run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.mt_engine_create.argtypes = [i32, i64, ctypes.POINTER(_Caps), ctypes.POINTER(vp)]
        L.mt_engine_destroy.argtypes = [vp]
        L.mt_engine_last_error.argtypes = [vp]
        L.mt_engine_last_error.restype = ctypes.c_char_p
        L.mt_engine_start_collab.argtypes = [vp, vp, i32, i32]
        L.mt_engine_start_collab_docs.argtypes = [vp, vp, vp, vp]
        L.mt_engine_pos_from_relative_pos.argtypes = [vp, i64, i32, i32, i32, i32, i32, i32, i32, vp]
        L.mt_engine_handle_table.argtypes = [vp, i64, vp, i64]
        L.mt_engine_handle_table.restype = i64
        L.mt_engine_get_handle.argtypes = [vp, i64, i32, vp]
        L.mt_engine_submit.argtypes = [vp, vp, vp, vp, i64, vp, vp, i64, vp, vp, i64, vp]
        L.mt_engine_run.argtypes = [vp]
        L.mt_engine_submit_run.argtypes = [vp, vp, vp, vp, i64, vp, vp, i64, vp, vp, i64, vp]
        L.mt_engine_submit_docs.argtypes = [vp, i64, vp, vp, vp, vp, i64, vp, vp, i64, vp, vp, i64, vp]
        L.mt_engine_doc_error.argtypes = [vp, i64, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.mt_host_alloc.argtypes = [i64, ctypes.POINTER(vp)]
        L.mt_host_free.argtypes = [vp]
        L.mt_engine_reset.argtypes = [vp]
        L.mt_engine_work.argtypes = [vp, vp]
        L.mt_engine_doc_times.argtypes = [vp, vp]
        L.mt_engine_set_order.argtypes = [vp, vp]
        L.mt_engine_set_variant.argtypes = [vp, i32, i32]
        L.mt_engine_set_value_kinds.argtypes = [vp, vp, i32]
        L.mt_engine_sync.argtypes = [vp]
        L.mt_engine_promoted.argtypes = [vp, vp, i64]
        L.mt_engine_promoted.restype = i64
        L.mt_engine_last_run_ms.argtypes = [vp]
        L.mt_engine_last_run_ms.restype = ctypes.c_float
        L.mt_engine_stream.argtypes = [vp]
        L.mt_engine_stream.restype = vp
        L.mt_engine_errors.argtypes = [vp, vp, vp]
        L.mt_engine_digests.argtypes = [vp, vp]
        L.mt_engine_dump.argtypes = [vp, i64, vp, i64]
        L.mt_engine_dump.restype = i64
        L.mt_engine_get_length.argtypes = [vp, i64, i32, i32, ctypes.POINTER(i32)]
        L.mt_engine_get_text.argtypes = [vp, i64, i32, i32, vp, i64]
        L.mt_engine_get_text.restype = i64
        L.mt_engine_get_text_range.argtypes = [vp, i64, i32, i32, vp, i32, i32, i32, vp, i64]
        L.mt_engine_get_text_range.restype = i64
        L.mt_engine_get_items.argtypes = [vp, i64, i32, i32, vp, i64]
        L.mt_engine_get_items.restype = i64
        L.mt_engine_stats.argtypes = [vp, vp]
        L.mt_engine_get_containing_segment.argtypes = [vp, i64, i32, i32, i32, ctypes.POINTER(SegRef)]
        L.mt_engine_get_position.argtypes = [vp, i64, i32, i32, i32, i32, ctypes.POINTER(i32)]
        L.mt_engine_delta_state.argtypes = [vp, vp, vp]
        L.mt_engine_ref_positions.argtypes = [vp, vp, vp]
        L.mt_engine_deltas.argtypes = [vp, i64, vp, i64]
        L.mt_engine_deltas.restype = i64
        L.mt_engine_resolve_remote_client_position.argtypes = [vp, i64, i32, i32, i32, ctypes.POINTER(i32)]
        L.mt_engine_adjust_position.argtypes = [vp, i64, i32, i32, i32, ctypes.POINTER(i32)]
        L.mt_engine_handle_to_position.argtypes = [vp, i64, i32, i32, ctypes.POINTER(i32)]
        L.mt_engine_get_marker_from_id.argtypes = [vp, i64, i32, i32, ctypes.POINTER(SegRef)]
        L.mt_engine_segment_ids.argtypes = [vp, i64, vp, i64]
        L.mt_engine_segment_ids.restype = i64
        L.mt_engine_ndocs.argtypes = [vp]
        L.mt_engine_ndocs.restype = i64
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_caps(ops_per_doc: int, config: int = 3) -> dict:
    """Capacities sized for the synthetic configs (high-water marks measured with the oracle)."""
    if config == 4:
        # tiled large-document profile (HotHuge: 262,144 nodes, 32-bit ids); a 1M-op config-4
        # document peaks at ~112k nodes, 422k rows and 3.2M text units
        return dict(ncap=1 << 18, hcap=1 << 12, acap=1 << 22, mcap=4096, gcap=1024, ccap=254)
    if config == 5 and ops_per_doc <= 5_000:
        # PermutationVector replicas (HotMat: 640 nodes / 5120 slots; peak ~540 nodes at 4,096)
        return dict(ncap=640, hcap=1024, acap=1 << 4, mcap=1024, gcap=1024, ccap=254)
    if config == 5:
        return dict(ncap=2048, hcap=4096, acap=1 << 4, mcap=2048, gcap=1024, ccap=254)
    if ops_per_doc <= 20_000:
        # LDS-resident profile (HotSmall: 192 nodes / 1536 slots)
        return dict(ncap=192, hcap=256, acap=1 << 16, mcap=1024, gcap=1024, ccap=254)
    return dict(ncap=16384, hcap=32768, acap=1 << 22, mcap=4096, gcap=1024, ccap=254)


class Engine:
    """A batch of `ndocs` replicas on HIP device `device`. caps["dcap"] > 0 turns on the delta event
    stream (include/mt_oplog.h MT_DELTA_*: what SharedString "sequenceDelta" / "maintenance"
    listeners see), logging up to dcap words per document; caps["rcap"] > 0 keeps up to rcap local
    references per document (MT_OP_REF records); caps["pcap"] > 0 gives every document a PermutationVector
    HandleTable of pcap handles (getAllocatedHandle records, MT_OP_NOOP | MT_OPF_LOCAL)."""

    def __init__(self, ndocs: int, device: int = 0, waves: Optional[int] = None, wide: Optional[bool] = None,
                 **caps):
        """`waves` (1 = the LDS-image build | 4 | 8) and `wide` pick a kernel build (mt_engine_set_variant); None keeps the engine's choice."""
        c = default_caps(0)
        c.update(caps)
        self.L = lib()
        self.caps = _Caps(**c)
        h = ctypes.c_void_p()
        rc = self.L.mt_engine_create(device, ndocs, ctypes.byref(self.caps), ctypes.byref(h))
        if rc != 0:
            raise EngineError(f"mt_engine_create failed: status {rc}")
        self.h = h.value
        self.ndocs = ndocs
        if waves is not None:
            self.set_variant(MT_VAR_SMALL_WAVES, waves)
        if wide is not None:
            self.set_variant(MT_VAR_TILED_WIDE, int(bool(wide)))

    def set_value_kinds(self, kinds):
        """What an incr annotate makes of each value id (oplog.value_kinds(interner); mt_engine_set_value_kinds)."""
        k = np.ascontiguousarray(kinds, np.uint8)
        self._check(self.L.mt_engine_set_value_kinds(self.h, _p(k), len(k)), "set_value_kinds")

    def set_variant(self, key: int, value: int):
        """Kernel build selection (include/mt_engine.h mt_engine_set_variant); results do not depend on it."""
        self._check(self.L.mt_engine_set_variant(self.h, key, value), "set_variant")

    def close(self):
        if getattr(self, "h", None):
            self.L.mt_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self.L.mt_engine_last_error(self.h)
            raise EngineError(f"{what} failed: status {rc}: {msg.decode() if msg else ''}", rc)

    def start_collab(self, local_long_ids, min_seq=0, cur_seq=0):
        """Client.startOrUpdateCollaboration for every document (client.ts:1053-1073); min_seq / cur_seq are
        one value for all documents or one per document (mt_engine_start_collab_docs)."""
        def per_doc(x):
            return np.ascontiguousarray(np.broadcast_to(np.asarray(x, np.int32), (self.ndocs,)))
        ids, mins, curs = per_doc(local_long_ids), per_doc(min_seq), per_doc(cur_seq)
        self._check(self.L.mt_engine_start_collab_docs(self.h, _p(ids), _p(mins), _p(curs)), "start_collab")

    def submit(self, b: ol.Batch):
        if b.ndocs != self.ndocs:
            raise EngineError("batch doc count != engine doc count")
        ops = b.ops if len(b.ops) else np.zeros(1, ol.OP_DTYPE)
        self._keep = (ops, b)
        self._check(self.L.mt_engine_submit(self.h, _p(ops), _p(b.op_off), _p(b.text), len(b.text), _p(b.text_off),
                                             _p(b.props), len(b.props), _p(b.props_off), _p(b.kv), len(b.kv),
                                             _p(b.kv_off)), "submit")

    def submit_run(self, b: ol.Batch):
        """submit + run with the hand-off overlapped (mt_engine_submit_run): chunk k of the documents replays while
        chunk k+1 is checked and copied. Returns with the replay running; sync() waits."""
        if b.ndocs != self.ndocs:
            raise EngineError("batch doc count != engine doc count")
        ops = b.ops if len(b.ops) else np.zeros(1, ol.OP_DTYPE)
        self._keep = (ops, b)
        self._check(self.L.mt_engine_submit_run(self.h, _p(ops), _p(b.op_off), _p(b.text), len(b.text),
                                                 _p(b.text_off), _p(b.props), len(b.props), _p(b.props_off),
                                                 _p(b.kv), len(b.kv), _p(b.kv_off)), "submit_run")

    def submit_docs(self, docs, b: ol.Batch):
        """Stage records for some documents only (mt_engine_submit_docs): `b` holds one log per entry of `docs`
        (increasing document ids); the next run() replays those documents alone."""
        d = np.ascontiguousarray(docs, np.int64)
        if b.ndocs != len(d):
            raise EngineError("one log per listed document")
        ops = b.ops if len(b.ops) else np.zeros(1, ol.OP_DTYPE)
        self._keep = (ops, b, d)
        self._check(self.L.mt_engine_submit_docs(self.h, len(d), _p(d), _p(ops), _p(b.op_off), _p(b.text), len(b.text),
                                                  _p(b.text_off), _p(b.props), len(b.props), _p(b.props_off),
                                                  _p(b.kv), len(b.kv), _p(b.kv_off)), "submit_docs")

    def doc_error(self, doc: int):
        """(err, err_op) of one document (mt_engine_doc_error)."""
        e, o = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.L.mt_engine_doc_error(self.h, doc, ctypes.byref(e), ctypes.byref(o)), "doc_error")
        return e.value, o.value

    def reset(self):
        self._check(self.L.mt_engine_reset(self.h), "reset")

    def work(self) -> np.ndarray:
        """(ndocs, 3) int64: sequenced messages applied, sum of rows before each, rows written."""
        out = np.zeros((self.ndocs, 3), np.int64)
        self._check(self.L.mt_engine_work(self.h, _p(out)), "work")
        return out

    def doc_times(self) -> np.ndarray:
        """(ndocs, 2) int64: each document's replay start / end in the last run, GPU constant-clock ticks
        (100 MHz, s_memrealtime)."""
        out = np.zeros((self.ndocs, 2), np.int64)
        self._check(self.L.mt_engine_doc_times(self.h, _p(out)), "doc_times")
        return out

    def set_order(self, order=None):
        """Dispatch order of the replay kernel (a permutation of the documents; None: document order)."""
        if order is None:
            self._check(self.L.mt_engine_set_order(self.h, None), "set_order")
            return
        o = np.ascontiguousarray(order, np.int32)
        if o.shape != (self.ndocs,):
            raise EngineError("set_order needs one entry per document")
        self._check(self.L.mt_engine_set_order(self.h, _p(o)), "set_order")

    def run(self):
        self._check(self.L.mt_engine_run(self.h), "run")

    def sync(self):
        self._check(self.L.mt_engine_sync(self.h), "sync")

    def replay(self, b: ol.Batch):
        self.submit(b)
        self.run()
        self.sync()

    @property
    def last_run_ms(self) -> float:
        return float(self.L.mt_engine_last_run_ms(self.h))

    @property
    def stream(self) -> int:
        return int(self.L.mt_engine_stream(self.h) or 0)

    def errors(self):
        e = np.zeros(self.ndocs, np.int32)
        eo = np.zeros(self.ndocs, np.int32)
        self._check(self.L.mt_engine_errors(self.h, _p(e), _p(eo)), "errors")
        return e, eo

    def digests(self) -> np.ndarray:
        out = np.zeros(self.ndocs, np.uint64)
        self._check(self.L.mt_engine_digests(self.h, _p(out)), "digests")
        return out

    def dump(self, doc: int) -> bytes:
        n = self.L.mt_engine_dump(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"dump failed {n}")
        buf = np.zeros(max(n, 1), np.uint8)
        n2 = self.L.mt_engine_dump(self.h, doc, _p(buf), n)
        if n2 != n:
            raise EngineError("dump size changed")
        return buf[:n].tobytes()

    def get_length(self, doc: int, ref_seq: int = 0, long_client: int = -1) -> int:
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_get_length(self.h, doc, ref_seq, long_client, ctypes.byref(v)), "get_length")
        return v.value

    def get_text(self, doc: int, ref_seq: int = 0, long_client: int = -1, placeholder: str = "",
                 start: Optional[int] = None, end: Optional[int] = None) -> str:
        """MergeTreeTextHelper.getText(refSeq, clientId, placeholder, start, end) (textSegment.ts:154-186);
        long_client < 0 = the local view (Client.getText). start / end None = getValidRange's defaults."""
        ph = np.frombuffer(placeholder.encode("utf-16-le"), "<u2").copy() if placeholder else None
        pl = 0 if ph is None else len(ph)
        a = TEXT_DEFAULT if start is None else start
        b = TEXT_DEFAULT if end is None else end
        pp = None if ph is None else _p(ph)
        n = self.L.mt_engine_get_text_range(self.h, doc, ref_seq, long_client, pp, pl, a, b, None, 0)
        if n < 0:
            raise EngineError(f"get_text failed {n}", -n)
        buf = np.zeros(max(n, 1), "<u2")
        self.L.mt_engine_get_text_range(self.h, doc, ref_seq, long_client, pp, pl, a, b, _p(buf), n)
        return buf[:n].tobytes().decode("utf-16-le")

    def get_items(self, doc: int, start: int, end: Optional[int] = None) -> list:
        """SharedSequence.getItems(start, end) (sequence sharedSequence.ts:150-183) of a SubSequence document in the
        local view: item ids (oplog.Interner.item_obj maps them back; end None = undefined)."""
        b = TEXT_DEFAULT if end is None else end
        n = self.L.mt_engine_get_items(self.h, doc, start, b, None, 0)
        if n < 0:
            raise EngineError(f"get_items failed {n}", -n)
        buf = np.zeros(max(n, 1), "<u2")
        self.L.mt_engine_get_items(self.h, doc, start, b, _p(buf), n)
        return buf[:n].tolist()

    def pos_from_relative_pos(self, doc: int, key_id: int, value_id: int, before: bool = False,
                              offset: Optional[int] = None, ref_seq: int = 0, long_client: int = -1) -> int:
        """MergeTree.posFromRelativePos (mergeTree.ts:1976-1999) of IRelativePosition {id, before, offset}: the
        marker whose property key_id (the interned "markerId") holds value_id; -1 if none holds it."""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_pos_from_relative_pos(self.h, doc, key_id, value_id, int(before),
                                                           int(offset is not None), offset or 0, ref_seq,
                                                           long_client, ctypes.byref(v)), "pos_from_relative_pos")
        return v.value

    def get_containing_segment(self, doc: int, pos: int, ref_seq: int = 0, long_client: int = -1) -> Optional[SegRef]:
        """MergeTree.getContainingSegment (mergeTree.ts:1656-1667); long_client < 0 = the local view
        (Client.getContainingSegment). None where the reference returns `segment: undefined`."""
        r = SegRef()
        self._check(self.L.mt_engine_get_containing_segment(self.h, doc, pos, ref_seq, long_client, ctypes.byref(r)),
                    "get_containing_segment")
        return None if r.rid < 0 else r

    def get_position(self, doc: int, seg: SegRef, ref_seq: int = 0, long_client: int = -1) -> int:
        """MergeTree.getPosition of a segment handle (mergeTree.ts:1619-1636)."""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_get_position(self.h, doc, seg.rid, seg.gen, ref_seq, long_client, ctypes.byref(v)),
                    "get_position")
        return v.value

    def resolve_remote_client_position(self, doc: int, pos: int, ref_seq: int, long_client: int) -> Optional[int]:
        """MergeTree.resolveRemoteClientPosition (mergeTree.ts:2140-2160); None = undefined."""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_resolve_remote_client_position(self.h, doc, pos, ref_seq, long_client,
                                                                    ctypes.byref(v)), "resolve_remote_client_position")
        return None if v.value < 0 else v.value

    def adjust_position(self, doc: int, pos: int, from_seq: int, long_client: int) -> Optional[int]:
        """PermutationVector.adjustPosition (permutationvector.ts:185-196); None = undefined."""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_adjust_position(self.h, doc, pos, from_seq, long_client, ctypes.byref(v)),
                    "adjust_position")
        return None if v.value < 0 else v.value

    def handle_to_position(self, doc: int, handle: int, local_seq: int) -> int:
        """PermutationVector.handleToPosition (permutationvector.ts:198-253)."""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_handle_to_position(self.h, doc, handle, local_seq, ctypes.byref(v)),
                    "handle_to_position")
        return v.value

    def get_marker_from_id(self, doc: int, key_id: int, value_id: int) -> Optional[SegRef]:
        """MergeTree.getMarkerFromId (mergeTree.ts:1965-1967); None if no marker holds the id."""
        r = SegRef()
        self._check(self.L.mt_engine_get_marker_from_id(self.h, doc, key_id, value_id, ctypes.byref(r)),
                    "get_marker_from_id")
        return None if r.rid < 0 else r

    def segment_ids(self, doc: int) -> np.ndarray:
        """(nsegs, 2) int32: every segment's (rid, gen) in walkAllSegments (canonical dump) order."""
        n = self.L.mt_engine_segment_ids(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"segment_ids failed {n}", -n)
        out = np.zeros((max(n, 1), 2), np.int32)
        m = self.L.mt_engine_segment_ids(self.h, doc, _p(out), n)
        if m != n:
            raise EngineError("segment count changed")
        return out[:n]

    def promoted(self) -> np.ndarray:
        """The documents the last sync re-replayed in a larger profile (capacity promotion)."""
        n = self.L.mt_engine_promoted(self.h, None, 0)
        out = np.zeros(max(n, 1), np.int64)
        self.L.mt_engine_promoted(self.h, _p(out), n)
        return out[:n]

    def delta_state(self):
        """Per doc (words emitted since create/reset, FNV-1a-64 of them) of the delta stream."""
        n = np.zeros(self.ndocs, np.int64)
        h = np.zeros(self.ndocs, np.uint64)
        self._check(self.L.mt_engine_delta_state(self.h, _p(n), _p(h)), "delta_state")
        return n, h

    def deltas(self, doc: int) -> np.ndarray:
        """The logged delta-stream words of one document (at most dcap)."""
        n = self.L.mt_engine_deltas(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"deltas failed {n}")
        buf = np.zeros(max(n, 1), np.int32)
        self.L.mt_engine_deltas(self.h, doc, _p(buf), n)
        return buf[:n]

    def ref_positions(self):
        """Per doc the number of local references, and (ndocs, rcap) LocalReference.toPosition() of each
        (-1: detached)."""
        n = np.zeros(self.ndocs, np.int32)
        pos = np.full((self.ndocs, max(self.caps.rcap, 1)), -1, np.int32)
        self._check(self.L.mt_engine_ref_positions(self.h, _p(n), _p(pos)), "ref_positions")
        return n, pos

    def handle_table(self, doc: int) -> np.ndarray:
        """PermutationVector's HandleTable.snapshot() of one document (handletable.ts:80-82)"""
        n = self.L.mt_engine_handle_table(self.h, doc, None, 0)
        if n < 0:
            raise EngineError(f"handle_table failed {n}")
        buf = np.zeros(max(n, 1), np.int32)
        self.L.mt_engine_handle_table(self.h, doc, _p(buf), n)
        return buf[:n]

    def get_handle(self, doc: int, pos: int) -> int:
        """PermutationVector.getMaybeHandle(pos) (HandleCache.getHandle): start + offset, -2**31 unallocated"""
        v = ctypes.c_int32()
        self._check(self.L.mt_engine_get_handle(self.h, doc, pos, ctypes.byref(v)), "get_handle")
        return v.value

    def stats(self) -> np.ndarray:
        out = np.zeros((self.ndocs, 4), np.int32)
        self._check(self.L.mt_engine_stats(self.h, _p(out)), "stats")
        return out


class PinnedArray:
    """A numpy array over pinned host memory (mt_host_alloc): op logs built or kept there hand off by DMA alone."""

    def __init__(self, shape, dtype):
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        p = ctypes.c_void_p()
        rc = lib().mt_host_alloc(n, ctypes.byref(p))
        if rc != 0:
            raise EngineError(f"mt_host_alloc({n}) failed: status {rc}")
        self._p = p.value
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(self._p)
        self.array = np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if getattr(self, "_p", None):
            self.array = None
            lib().mt_host_free(self._p)
            self._p = None

    __del__ = close


def pinned_batch(b: ol.Batch):
    """A copy of the batch with its records and text in pinned host memory; returns (batch, keep-alive handles)."""
    import dataclasses
    ops = PinnedArray(b.ops.shape, b.ops.dtype)
    ops.array[...] = b.ops
    text = PinnedArray(b.text.shape, b.text.dtype)
    text.array[...] = b.text
    return dataclasses.replace(b, ops=ops.array, text=text.array), (ops, text)
