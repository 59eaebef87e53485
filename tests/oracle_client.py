"""ctypes wrapper of the CPU oracle (oracle/build/libmt_oracle.so) — TEST INFRASTRUCTURE.

`OracleClient` mirrors the reference's `TestClient` surface
(packages/dds/merge-tree/src/test/testClient.ts:42-261) so that the reference's known-answer
scenarios read the same here: local edits return an op that is later sequenced with
`make_op_message` and fed back through `apply_msg`.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import subprocess
from typing import Any, Dict, List, Optional

import numpy as np

from fluidframework_amd import oplog as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ROOT, "oracle", "build", "libmt_oracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(path)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.mto_create.restype = vp
        L.mto_destroy.argtypes = [vp]
        L.mto_set_options.argtypes = [vp, i32]
        L.mto_start_collab.argtypes = [vp, i32, i32, i32]
        L.mto_apply.argtypes = [vp, vp, vp, vp, vp]
        L.mto_replay.argtypes = [vp, vp, i64, vp, vp, vp]
        L.mto_error.argtypes = [vp]
        L.mto_local_length.argtypes = [vp]
        L.mto_get_length.argtypes = [vp, i32, i32]
        L.mto_get_text.argtypes = [vp, i32, i32, vp, i64]
        L.mto_get_text.restype = i64
        L.mto_short_id.argtypes = [vp, i32]
        L.mto_current_seq.argtypes = [vp]
        L.mto_min_seq.argtypes = [vp]
        L.mto_pending_groups.argtypes = [vp]
        L.mto_dump.argtypes = [vp, vp, i64]
        L.mto_dump.restype = i64
        L.mto_digest.argtypes = [vp]
        L.mto_digest.restype = ctypes.c_uint64
        L.mto_stats.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int)] * 4
        L.mto_check_partials.argtypes = [vp, i32, i32]
        L.mto_get_containing.argtypes = [vp, i32, i32, i32, vp]
        L.mto_replay_batch.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp]
        L.mto_replay_batch.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclasses.dataclass
class Msg:
    """An op (IMergeTreeOp) plus, once sequenced, its ISequencedDocumentMessage fields."""

    kind: int
    pos1: int = 0
    pos2: int = 0
    text: Optional[str] = None
    marker: Optional[int] = None
    props: Optional[Dict[str, Any]] = None
    combining: int = ol.COMBINE_NONE
    client: int = 0
    seq: int = -1
    ref_seq: int = 0
    min_seq: int = 0

    def sequenced(self, seq: int, ref_seq: int, client: int, min_seq: int = 0) -> "Msg":
        return dataclasses.replace(self, seq=seq, ref_seq=ref_seq, client=client, min_seq=min_seq)

    def add_to(self, log: ol.DocLog, local: bool = False) -> None:
        kind = self.kind | (ol.OPF_LOCAL if local else 0)
        log.add(kind, client=self.client, seq=self.seq, ref_seq=self.ref_seq, min_seq=self.min_seq,
                pos1=self.pos1, pos2=self.pos2, text=self.text, marker=self.marker, props=self.props,
                combining=self.combining)


class OracleClient:
    """One replica (reference `Client`) held by the C oracle."""

    def __init__(self, interner: Optional[ol.Interner] = None, verify: bool = False):
        self.L = lib()
        self.h = self.L.mto_create()
        self.interner = interner or ol.Interner()
        self.long_client_id: Optional[int] = None
        if verify:
            self.L.mto_set_options(self.h, 1)

    def __del__(self):
        try:
            if self.h:
                self.L.mto_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # --- collaboration -------------------------------------------------------------------
    def start_collab(self, long_id: int, min_seq: int = 0, cur_seq: int = 0) -> None:
        self.long_client_id = long_id
        self.L.mto_start_collab(self.h, long_id, min_seq, cur_seq)

    # --- apply ---------------------------------------------------------------------------
    def _apply(self, m: Msg, local: bool) -> int:
        log = ol.DocLog(self.interner)
        m.add_to(log, local)
        ops, text, props, kv = log.arrays()
        return self.L.mto_apply(self.h, _p(ops), _p(text), _p(props), _p(kv))

    def apply_msg(self, m: Msg) -> int:
        return self._apply(m, False)

    def replay(self, log: ol.DocLog) -> int:
        ops, text, props, kv = log.arrays()
        return self.L.mto_replay(self.h, _p(ops), len(ops), _p(text), _p(props), _p(kv))

    def replay_arrays(self, ops, text, props, kv) -> int:
        return self.L.mto_replay(self.h, _p(ops), len(ops), _p(text), _p(props), _p(kv))

    def insert_text_local(self, pos: int, text: str, props=None) -> Optional[Msg]:
        m = Msg(ol.OP_INSERT, pos1=pos, text=text, props=props)
        if len(text) == 0:
            return None
        return m if self._apply(m, True) == 0 else None

    def insert_marker_local(self, pos: int, ref_type: int, props=None) -> Optional[Msg]:
        m = Msg(ol.OP_INSERT, pos1=pos, marker=ref_type, props=props)
        return m if self._apply(m, True) == 0 else None

    def remove_range_local(self, start: int, end: int) -> Optional[Msg]:
        m = Msg(ol.OP_REMOVE, pos1=start, pos2=end)
        return m if self._apply(m, True) == 0 else None

    def annotate_range_local(self, start: int, end: int, props, combining=ol.COMBINE_NONE) -> Optional[Msg]:
        m = Msg(ol.OP_ANNOTATE, pos1=start, pos2=end, props=props, combining=combining)
        return m if self._apply(m, True) == 0 else None

    def make_op_message(self, op: Msg, seq: int, ref_seq: Optional[int] = None,
                        long_client: Optional[int] = None, min_seq: int = 0) -> Msg:
        """TestClient.makeOpMessage (testClient.ts:213-234)."""
        if ref_seq is None:
            ref_seq = self.current_seq
        if long_client is None:
            long_client = self.long_client_id
        return op.sequenced(seq, ref_seq, long_client, min_seq)

    # --- reads ---------------------------------------------------------------------------
    @property
    def error(self) -> int:
        return self.L.mto_error(self.h)

    @property
    def current_seq(self) -> int:
        return self.L.mto_current_seq(self.h)

    @property
    def min_seq(self) -> int:
        return self.L.mto_min_seq(self.h)

    def get_length(self) -> int:
        return self.L.mto_local_length(self.h)

    def get_length_at(self, ref_seq: int, long_client: int) -> int:
        return self.L.mto_get_length(self.h, ref_seq, self.short_id(long_client))

    def short_id(self, long_client: int) -> int:
        return self.L.mto_short_id(self.h, long_client)

    def get_text(self) -> str:
        return self._text(0, -100)

    def get_text_at(self, ref_seq: int, long_client: int) -> str:
        return self._text(ref_seq, self.short_id(long_client))

    def _text(self, ref_seq: int, short: int) -> str:
        n = self.L.mto_get_text(self.h, ref_seq, short, None, 0)
        buf = np.zeros(max(n, 1), "<u2")
        self.L.mto_get_text(self.h, ref_seq, short, _p(buf), n)
        return buf[:n].tobytes().decode("utf-16-le")

    def containing(self, pos: int, ref_seq: int = 0, long_client: Optional[int] = None):
        """(found, offset, length, seq, long client, position): getContainingSegment(pos) and
        getPosition of that segment (mergeTree.ts:1656-1667, 1619-1636); None client = local view."""
        out = np.zeros(6, np.int32)
        short = -100 if long_client is None else self.short_id(long_client)
        if long_client is not None and short < 0:
            short = 0x7fff
        self.L.mto_get_containing(self.h, pos, ref_seq, short, _p(out))
        return tuple(int(x) for x in out)

    def pending_groups(self) -> int:
        return self.L.mto_pending_groups(self.h)

    def dump(self) -> bytes:
        n = self.L.mto_dump(self.h, None, 0)
        buf = np.zeros(n, np.uint8)
        self.L.mto_dump(self.h, _p(buf), n)
        return buf.tobytes()

    def digest(self) -> int:
        return int(self.L.mto_digest(self.h))

    def stats(self):
        v = [ctypes.c_int() for _ in range(4)]
        self.L.mto_stats(self.h, *[ctypes.byref(x) for x in v])
        return dict(nsegs=v[0].value, nleaf=v[1].value, height=v[2].value, nlive=v[3].value)

    def check_partials(self, ref_seq: int, short: int) -> int:
        return self.L.mto_check_partials(self.h, ref_seq, short)


def replay_batch(batch: ol.Batch, threads: int = 1):
    """Replay every document of a batch on the oracle; returns (seconds, digests, errors)."""
    L = lib()
    dig = np.zeros(batch.ndocs, np.uint64)
    err = np.zeros(batch.ndocs, np.int32)
    ops = batch.ops if len(batch.ops) else np.zeros(1, ol.OP_DTYPE)
    secs = L.mto_replay_batch(batch.ndocs, _p(ops), _p(batch.op_off), _p(batch.text), _p(batch.text_off),
                              _p(batch.props), _p(batch.props_off), _p(batch.kv), _p(batch.kv_off),
                              _p(batch.local_long_id), threads, _p(dig), _p(err))
    return secs, dig, err
