"""Synthetic workloads for BASELINE.json's configs (native generator ``csrc/mt_gen.c``)."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import native
from . import oplog as ol

MTG_FARM, MTG_OBSERVER, MTG_LAGGED, MTG_MATRIX = 1, 2, 3, 5
ALNUM = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789"
N_PROPS = 20 + 4096 + 32 + 20 + 8  # mtg_props_table records
N_KV = N_PROPS + 16  # their key/value entries (the last 8 records hold two each, after the others)


class _Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "mode", "ops_per_doc", "nclients", "max_lag", "local_pct", "ack_lag", "pct_insert",
        "pct_remove", "max_ins_len", "max_rem_len", "distinct_props", "newline_pct", "model_ncap",
        "model_acap", "perm", "round_ops", "min_length", "group_pct", "rewrite_pct", "_pad0")] + [
        ("seed_base", ctypes.c_uint64)]


@dataclass
class Workload:
    mode: int
    ops_per_doc: int
    nclients: int = 8
    max_lag: int = 0
    local_pct: int = 0
    ack_lag: int = 64
    pct_insert: int = 60
    pct_remove: int = 30
    max_ins_len: int = 8
    max_rem_len: int = 16
    distinct_props: int = 0
    newline_pct: int = 0
    model_ncap: int = 0
    model_acap: int = 0
    perm: int = 0
    round_ops: int = 0
    min_length: int = 0
    group_pct: int = 0
    rewrite_pct: int = 0
    _pad0: int = 0
    seed_base: int = 0x5EED0000


# BASELINE.json configs (BASELINE.md "CPU-baseline plan" table)
def config1(ops: int = 10_000, nclients: int = 8) -> Workload:
    """The reference's TestClient conflict farm: 1 document, `nclients` replicas (client 0
    observes), `ops` ops in rounds of 100, minLength 64, ops [remove, annotate, insert]
    (mergeTreeOperationRunner.ts:58-178, client.conflictFarm.spec.ts:25-48). One farm is
    `nclients` documents of the batch: doc c = replica c's event stream."""
    return Workload(MTG_FARM, ops, nclients=nclients, round_ops=100, min_length=64)


def config2(ops_per_doc: int = 10_000) -> Workload:
    """4,096 docs x 10k ops, observer replica, refSeq = MSN = seq - 1, 60/30/10."""
    return Workload(MTG_OBSERVER, ops_per_doc)


def config3(ops_per_doc: int = 4_096) -> Workload:
    """65,536 docs, 8 clients, lag <= 64, local-pending replica (~1/8 local edits); 4% of the edits
    (local and remote) are SharedString.replaceRange groups (insert + remove in one message); a
    quarter of the annotates (local and remote) carry combiningOp "rewrite"."""
    return Workload(MTG_LAGGED, ops_per_doc, max_lag=64, local_pct=12, ack_lag=64, group_pct=4, rewrite_pct=25)


def config4(ops_per_doc: int = 1_000_000) -> Workload:
    """256 large docs, lag 64, 70/25/5, coalescing defeated by distinct props + newlines."""
    return Workload(MTG_LAGGED, ops_per_doc, max_lag=64, local_pct=0, pct_insert=70, pct_remove=25,
                    distinct_props=1, newline_pct=25, model_ncap=32000, model_acap=1 << 22)


def config5(ops_per_doc: int = 4_096) -> Workload:
    """SharedMatrix PermutationVector replay: docs 2m / 2m+1 = rows / cols vectors of matrix m,
    one sequenced stream per matrix, PermutationSegment inserts of U{1..8} rows, removes of
    U{1..4}, 50% annotate (a quarter of them "rewrite"); 8 clients, lag <= 64, local-pending replica."""
    return Workload(MTG_MATRIX, ops_per_doc, max_lag=64, local_pct=12, ack_lag=64, pct_insert=32,
                    pct_remove=18, max_ins_len=8, max_rem_len=4, perm=1, rewrite_pct=25)


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        L = ctypes.CDLL(native.build_gen())
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.mtg_generate.argtypes = [ctypes.POINTER(_Params), i64, i64, i64, i64, vp, vp, vp, vp, ctypes.c_int]
        L.mtg_generate_ids.argtypes = [ctypes.POINTER(_Params), vp, i64, i64, i64, vp, vp, vp, vp, ctypes.c_int]
        L.mtg_props_table.argtypes = [vp, vp]
        _LIB = L
    return _LIB


def generator_interner() -> ol.Interner:
    """The key/value ids mtg_props_table uses: keys b,i,u,c,s,client = 1..6; value id v+1 =
    JSON v for v < 4096; value id 4097+k = the farm client name ALNUM[k]."""
    it = ol.Interner()
    for k in ("b", "i", "u", "c", "s", "client"):
        it.key(k)
    for v in range(4096):
        it.value(v)
    for k in range(32):
        it.value(ALNUM[k])
    return it


def props_table():
    props = np.zeros(N_PROPS, ol.PROPS_DTYPE)
    kv = np.zeros(N_KV, ol.KV_DTYPE)
    n = _lib().mtg_props_table(props.ctypes.data, kv.ctypes.data)
    assert n == len(props)
    return props, kv


def generate(w: Workload, ndocs: int = 0, doc_base: int = 0, threads: int = 0, ids=None) -> ol.Batch:
    """Generate document logs as one Batch: docs doc_base .. doc_base+ndocs-1, or the document ids
    `ids` (in that order) when given. A document's log depends only on its id."""
    if threads <= 0:
        threads = min(16, os.cpu_count() or 1)
    if ids is not None:
        ids = np.ascontiguousarray(np.asarray(ids, np.int64))
        ndocs = len(ids)
    p = _Params(**{k: int(getattr(w, k)) for k, _ in _Params._fields_})
    if w.mode == MTG_FARM:
        op_stride = 2 * w.ops_per_doc + 16
    else:
        op_stride = int(w.ops_per_doc * (1 + w.local_pct / 50.0)) + 16
    text_stride = op_stride * w.max_ins_len
    ops = np.zeros(ndocs * op_stride, ol.OP_DTYPE)
    text = np.zeros(ndocs * text_stride, "<u2")
    nops = np.zeros(ndocs, np.int64)
    ntext = np.zeros(ndocs, np.int64)
    if ids is None:
        rc = _lib().mtg_generate(ctypes.byref(p), doc_base, ndocs, op_stride, text_stride, ops.ctypes.data,
                                 nops.ctypes.data, text.ctypes.data, ntext.ctypes.data, threads)
    else:
        rc = _lib().mtg_generate_ids(ctypes.byref(p), ids.ctypes.data, ndocs, op_stride, text_stride,
                                     ops.ctypes.data, nops.ctypes.data, text.ctypes.data, ntext.ctypes.data, threads)
    if rc == -1:
        raise RuntimeError("generator buffer overflow")
    if rc == -2:
        raise RuntimeError("generator model replica reported an error (capacity)")
    # compact the fixed-stride buffers
    op_off = np.zeros(ndocs + 1, np.int64)
    op_off[1:] = np.cumsum(nops)
    text_off = np.zeros(ndocs + 1, np.int64)
    text_off[1:] = np.cumsum(ntext)
    # compact the per-doc fixed-stride buffers (slices: no index matrices, ~2x output memory)
    ops_c = np.empty(int(op_off[-1]), ol.OP_DTYPE)
    text_c = np.empty(int(text_off[-1]), "<u2")
    for d in range(ndocs):
        ops_c[op_off[d]: op_off[d + 1]] = ops[d * op_stride: d * op_stride + nops[d]]
        text_c[text_off[d]: text_off[d + 1]] = text[d * text_stride: d * text_stride + ntext[d]]
    del ops, text
    if len(text_c) == 0:
        text_c = np.zeros(1, "<u2")
    props, kv = props_table()
    zeros = np.zeros(ndocs + 1, np.int64)
    doc_ids = ids if ids is not None else np.arange(doc_base, doc_base + ndocs, dtype=np.int64)
    if w.mode == MTG_FARM:
        local = (doc_ids % w.nclients).astype(np.int32)
    else:
        local = np.full(ndocs, 0 if w.mode == MTG_OBSERVER else 1, np.int32)
    return ol.Batch(ops_c, op_off, text_c, text_off, props, zeros, kv, zeros.copy(), local)
