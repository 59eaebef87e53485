"""Annotates with combining ops "incr" / "consensus" (mt_oplog.h MT_COMBINE_INCR / CONSENSUS) injected into
generator logs — test infrastructure for the combining-op fixtures (tools/make_ref_goldens.py --combine,
tests/test_ref_combine.py).

A share of each document's annotate records (sequenced and local, never group members) get a property record
of their own that carries the combining op instead of a plain set. The reference applies them as its
addProperties does (segmentPropertiesManager.ts:92-106: every key modified, combine with newValue undefined,
properties.ts:26-59): "consensus" keeps a value a row already has and writes an object where it has none,
"incr" writes NaN. Most injected ops are consensus, so documents run long stretches of kept values before the
first object; a late incr (sequenced or local) in every other document ends those that get that far. Local
annotates get no consensus op: the reference's ack of one throws (client.ts:982-989) unless
annotateMarkerNotifyConsensus made it; the engine refuses them (MT_E_UNSUPPORTED at the local record)."""
from __future__ import annotations

import dataclasses

import numpy as np

from fluidframework_amd import oplog as ol


STRING0, NSTRING = 4097, 32  # the generator interner's string values (gen.generator_interner: ALNUM[k])


def inject(b: ol.Batch, frac: float = 0.08, seed: int = 3131, sfrac: float = 0.15) -> ol.Batch:
    """The generator's property records are one pool all documents share (props_off 0): the pool gets, after
    its own records, a consensus copy and an incr copy of each, and the picked records point at those. So that incr
    meets strings too (`"s" + undefined`, include/mt_oplog.h MT_VALUE_STRCAT0), a share `sfrac` of the plain remote
    annotates set string values instead (a third copy of each record, its values mapped onto the interner's strings),
    and documents with a late incr get a second one after it."""
    assert not b.props_off.any() and not b.kv_off.any(), "shared property pools"
    n = len(b.props)
    extra = np.repeat(b.props, 2)
    extra["combining"][0::2] = ol.COMBINE_CONSENSUS
    extra["combining"][1::2] = ol.COMBINE_INCR
    strs = b.props.copy()  # the string copies: their kv entries appended to the pool
    kv = b.kv.copy()
    skv = []
    for i, r in enumerate(b.props):
        o, m = int(r["kv_off"]), int(r["nkv"])
        strs[i]["kv_off"] = len(kv) + len(skv)
        for j in range(m):
            key, v = int(b.kv[o + j]["key"]), int(b.kv[o + j]["value"])
            skv.append((key, (STRING0 + (key + (v & 0x7FFF)) % NSTRING) if v else 0))
    kv = np.concatenate([kv, np.array(skv, ol.KV_DTYPE)])
    assert n + len(extra) + len(strs) < 0xFFFF
    props = np.concatenate([b.props, extra, strs])
    s0 = n + len(extra)  # 0-based index of the first string copy
    ops_all = b.ops.copy()
    for d in range(b.ndocs):
        o0, o1 = int(b.op_off[d]), int(b.op_off[d + 1])
        ops = ops_all[o0:o1]  # a view: edited in place
        rng = np.random.default_rng(seed + d)
        ann = np.nonzero(((ops["kind"] & 7) == ol.OP_ANNOTATE) & ((ops["kind"] & ol.OPF_GROUPED) == 0) &
                         (ops["props"] > 0))[0]
        # consensus on sequenced annotates only: the ack of a local one throws in the reference unless it was made
        # by annotateMarkerNotifyConsensus (client.ts:982-989 reads op.relativePos1.id), which the engine refuses
        remote = ann[((ops["kind"][ann] & ol.OPF_LOCAL) == 0) & (ops["client"][ann] != b.local_long_id[d])]  # not acks
        spick = remote[rng.random(len(remote)) < sfrac]
        pick = remote[rng.random(len(remote)) < frac]
        spick = np.setdiff1d(spick, pick)
        ops["props"][spick] = s0 + ops["props"][spick].astype(np.int64)  # the string copy (1-based)
        ops["props"][pick] = n + 2 * (ops["props"][pick].astype(np.int64) - 1) + 1  # the consensus copy (1-based)
        late = ann[ann > 0.7 * len(ops)]
        if d % 2 == 0 and len(late):
            for _ in range(2):
                i = int(late[int(rng.integers(0, len(late)))])
                p0 = int(ops["props"][i])
                if p0 > s0:  # a string copy: back to its original
                    p0 -= s0
                elif p0 > n:  # a consensus or incr copy: back to its original
                    p0 = (p0 - n - 1) // 2 + 1
                ops["props"][i] = n + 2 * (p0 - 1) + 2  # the incr copy
    return dataclasses.replace(b, ops=ops_all, props=props, kv=kv)
