"""PermutationVector.getAllocatedHandle records (mt_oplog.h MT_OP_NOOP | MT_OPF_LOCAL) injected into config-5
logs — test infrastructure for the §8(f) f3 handle fixtures (tools/make_ref_goldens.py --handles,
tests/test_ref_handles.py).

getAllocatedHandle is a local read-then-write (SharedMatrix.setCell allocates the row / column handle of the
cell it writes), so an injected record changes no sequenced state: it splits a one-row segment out where the
row has no handle yet and allocates it from the document's HandleTable; zamboni's unlinks free handles,
and handles then steer which PermutationSegments zamboni may append (canAppend compares starts). Each
document gets `nalloc` of them at seeded points of its stream (never inside a group message), each at a
position drawn from the replica's local length at that point (measured with the host build of the engine
core; a point with an empty vector gets none), a third of them at a position an earlier record allocated."""
from __future__ import annotations

import dataclasses

import numpy as np

from fluidframework_amd import oplog as ol
import core_host


def inject(b: ol.Batch, caps, nalloc: int = 40, seed: int = 5151) -> ol.Batch:
    st = core_host.HostStore(b.ndocs, caps, pcap=1 << 14)
    out, off = [], [0]
    for d in range(b.ndocs):
        ops, text, props, kv = b.doc(d)
        st.start_collab(d, int(b.local_long_id[d]))
        rng = np.random.default_rng(seed + d)
        grouped = (ops["kind"] & ol.OPF_GROUPED) != 0
        ok = np.ones(len(ops) + 1, bool)
        ok[1:] = ~grouped  # not right after a group member
        cand = np.nonzero(ok)[0]
        at = np.sort(rng.choice(cand, size=min(nalloc, len(cand)), replace=False))
        pieces, prev, used = [], 0, []
        for i in at:
            if i > prev:
                assert st.replay(d, ops[prev:i], text, props, kv) == 0
            pieces.append(ops[prev:i])
            prev = i
            L = st.L.mth_length_local(st.h, d)
            if L <= 0:
                continue
            pos = int(rng.integers(0, L))
            if used and rng.random() < 1 / 3:
                pos = min(used[int(rng.integers(0, len(used)))], L - 1)
            used.append(pos)
            r = np.zeros(1, ol.OP_DTYPE)
            r["kind"] = ol.OP_NOOP | ol.OPF_LOCAL
            r["pos1"] = pos
            assert st.replay(d, r, text, props, kv) == 0
            pieces.append(r)
        pieces.append(ops[prev:])
        merged = np.concatenate(pieces)
        out.append(merged)
        off.append(off[-1] + len(merged))
    return dataclasses.replace(b, ops=np.concatenate(out), op_off=np.asarray(off, np.int64))
