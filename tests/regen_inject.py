"""Reconnects (mt_oplog.h MT_OPF_REGEN) injected into config-3 logs — test infrastructure for the §8(f) f4
reconnect fixtures (tools/make_ref_goldens.py --regen, tests/test_ref_regen.py).

At a seeded point of each document's stream where its replica has ops in flight, the runtime reconnects:
one REGEN record per pending segment group, in queue order (what SharedSegmentSequence.reSubmitCore does
for every unacked message, client.ts:855-893). Each resubmitted message is then sequenced where the
original was: its ack becomes one member record per regenerated op (a NOOP from the replica when none
is left), with the original's seq / ref_seq / min_seq and props. The other records are unchanged: the
replica's tree does not depend on where a resubmitted op says it goes, only on its segment groups. The
number of regenerated ops per group comes from the host build of the engine core (its MT_DELTA_REGEN
events)."""
from __future__ import annotations

import dataclasses

import numpy as np

from fluidframework_amd import oplog as ol
import core_host

OPF_REGEN = 0x10


def _acks(ops, local):
    """Indices of the replica's own sequenced op records (acks), in order, and per record the number of
    segment groups it acks (its message's members)."""
    kind = ops["kind"]
    own = ((kind & ol.OPF_LOCAL) == 0) & (ops["client"] == local) & ((kind & 7) != ol.OP_NOOP)
    return np.nonzero(own)[0]


def inject(b: ol.Batch, caps, seed: int = 9090) -> ol.Batch:
    out, off = [], [0]
    for d in range(b.ndocs):
        ops, text, props, kv = b.doc(d)
        local = int(b.local_long_id[d])
        st = core_host.HostStore(1, caps, dcap=1 << 22)
        st.start_collab(0, local)
        ack_idx = _acks(ops, local)
        grouped = (ops["kind"] & ol.OPF_GROUPED) != 0
        rng = np.random.default_rng(seed + d)
        # candidate cuts: not inside a group message, with >= 1 ack still ahead
        cand = [i for i in range(1, len(ops)) if not grouped[i - 1] and len(ack_idx) and ack_idx[-1] >= i]
        if not cand:
            out.append(ops)
            off.append(off[-1] + len(ops))
            continue
        cut = int(rng.choice(cand))
        assert st.replay(0, ops[:cut], text, props, kv) == 0
        m = st.pending(0)
        later = [int(a) for a in ack_idx if a >= cut]
        if m == 0 or len(later) < m or grouped[later[m - 1]]:  # whole messages only
            out.append(ops)
            off.append(off[-1] + len(ops))
            continue
        targets = later[:m]  # the ack member records of the m pending groups, in queue order
        regen = np.zeros(m, ol.OP_DTYPE)
        for j, a in enumerate(targets):
            regen[j]["kind"] = (ops[a]["kind"] & 7) | ol.OPF_LOCAL | OPF_REGEN
            regen[j]["props"] = ops[a]["props"]
        n0 = st.deltas(0)[0]
        assert st.replay(0, regen, text, props, kv) == 0
        words = st.deltas(0)[2][n0:]
        k, i = [], 0  # regenerated ops per group, from the MT_DELTA_REGEN events
        while i < len(words):
            assert words[i] == 3
            j = i + 2
            while words[j] != -(1 << 31):
                j += 3
            k.append(int(words[j + 1]))
            i = j + 2
        assert len(k) == m
        # rebuild: [0, cut) + REGEN + the rest, each acking message rewritten member by member
        recs = list(ops[:cut]) + list(regen)
        g = 0
        i = cut
        while i < len(ops):
            if g < m and i == targets[g]:
                # one message: the records from here through its last member (no GROUPED flag)
                e = i
                while ops[e]["kind"] & ol.OPF_GROUPED:
                    e += 1
                members = list(range(i, e + 1))
                new = []
                for a in members:
                    r = ops[a].copy()
                    r["kind"] = r["kind"] & 7
                    new += [r] * k[g]
                    g += 1
                if not new:
                    r = ops[e].copy()
                    r["kind"] = ol.OP_NOOP
                    r["props"] = 0
                    new = [r]
                for q, r in enumerate(new):
                    r = r.copy()
                    if q < len(new) - 1:
                        r["kind"] |= ol.OPF_GROUPED
                    recs.append(r)
                i = e + 1
                continue
            recs.append(ops[i])
            i += 1
        merged = np.array(recs, ol.OP_DTYPE)
        out.append(merged)
        off.append(off[-1] + len(merged))
    return dataclasses.replace(b, ops=np.concatenate(out), op_off=np.asarray(off, np.int64))
