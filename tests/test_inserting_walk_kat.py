"""mergeTree.insertingWalk.spec.ts:26-253 as known-answer tests, on the oracle, the host core and the GPU.

The spec's three trees — "single segment tree" (26-52), "Full single layer tree" (53-108: "0".."6", seven
children of one block) and "Tree with remove segments" (109-172: "0".."31" with a quarter of the text removed
from each end before collaboration) — are built with MergeTree-level records (mt_oplog.h MT_OPF_TREE: the
spec's insertSegments / insertText / markRangeRemoved calls with their explicit refSeq, clientId and seq),
then startCollaboration(localClientId, 0, 0) (an MT_OP_COLLAB record), then one insertText of "a" at the
beginning, the end and the middle (187-253) by the local client at refSeq 0 with UnassignedSequenceNumber.
The expected text and length are the spec's own (`a${initialText}`, `${initialText}a`, and "a" at
`middle`); the spec's local client id 17 is a long client id here (its short id is not observable)."""
import math

import pytest

import core_host
import oracle_client as oc
from fluidframework_amd import oplog as ol

LOCAL_CLIENT = 0xFFFE  # mt_oplog.h MT_CLIENT_LOCAL: LocalClientId (constants.ts:14)
CLIENT = 17            # the spec's localClientId (line 24), as a long client id
UNIVERSAL, UNASSIGNED = 0, -1
MAX_NODES = 8          # MaxNodesInBlock (mergeTreeNodes.ts)
TREE = ol.OPF_TREE


def js_round(x: float) -> int:
    return math.floor(x + 0.5)  # Math.round


def build(shape: str):
    """(log, initialText, middle): the spec's tree factory (26-173) as records, collaboration started"""
    L = ol.DocLog(ol.Interner(), local_long_id=CLIENT)
    if shape == "single segment tree":
        text = "hello world"
        L.add(ol.OP_INSERT | TREE, client=LOCAL_CLIENT, seq=UNIVERSAL, ref_seq=UNIVERSAL, pos1=0, text=text)
        middle = js_round(len(text) / 2)
    else:
        text = "0"
        L.add(ol.OP_INSERT | TREE, client=LOCAL_CLIENT, seq=UNIVERSAL, ref_seq=UNIVERSAL, pos1=0, text=text)
        n = MAX_NODES - 1 if shape == "Full single layer tree" else MAX_NODES * 4
        for i in range(1, n):  # insertText at getLength(UniversalSequenceNumber, localClientId)
            L.add(ol.OP_INSERT | TREE, client=CLIENT, seq=UNIVERSAL, ref_seq=UNIVERSAL, pos1=len(text), text=str(i))
            text += str(i)
        if shape == "Full single layer tree":
            middle = js_round(MAX_NODES / 2)
        else:
            remove = js_round(len(text) / 4)
            L.add(ol.OP_REMOVE | TREE, client=CLIENT, seq=UNASSIGNED, ref_seq=UNIVERSAL, pos1=0, pos2=remove)
            text = text[remove:]
            L.add(ol.OP_REMOVE | TREE, client=CLIENT, seq=UNASSIGNED, ref_seq=UNIVERSAL, pos1=len(text) - remove,
                  pos2=len(text))
            text = text[:len(text) - remove]
            middle = js_round(len(text) / 2)
    L.add(ol.OP_COLLAB, client=CLIENT, seq=UNIVERSAL, min_seq=UNIVERSAL)
    return L, text, middle


SHAPES = ("single segment tree", "Full single layer tree", "Tree with remove segments")
CASES = ("at beginning", "at end", "in middle")


def cases():
    """every (shape, case): (log, expected text) — the spec's asserts (199-206, 220-227, 241-252)"""
    out = []
    for shape in SHAPES:
        for case in CASES:
            L, text, middle = build(shape)
            pos = {"at beginning": 0, "at end": len(text), "in middle": middle}[case]
            L.add(ol.OP_INSERT | TREE, client=CLIENT, seq=UNASSIGNED, ref_seq=UNIVERSAL, pos1=pos, text="a")
            out.append(((shape, case), L, text[:pos] + "a" + text[pos:]))
    return out


def test_spec_shapes():
    """the factories' own asserts: "Full single layer tree" is 7 children of one block (79-92)"""
    _, text, middle = build("Full single layer tree")
    assert text == "0123456" and middle == 4
    _, text, middle = build("Tree with remove segments")
    full = "".join(str(i) for i in range(MAX_NODES * 4))
    assert len(full) == 54 and text == full[14:40] and middle == 13


def test_oracle_inserting_walk():
    for name, L, want in cases():
        o = oc.OracleClient(L.interner)
        assert o.replay(L) == 0, name
        assert (o.get_text(), o.get_length()) == (want, len(want)), name
        assert o.get_length_at(UNIVERSAL, CLIENT) == len(want), name  # getLength(refSeq, localClientId)
        assert o.get_text_at(UNIVERSAL, CLIENT) == want, name


def test_host_core_inserting_walk():
    cs = cases()
    b = ol.Batch.from_logs([L for _, L, _ in cs])
    hs = core_host.HostStore(b.ndocs)  # no start_collab: the COLLAB record starts it
    for d in range(b.ndocs):
        assert hs.replay(d, *b.doc(d)) == 0, cs[d][0]
    for d, (name, L, want) in enumerate(cs):
        assert hs.text(d) == want, name
        assert hs.L.mth_length_local(hs.h, d) == len(want), name
        o = oc.OracleClient(L.interner)
        o.replay(L)
        assert hs.dump(d) == o.dump(), name  # the whole canonical dump: segments, seqs, clients, leaf ordinals


@pytest.mark.gpu
def test_gpu_inserting_walk():
    from fluidframework_amd.engine import Engine
    cs = cases()
    b = ol.Batch.from_logs([L for _, L, _ in cs])
    eng = Engine(b.ndocs, ncap=2048, hcap=4096, acap=1 << 17, mcap=4096, gcap=1024, ccap=64)
    eng.replay(b)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err, err_op)
    dig = eng.digests()
    for d, (name, L, want) in enumerate(cs):
        assert (eng.get_text(d), eng.get_length(d)) == (want, len(want)), name
        o = oc.OracleClient(L.interner)
        o.replay(L)
        assert int(dig[d]) == o.digest(), name
    eng.close()
