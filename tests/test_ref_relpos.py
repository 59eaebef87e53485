"""Relative positions (IRelativePosition, ops.ts:56-61; mt_oplog.h MT_SEG_RELPOS) against the REFERENCE
(tests/golden/refrelpos.npz, tools/make_ref_goldens.py --relpos).

tests/relpos_logs.py draws logs in which remote clients insert text and markers with unique "markerId"
properties, and a third of the inserts / removes / annotates name their positions relative to a live marker:
before / after it with offsets, SharedString.annotateMarker's {id, before: true} .. {id} range, removes that
start or end at a marker. The reference resolves them in Client.getValidOpRange with
MergeTree.posFromRelativePos under each op's refSeq and client (client.ts:486-503, mergeTree.ts:1976-1999).
Its digests of the replicas and its posFromRelativePos answers in the local view after the replay (live ids
before / after, with and without offset; an id no marker holds: -1) must be reproduced by the host build of
the engine core and by the HIP engine (client-feature build: caps.dcap > 0)."""
import os

import numpy as np
import pytest

import core_host
import relpos_logs
from make_goldens_sha import log_sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAPS = (192, 256, 1 << 16, 4096, 1024, 64)


def load():
    z = np.load(os.path.join(GOLDEN, "refrelpos.npz"), allow_pickle=False)
    b, interner, _ = relpos_logs.build(int(z["ndocs"]), int(z["nmsg"]), int(z["seed"]))
    assert log_sha(b) == str(z["log_sha256"]), "the logs differ from the fixture's"
    assert int(((b.ops["seg_kind"] & relpos_logs.SEG_RELPOS) != 0).sum()) == int(z["nrel"])
    return z, b, interner


def queries(z, interner):
    kid = interner.key(relpos_logs.MARKER_KEY)
    for d, mid, before, off in zip(z["q_doc"], z["q_id"], z["q_before"], z["q_offset"]):
        vid = interner.value(str(mid))
        yield int(d), kid, vid, bool(before), None if off < 0 else int(off)


def test_host_core_relative_positions_match_reference():
    z, b, interner = load()
    dig, err, st = core_host.replay_batch(b, CAPS, dcap=4096)
    assert (err == 0).all()
    assert np.array_equal(dig, z["digests"])
    got = [st.pos_from_relative_pos(d, k, v, bf, o) for d, k, v, bf, o in queries(z, interner)]
    assert got == z["answers"].tolist()
    assert (z["answers"] == -1).sum() >= b.ndocs  # the id no marker holds


def test_relative_positions_need_the_client_feature_build():
    """the hot build (no delta log, no references) latches MT_E_UNSUPPORTED at the first relative op; so does a
    marker id two markers hold"""
    from fluidframework_amd import oplog as ol
    it = ol.Interner()
    L = ol.DocLog(it, local_long_id=0)
    base = dict(client=1, ref_seq=0, min_seq=0)
    L.add(ol.OP_INSERT, seq=1, pos1=0, text="abc", **base)
    L.add(ol.OP_INSERT, seq=2, pos1=1, marker=0, props={"markerId": "m"}, **base)
    L.add(ol.OP_INSERT, seq=3, pos1=0, marker=0, props={"markerId": "m"}, **base)
    relpos_logs.add_rel(L, ol.OP_INSERT, ("m", False, None), None, seq=4, pos1=0, text="x", **base)
    b = ol.Batch.from_logs([L])
    _, err, st = core_host.replay_batch(b, CAPS, dcap=64)
    assert err[0] == 4 and st.error_op(0) == 3


@pytest.mark.gpu
def test_gpu_relative_positions_match_reference():
    from fluidframework_amd.engine import Engine
    z, b, interner = load()
    eng = Engine(b.ndocs, ncap=192, hcap=256, acap=1 << 16, mcap=4096, gcap=1024, ccap=64, dcap=4096)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert np.array_equal(eng.digests(), z["digests"])
    got = [eng.pos_from_relative_pos(d, k, v, bf, o) for d, k, v, bf, o in queries(z, interner)]
    assert got == z["answers"].tolist()


def _annotated_id_log():
    """a marker inserted with markerId "a" whose markerId a later annotate sets to "b"; then a relative
    insert after "b". The reference's idToSegment still maps "a" (written at insert, mergeTree.ts:1218-1221)
    and has no "b", so it would place the insert at -1; the engine refuses the lookup."""
    from fluidframework_amd import oplog as ol
    it = ol.Interner()
    L = ol.DocLog(it, local_long_id=0)
    base = dict(client=1, ref_seq=0, min_seq=0)
    L.add(ol.OP_INSERT, seq=1, pos1=0, text="abc", **base)
    L.add(ol.OP_INSERT, seq=2, pos1=1, marker=0, props={"markerId": "a"}, **base)
    L.add(ol.OP_ANNOTATE, seq=3, pos1=1, pos2=2, props={"markerId": "b"}, **base)
    L.add(ol.OP_INSERT, seq=4, pos1=0, text="y", **base)
    n = len(L.ops)
    relpos_logs.add_rel(L, ol.OP_INSERT, ("b", False, None), None, seq=5, pos1=0, text="x", **base)
    return it, L, n


def test_annotated_marker_id_is_refused_host():
    it, L, n = _annotated_id_log()
    from fluidframework_amd import oplog as ol
    b = ol.Batch.from_logs([L])
    _, err, st = core_host.replay_batch(b, CAPS, dcap=64)
    assert err[0] == 4 and st.error_op(0) == n
    b0 = ol.Batch.from_arrays([tuple(a[:n] if i == 0 else a for i, a in enumerate(L.arrays()))], [0])
    _, err, st = core_host.replay_batch(b0, CAPS, dcap=64)
    assert err[0] == 0
    kid = it.key(relpos_logs.MARKER_KEY)
    with pytest.raises(RuntimeError):
        st.pos_from_relative_pos(0, kid, it.value("b"))


@pytest.mark.gpu
def test_annotated_marker_id_is_refused_gpu():
    from fluidframework_amd import oplog as ol
    from fluidframework_amd.engine import Engine, EngineError
    it, L, n = _annotated_id_log()
    eng = Engine(1, ncap=192, hcap=256, acap=1 << 16, mcap=4096, gcap=1024, ccap=64, dcap=64)
    eng.start_collab([0])
    eng.replay(ol.Batch.from_logs([L]))
    err, err_op = eng.errors()
    assert err[0] == 4 and err_op[0] == n
    eng.close()
    eng = Engine(1, ncap=192, hcap=256, acap=1 << 16, mcap=4096, gcap=1024, ccap=64)  # hot build: query path
    eng.start_collab([0])
    eng.replay(ol.Batch.from_arrays([tuple(a[:n] if i == 0 else a for i, a in enumerate(L.arrays()))], [0]))
    assert (eng.errors()[0] == 0).all()
    with pytest.raises(EngineError):
        eng.pos_from_relative_pos(0, it.key(relpos_logs.MARKER_KEY), it.value("b"))
    eng.close()
