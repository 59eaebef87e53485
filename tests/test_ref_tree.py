"""MergeTree-level calls with explicit (refSeq, clientId, seq) — MergeTree.insertSegments / markRangeRemoved
/ annotateRange (mergeTree.ts:2001-2031, 2598-2738), mt_oplog.h MT_OPF_TREE — against the REFERENCE
(tests/golden/reftree_*.npz, tools/make_ref_goldens.py --tree).

The fixture logs are config-3 and config-5 logs in which every third plain remote op message became the
MergeTree-level call plus a NOOP message of the same seq, and every fourth plain local edit became the
MergeTree-level call with the replica's client id, UnassignedSequenceNumber and its currentSeq
(tests/tree_ops.py). The reference replayed them; its digests equal its own digests of the unconverted logs
(checked when the fixture was made). The host build of the engine core and the HIP engine must reproduce
them on every document."""
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
import tree_ops
from make_goldens_sha import log_sha
from test_ref_goldens import caps_for

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ("c3_lagged", "c5_perm")


def load(name):
    z = np.load(os.path.join(GOLDEN, f"reftree_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    b = tree_ops.to_tree_ops(gen.generate(w, ids=z["doc_ids"], threads=8))
    assert log_sha(b) == str(z["log_sha256"]), "the converted logs differ from the fixture's"
    assert int(((b.ops["kind"] & tree_ops.OPF_TREE) != 0).sum()) == int(z["ntree"])
    return z, w, b


@pytest.mark.parametrize("name", NAMES)
def test_host_core_tree_records_match_reference(name):
    z, w, b = load(name)
    c = caps_for(w)
    dig, err, _ = core_host.replay_batch(b, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]))
    assert (err == 0).all()
    assert np.array_equal(dig, z["digests"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_tree_records_match_reference(name):
    """the oracle restates the MergeTree-level calls too (mt_oracle.c applyEdit): pinned by the same fixtures"""
    import oracle_client as oc
    z, _, b = load(name)
    _, dig, err = oc.replay_batch(b, threads=8)
    assert (err == 0).all()
    assert np.array_equal(dig, z["digests"])


def test_tree_record_flag_rules():
    """a TREE record that is also LOCAL, or an empty text insert, latches MT_E_UNSUPPORTED"""
    from fluidframework_amd import oplog as ol
    L = ol.DocLog(ol.Interner(), local_long_id=0)
    L.add(ol.OP_INSERT | tree_ops.OPF_TREE, client=1, seq=1, ref_seq=0, min_seq=0, pos1=0, text="ab")
    L.add(ol.OP_NOOP, client=1, seq=1, ref_seq=0, min_seq=0)
    L.add(ol.OP_INSERT | tree_ops.OPF_TREE | ol.OPF_LOCAL, client=0, seq=-1, ref_seq=1, pos1=0, text="x")
    b = ol.Batch.from_logs([L])
    dig, err, st = core_host.replay_batch(b)
    assert err[0] == 4 and st.error_op(0) == 2
    import oracle_client as oc
    o = oc.OracleClient(L.interner)
    assert o.replay(L) == 4  # MTO_ERR_UNSUPPORTED at the same record


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])  # both config-2/3 kernel builds (mt_engine_set_variant)
@pytest.mark.parametrize("name", NAMES)
def test_gpu_tree_records_match_reference(name, waves):
    from fluidframework_amd.engine import Engine
    z, w, b = load(name)
    eng = Engine(b.ndocs, waves=waves, **caps_for(w))
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert np.array_equal(eng.digests(), z["digests"])
