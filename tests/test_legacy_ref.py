"""SharedString's default summary (SnapshotLegacy, snapshotlegacy.ts:104-242) pinned to the REFERENCE
(tests/golden/reflegacy_*.npz, tools/make_ref_goldens.py --legacy).

For every document of a fixture set the reference replayed records [0, cut) through a Client while
keeping SharedString's messagesSinceMSNChange (sequence.ts:579-616: messages whose refSeq is not
seq - 1 are stashed rebased, their contents createOpsFromDelta of the sequenceDelta events they fire),
summarized with SnapshotLegacy (the catch-up messages are those above the MSN), and a fresh client
loaded the tree and applied the catch-up messages. Stored: the tree's canonical SHA-256, the loaded
client's digest, and the documents where the summarizing SharedString throws (an annotate that pending
local rewrites blocked has no property deltas: createOpsFromDelta's Object.keys(undefined)) or where the
tree does not load (a rebased catch-up op the loaded client cannot place).

Here the same is done with the product path: the prefix replays on the engine with its delta stream on
(the host build of the core, or the HIP engine), snapshot.catchup_messages rebases from the stream,
snapshot.emit_legacy writes the tree, and the loaded replica (snapshot.load_records: header, body and
catch-up messages) replays on the same engine.
"""
import glob
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
from fluidframework_amd import snapshot as sn
import core_host
from test_ref_goldens import caps_for
from test_snapshot_ref import client_index, long_name, sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(os.path.basename(f)[10:-4] for f in glob.glob(os.path.join(GOLDEN, "reflegacy_*.npz")))
DCAP = 1 << 21  # delta-stream words per document: the whole prefix's events


def fixture(name):
    z = np.load(os.path.join(GOLDEN, f"reflegacy_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    b = gen.generate(w, ids=z["doc_ids"], threads=8)
    return z, w, b


def prefix(b, d, cut):
    ops, text, props, kv = b.doc_arrays(d)
    return ops[:cut], text, props, kv


def summarize(z, b, d, dump, words):
    """(tree, None) or (None, "emit") when the summarizing SharedString throws, as the reference's."""
    it = gen.generator_interner()
    hdr, segs = ol.parse_dump(dump)
    ops, text, props, kv = prefix(b, d, int(z["cut"][d]))
    try:
        msgs = sn.catchup_messages(ops, text, props, kv, words, it, long_name, hdr["minSeq"])
    except ValueError:
        assert z["emit_error"][d], f"doc {d}: rebasing the catch-up messages failed; the reference did not"
        return None
    assert not z["emit_error"][d], f"doc {d}: the reference's summarizing SharedString throws; not here"
    tree = sn.emit_legacy(hdr, segs, it, msgs)
    assert sha(tree) == str(z["sha256"][d]), f"doc {d}: legacy summary differs from the reference's"
    return tree


def load_log(tree, loader):
    log = ol.DocLog(gen.generator_interner())
    sn.load_records(tree, log, client_index, long_name(loader))
    return log.arrays()


def check_loaded(z, d, err, digest):
    if z["load_error"][d]:
        assert err == 1, f"doc {d}: the reference cannot load its legacy summary (insert failed); here err {err}"
    else:
        assert err == 0, f"doc {d}: loading the legacy summary failed: err {err}"
        assert digest == int(z["loaded_digests"][d]), f"doc {d}: loaded replica differs from the reference's"


def test_fixture_sets():
    assert set(NAMES) >= {"c1_farm", "c2_observer", "c3_lagged"}
    z, _, _ = fixture("c3_lagged")
    assert z["emit_error"].any() and z["load_error"].any() and not z["load_error"].all()


@pytest.mark.parametrize("name", NAMES)
def test_host_core_legacy_summary_matches_reference(name):
    z, w, b = fixture(name)
    c = caps_for(w)
    caps = (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"])
    st = core_host.HostStore(b.ndocs, caps, dcap=DCAP)
    ld = core_host.HostStore(b.ndocs, caps)
    loader = int(z["loader"])
    for d in range(b.ndocs):
        st.start_collab(d, int(b.local_long_id[d]))
        assert st.replay(d, *prefix(b, d, int(z["cut"][d]))) == 0
        n, _h, words = st.deltas(d)
        assert n == len(words), "delta log too small"
        tree = summarize(z, b, d, st.dump(d), words)
        if tree is None:
            continue
        err = ld.replay(d, *load_log(tree, loader))
        check_loaded(z, d, err, ld.digest(d) if err == 0 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_legacy_summary_matches_reference(name):
    from fluidframework_amd.engine import Engine
    z, w, b = fixture(name)
    caps = caps_for(w)
    pre = Engine(b.ndocs, **dict(caps, dcap=DCAP))
    pre.start_collab(b.local_long_id)
    pre.replay(ol.Batch.from_arrays([prefix(b, d, int(z["cut"][d])) for d in range(b.ndocs)], b.local_long_id))
    err, _ = pre.errors()
    assert (err == 0).all()
    nw, _ = pre.delta_state()
    loads, docs = [], []
    for d in range(b.ndocs):
        words = pre.deltas(d)
        assert nw[d] == len(words), "delta log too small"
        tree = summarize(z, b, d, pre.dump(d), words)
        if tree is not None:
            loads.append(load_log(tree, int(z["loader"])))
            docs.append(d)
    pre.close()
    if not loads:
        return
    eng = Engine(len(loads), **caps)  # each loaded replica starts detached
    eng.replay(ol.Batch.from_arrays(loads, np.full(len(loads), -1, np.int32)))
    err, _ = eng.errors()
    dig = eng.digests()
    for i, d in enumerate(docs):
        check_loaded(z, d, int(err[i]), int(dig[i]))
