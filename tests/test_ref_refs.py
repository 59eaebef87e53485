"""Local references against the REFERENCE merge-tree (tests/golden/refrefs_*.npz).

Each fixture document's log gets 24 MT_OP_REF records (tests/refs_inject.py: seeded points, positions
drawn from the replica's local length, 60 % SlideOnRemove). The reference (tools/ref_replay.mjs, via
tools/make_ref_goldens.py --refs) creates `new LocalReference(client, segment, offset, refType)` +
Client.addLocalReference for Client.getContainingSegment(pos) at each record and reports
LocalReference.toPosition() of every reference after the whole stream: references ride their segment
through splits (LocalReferenceCollection.split) and zamboni appends (.append), a remove slides
SlideOnRemove references to the next segment (or the end) and detaches the others, and zamboni unlinks
detach (toPosition -1). -2 marks a reference the reference itself could not add (its addLocalRef pushes
onto the missing `at` list of an offset holding only slid references, localReference.ts:195-201); the
engine reproduces that case too (REF_GHOST), so every reference is compared. The fixture also holds the
reference's digests of the same replicas: references change nothing else. After the whole stream every
document also gets up to 4 insertAtReferencePositionLocal records (MT_OPF_ATREF, on references the
reference left attached; mergeTree.ts:2033-2130: split at the reference's offset, left excursion over
zero-length segments, insert before), so the digests pin where those inserts land.
"""
import glob
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
import refs_inject
from test_ref_goldens import caps_for
from make_goldens_sha import log_sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = [os.path.basename(f)[8:-4] for f in sorted(glob.glob(os.path.join(GOLDEN, "refrefs_*.npz")))]
RCAP = 32


def load(name):
    z = np.load(os.path.join(GOLDEN, f"refrefs_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    b = gen.generate(w, ids=z["doc_ids"], threads=8)
    c = caps_for(w)
    rb = refs_inject.inject(b, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]))
    rb = refs_inject.add_atref_inserts(rb, [t[t >= 0] for t in z["atref_targets"]])
    assert log_sha(rb) == str(z["log_sha256"]), "the injected logs differ from the fixture's"
    return z, w, rb, c


def compare(z, nref, pos):
    assert np.array_equal(nref, z["nref"])
    want = z["positions"]
    bad = []
    for d in range(len(nref)):
        n = int(nref[d])
        if not np.array_equal(pos[d, :n], want[d, :n]):
            bad.append(d)
    return bad


def test_ref_fixture_set_complete():
    assert set(NAMES) >= {"c1_farm", "c2_observer", "c3_lagged", "c4_scaled", "c5_perm"}


@pytest.mark.parametrize("name", NAMES)
def test_host_core_local_references_match_reference(name):
    z, w, rb, c = load(name)
    dig, err, st = core_host.replay_batch(rb, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]),
                                          rcap=RCAP)
    assert (err == 0).all()
    assert np.array_equal(dig, z["digests"])
    nref = np.zeros(rb.ndocs, np.int32)
    pos = np.full((rb.ndocs, RCAP), -1, np.int32)
    for d in range(rb.ndocs):
        p = st.ref_positions(d)
        nref[d] = len(p)
        pos[d, : len(p)] = p
    bad = compare(z, nref, pos)
    assert not bad, f"reference positions differ from the reference on docs {bad[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_local_references_match_reference(name):
    from fluidframework_amd.engine import Engine
    z, w, rb, c = load(name)
    eng = Engine(rb.ndocs, rcap=RCAP, **c)
    eng.start_collab(rb.local_long_id)
    eng.replay(rb)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
    assert np.array_equal(eng.digests(), z["digests"])
    nref, pos = eng.ref_positions()
    bad = compare(z, nref, pos)
    assert not bad, f"HIP engine's reference positions differ from the reference on docs {bad[:8]}"
