"""refsByOffset entries after Client.removeLocalReference, against the REFERENCE (ADVICE r4, medium;
tests/golden/refentry_kat.npz from tools/make_ref_goldens.py --refentry over tests/refs_entry_logs.py).

removeLocalRef (localReference.ts:225-264) leaves the reference's entry in its collection with the same shape:
an add at an offset whose entry a slide made throws (195-201: no `at` list), a slide onto an entry an add made
keeps its `at` list, and the entry rides the collection's splits and appends only while the collection holds
other references. Five handcrafted documents (one per case) and 48 fuzzed ones (many references, removals and
slides on a few short segments, zamboni merging at minSeq lag 3). Compared: every LocalReference.toPosition()
(-2: the reference's addLocalReference threw) and the replicas' digests, host core and HIP engine."""
import os

import numpy as np
import pytest

import core_host
import refs_entry_logs as rel
from make_goldens_sha import log_sha
from test_ref_refs import compare

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAPS = (192, 256, 1 << 16, 1024, 1024, 254)


def load():
    z = np.load(os.path.join(GOLDEN, "refentry_kat.npz"), allow_pickle=False)
    rb = rel.batch()
    assert log_sha(rb) == str(z["log_sha256"]), "the KAT logs differ from the fixture's"
    return z, rb


def test_fixture_exercises_the_entry_cases():
    z, rb = load()
    pos = z["positions"]
    # handcrafted: (a) throws, (b) adds, (c) throws after the split moved the entry, (d) adds, (e) throws
    assert pos[0, 1] == -2 and pos[0, 2] >= 0
    assert pos[1, 2] == 0
    assert pos[2, 2] == -2 and pos[2, 3] >= 0
    assert pos[3, 1] >= 0
    assert pos[4, 3] == -2
    assert int((pos[5:] == -2).sum()) > 100


def test_host_core_entries_match_reference():
    z, rb = load()
    dig, err, st = core_host.replay_batch(rb, CAPS, rcap=rel.RCAP)
    assert (err == 0).all()
    assert np.array_equal(dig, z["digests"])
    nref = np.zeros(rb.ndocs, np.int32)
    pos = np.full((rb.ndocs, rel.RCAP), -1, np.int32)
    for d in range(rb.ndocs):
        p = st.ref_positions(d)
        nref[d] = len(p)
        pos[d, : len(p)] = p
    bad = compare(z, nref, pos)
    assert not bad, f"reference positions differ from the reference on docs {bad[:8]}"


@pytest.mark.gpu
def test_gpu_entries_match_reference():
    from fluidframework_amd.engine import Engine
    z, rb = load()
    eng = Engine(rb.ndocs, rcap=rel.RCAP, ncap=CAPS[0], hcap=CAPS[1], acap=CAPS[2], mcap=CAPS[3], gcap=CAPS[4],
                 ccap=CAPS[5])
    eng.start_collab(rb.local_long_id)
    eng.replay(rb)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
    assert np.array_equal(eng.digests(), z["digests"])
    nref, pos = eng.ref_positions()
    bad = compare(z, nref, pos)
    assert not bad, f"HIP engine's reference positions differ from the reference on docs {bad[:8]}"
