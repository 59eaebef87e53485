"""Delta events against the REFERENCE merge-tree (tests/golden/refdelta_*.npz).

The fixtures hold the stream of callbacks the reference `Client` fires while it replays each fixture
document — mergeTreeDeltaCallback (INSERT / REMOVE / ANNOTATE with Client.getPosition of every delta
segment and the annotate propertyDeltas) and mergeTreeMaintenanceCallback (SPLIT / APPEND / UNLINK),
i.e. what SharedString's "sequenceDelta" / "maintenance" listeners see (sequence.ts:136-150) — in the
word format of include/mt_oplog.h. They were recorded by tools/ref_replay.mjs --deltas on the type-erased
reference (tools/make_ref_goldens.py --deltas) over the same generator logs as tests/golden/ref_*.npz:
per-document word counts and FNV-1a-64, plus the full streams of the first two documents.

CPU tier: the host build of the engine core emits the reference's stream on every document. GPU tier:
the HIP engine does, with a log too small for the longest streams (the digest still covers every word).
"""
import dataclasses
import glob
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
from test_ref_goldens import caps_for

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = [os.path.basename(f)[9:-4] for f in sorted(glob.glob(os.path.join(GOLDEN, "refdelta_*.npz")))]


def load(name):
    z = np.load(os.path.join(GOLDEN, f"refdelta_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    return z, w, gen.generate(w, ids=z["doc_ids"], threads=8)


def first_diff(a, b):
    m = min(len(a), len(b))
    i = np.nonzero(a[:m] != b[:m])[0]
    return int(i[0]) if len(i) else m


def test_delta_fixture_set_complete():
    assert set(NAMES) >= {"c1_farm", "c2_observer", "c3_lagged", "c3_lagged_long", "c4_scaled", "c5_perm"}


def test_delta_stream_format_example():
    """One annotated insert/remove/annotate sequence decoded by hand (mt_oplog.h MT_DELTA_*)."""
    from fluidframework_amd import oplog as ol
    it = gen.generator_interner()
    log = ol.DocLog(it, local_long_id=0)
    log.add(ol.OP_INSERT, client=1, seq=1, ref_seq=0, min_seq=0, pos1=0, text="hello")
    log.add(ol.OP_INSERT, client=1, seq=2, ref_seq=1, min_seq=1, pos1=2, text="XY")    # splits "hello"
    log.add(ol.OP_REMOVE, client=1, seq=3, ref_seq=2, min_seq=2, pos1=1, pos2=4)       # "h[eXY]llo"
    b = ol.Batch.from_logs([log])
    st = core_host.HostStore(1, core_host.DEFAULT_CAPS, dcap=4096)
    st.start_collab(0, 0)
    ops, text, props, kv = b.doc(0)
    assert st.replay(0, ops, text, props, kv) == 0
    n, _, w = st.deltas(0)
    E = -(1 << 31)  # MT_DELTA_END
    want = [0, 1, 0, 5, 0, E, 1,                      # INSERT seq 1: "hello" at 0
            -2, 2, -1, 2, 0, -1, 3, 0, E, 2,          # SPLIT at 2: "he" + "llo"
            0, 2, 2, 2, 0, E, 1,                      # INSERT seq 2: "XY" at 2
            -2, 3, -1, 1, 0, -1, 1, 0, E, 2,          # SPLIT "he" at 1 (remove start; the end is a boundary)
            1, 3, 1, 1, 0, 1, 2, 0, E, 2]             # REMOVE seq 3: "e" and "XY", both now at 1
    assert w.tolist()[: len(want)] == want
    assert n >= len(want)


@pytest.mark.parametrize("name", NAMES)
def test_host_core_delta_stream_matches_reference(name):
    z, w, b = load(name)
    c = caps_for(w)
    _, err, st = core_host.replay_batch(b, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]),
                                        dcap=1 << 16)
    assert (err == 0).all()
    bad = []
    for d in range(b.ndocs):
        n, h, _ = st.deltas(d)
        if n != z["nwords"][d] or h != int(z["hashes"][d]):
            bad.append(d)
    assert not bad, f"delta stream differs from the reference on docs {bad[:8]}"
    ko, kw = z["keep_off"], z["keep_words"]
    for d in range(len(ko) - 1):
        want = kw[ko[d]: ko[d + 1]]
        got = st.deltas(d)[2]
        if len(want) <= (1 << 16):
            assert np.array_equal(got, want), f"doc {d}: first difference at word {first_diff(got, want)}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_delta_stream_matches_reference(name):
    from fluidframework_amd.engine import Engine
    z, w, b = load(name)
    dcap = 1 << 15  # smaller than the longest streams: the digest covers the words past the log
    eng = Engine(b.ndocs, dcap=dcap, **caps_for(w))
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
    n, h = eng.delta_state()
    bad = np.nonzero((n != z["nwords"]) | (h != z["hashes"]))[0]
    assert len(bad) == 0, f"HIP engine's delta stream differs from the reference on docs {bad[:8]}"
    ko, kw = z["keep_off"], z["keep_words"]
    for d in range(len(ko) - 1):
        want = kw[ko[d]: ko[d + 1]][:dcap]
        got = eng.deltas(d)
        assert np.array_equal(got, want), f"doc {d}: first difference at word {first_diff(got, want)}"
    # the same engine with the stream off replays to the same trees (deltas observe, never steer)
    for waves in (1, 4, 8):  # every config-2/3 kernel build (mt_engine_set_variant)
        eng2 = Engine(b.ndocs, waves=waves, **caps_for(w))
        eng2.start_collab(b.local_long_id)
        eng2.replay(b)
        assert np.array_equal(eng.digests(), eng2.digests()), waves
        eng2.close()
