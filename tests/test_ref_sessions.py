"""Documents with more clients than the engine's 253 short-id slots, against the REFERENCE (tests/golden/refsess_*.npz,
tools/make_ref_goldens.py --sessions).

The logs are the generator's config-2/3/4/5 logs whose remote clients reconnect under a new long id at every message
that covers their previous one (tests/session_logs.py): 390 to 2,192 distinct clients per document, each registered by
the reference's getOrAddShortClientId (client.ts:637-661) without bound. The engine recycles the short ids of clients
with no row in the collaboration window (mt_core.h reclaim_shorts) and keeps a settled row's long ids in the
retired-client table, so the canonical dump — whose client fields are long ids — must still equal the reference's on
every document: the oracle and the host core on the CPU, the HIP engine (each build of the profile) on the GPU.
"""
import glob
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
import oracle_client as oc
import session_logs
from test_ref_goldens import _sha, caps_for

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(os.path.basename(f)[len("refsess_"):-4] for f in glob.glob(os.path.join(GOLDEN, "refsess_*.npz")))


def regenerate(name):
    z = np.load(os.path.join(GOLDEN, f"refsess_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    b = session_logs.with_sessions(gen.generate(w, ids=z["doc_ids"], threads=8), p=float(z["session_p"]))
    return z, w, b


def host_caps(w):
    """the host core has no capacity promotion: the profile that recycles short ids (HotMid or larger) directly"""
    c = dict(caps_for(w))
    if c["ncap"] < 2048:
        c.update(ncap=2048, hcap=max(c["hcap"], 4096))
    return c


def test_small_profiles_refuse_the_254th_client():
    """the config-2/3/5 profiles carry no short-id recycling: a document's 254th client latches E_CAPACITY there (and
    the engine's capacity promotion replays it in HotMid)"""
    z, w, b = regenerate("c3_sessions")
    c = caps_for(w)
    assert c["ncap"] <= 192
    _, herr, _ = core_host.replay_batch(b.subset(range(2)), (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"],
                                                           c["ccap"]))
    assert (herr == 5).all()  # MT_E_CAPACITY


def test_fixture_set_complete():
    assert set(NAMES) == {"c2_sessions", "c3_sessions", "c4_sessions", "c5_sessions"}
    for n in NAMES:
        z, _, _ = regenerate(n)
        assert int(z["nclients"].min()) > 253  # every document outgrows the short-id slots


@pytest.mark.parametrize("name", NAMES)
def test_oracle_and_host_core_match_reference(name):
    z, w, b = regenerate(name)
    assert _sha(b) == str(z["log_sha256"]), "generator or renaming no longer produces the fixture's op logs"
    assert list(z["nclients"]) == b.nclients
    _, odig, oerr = oc.replay_batch(b, threads=8)
    assert (oerr == 0).all() and (odig == z["digests"]).all()
    c = host_caps(w)
    hdig, herr, _ = core_host.replay_batch(b, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]))
    assert (herr == 0).all(), herr
    bad = np.nonzero(hdig != z["digests"])[0]
    assert len(bad) == 0, f"engine core (host build) differs from the reference on docs {bad[:8]}"


def _variants(name):
    _, w, _ = regenerate(name)
    c = caps_for(w)
    return [dict(waves=1), dict(waves=4), dict(waves=8)] if c["ncap"] <= 192 and w.mode != gen.MTG_MATRIX else [dict()]


GPU_CASES = [(n, v) for n in NAMES for v in _variants(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,variant", GPU_CASES,
                         ids=[n + "".join(f"-{k}{int(x)}" for k, x in v.items()) for n, v in GPU_CASES])
def test_gpu_engine_matches_reference(name, variant):
    from fluidframework_amd.engine import Engine
    z, w, b = regenerate(name)
    eng = Engine(b.ndocs, **variant, **caps_for(w))
    try:
        eng.start_collab(b.local_long_id)
        eng.replay(b)
        err, err_op = eng.errors()
        assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
        if caps_for(w)["ncap"] < 2048:  # the small profiles promote every such document to HotMid
            assert len(eng.promoted()) == b.ndocs
        bad = np.nonzero(eng.digests() != z["digests"])[0]
        assert len(bad) == 0, f"HIP engine differs from the reference on docs {bad[:8]}"
        # a settled row's client read back through the segment query: the long id, not a recycled slot's
        seg = eng.get_containing_segment(0, 0)
        assert seg is None or seg.client == -1 or seg.client < 0xFFFE
    finally:
        eng.close()
