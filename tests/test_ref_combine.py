"""Annotates with combining ops "incr" / "consensus" against the REFERENCE (tests/golden/
refcombine.npz from tools/make_ref_goldens.py --combine over tests/combine_inject.py).

addProperties (segmentPropertiesManager.ts:92-106) modifies every key of a combining annotate, pending local
updates notwithstanding, and calls Properties.combine (properties.ts:26-59) with newValue still undefined (SURVEY
Appendix A2): "incr" stores NaN, "consensus" keeps a value the row has and stores a {value: undefined, seq} object
where it has none. The engine keeps the kept values and latches MT_E_UNSUPPORTED on the record where the reference
first stores NaN or such an object. Compared, per document of config-3 and config-5 logs: the latched error and its
record against the reference's first such record, and the replica right before it (the log's prefix) against the
reference's digest of the same prefix — host core and HIP engine."""
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
import combine_inject
import core_host
from make_goldens_sha import log_sha
from test_ref_goldens import caps_for

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = {"c3": 64, "c5": 32}
E_UNSUPPORTED = 4


def load(name):
    z = np.load(os.path.join(GOLDEN, "refcombine.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z[f"{name}_workload"])))
    b = combine_inject.inject(gen.generate(w, ids=range(SETS[name]), threads=8))
    assert log_sha(b) == str(z[f"{name}_log_sha256"]), "the injected logs differ from the fixture's"
    first = z[f"{name}_first"]
    pre = ol.Batch.from_arrays([tuple(x if k else x[: (first[i] if first[i] >= 0 else len(x))]
                                      for k, x in enumerate(b.doc_arrays(i))) for i in range(b.ndocs)], b.local_long_id)
    c = caps_for(w)
    return z, b, pre, first, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]), c


def kept_before(b, first) -> int:
    """consensus annotates applied before each document's first combined value (their values are kept)"""
    n = 0
    for d in range(b.ndocs):
        ops = b.doc_arrays(d)[0][: max(int(first[d]), 0)]
        p = ops["props"][((ops["kind"] & 7) == ol.OP_ANNOTATE) & (ops["props"] > 0)].astype(np.int64)
        n += int((b.props[p - 1]["combining"] == ol.COMBINE_CONSENSUS).sum())
    return n


@pytest.mark.parametrize("name", sorted(SETS))
def test_fixture_has_kept_and_combined_values(name):
    z, b, pre, first, caps, c = load(name)
    assert (first >= 0).all()
    assert kept_before(b, first) > 0


@pytest.mark.parametrize("name", sorted(SETS))
def test_host_core_combining_ops_match_reference(name):
    z, b, pre, first, caps, c = load(name)
    dig, err, st = core_host.replay_batch(pre, caps)
    assert (err == 0).all()
    assert np.array_equal(dig, z[f"{name}_prefix_digests"])
    _, err, st = core_host.replay_batch(b, caps)
    assert (err == E_UNSUPPORTED).all()
    assert [st.error_op(d) for d in range(b.ndocs)] == first.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SETS))
def test_gpu_combining_ops_match_reference(name):
    from fluidframework_amd.engine import Engine
    z, b, pre, first, caps, c = load(name)
    eng = Engine(b.ndocs, **c)
    eng.start_collab(pre.local_long_id)
    eng.replay(pre)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert np.array_equal(eng.digests(), z[f"{name}_prefix_digests"])
    eng2 = Engine(b.ndocs, **c)
    eng2.start_collab(b.local_long_id)
    eng2.replay(b)
    err, err_op = eng2.errors()
    assert (err == E_UNSUPPORTED).all()
    assert err_op.tolist() == first.tolist()
