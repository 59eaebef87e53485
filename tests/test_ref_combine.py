"""Annotates with combining ops "incr" / "consensus" against the REFERENCE (tests/golden/
refcombine.npz from tools/make_ref_goldens.py --combine over tests/combine_inject.py).

addProperties (segmentPropertiesManager.ts:92-106) modifies every key of a combining annotate, pending local
updates notwithstanding, and calls Properties.combine (properties.ts:26-59) with newValue still undefined (SURVEY
Appendix A2): "incr" stores `current + undefined` (NaN from a number or nothing, a string with "undefined" appended
from a string or a consensus object), "consensus" keeps a value the row has and stores a {value: undefined, seq}
object where it has none. The engine holds those values per document (include/mt_oplog.h MT_VALUE_DERIVED; the
value kinds the host declares, mt_engine_set_value_kinds, tell numbers from strings) and its canonical dump writes
them by content, as tools/ref_replay.mjs does for the reference's replicas. Compared per document of config-3 and
config-5 logs: the final replica after the whole log against the reference's (every document reaches such values),
two documents' dumps byte for byte, and the replica right before the first such record — host core and HIP
engine. Without the value kinds an incr over a present value latches MT_E_UNSUPPORTED."""
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


KINDS = ol.value_kinds(gen.generator_interner())


def check_keep(z, name, dump):
    off = z[f"{name}_keep_dump_off"]
    for i, d in enumerate(z[f"{name}_keep_docs"]):
        assert dump(int(d)) == z[f"{name}_keep_dumps"][off[i]: off[i + 1]].tobytes(), f"doc {d}"


def test_keep_dumps_hold_derived_values():
    """the stored reference dumps decode (oplog.parse_dump) and hold NaN, strings with "undefined" appended and
    consensus objects"""
    z = np.load(os.path.join(GOLDEN, "refcombine.npz"), allow_pickle=False)
    kinds = set()
    for name in SETS:
        off = z[f"{name}_keep_dump_off"]
        for i in range(len(off) - 1):
            _, segs = ol.parse_dump(z[f"{name}_keep_dumps"][off[i]: off[i + 1]].tobytes())
            kinds |= {v.kind for sg in segs for _, v in sg["props"] if isinstance(v, ol.Derived)}
    assert kinds == {"nan", "strcat", "cons"}


@pytest.mark.parametrize("name", sorted(SETS))
def test_host_core_combining_ops_match_reference(name):
    z, b, pre, first, caps, c = load(name)
    dig, err, st = core_host.replay_batch(pre, caps, kinds=KINDS)
    assert (err == 0).all()
    assert np.array_equal(dig, z[f"{name}_prefix_digests"])
    dig, err, st = core_host.replay_batch(b, caps, kinds=KINDS)
    assert (err == 0).all(), [(d, st.error_op(d)) for d in np.nonzero(err)[0][:4]]
    bad = np.nonzero(dig != z[f"{name}_final_digests"])[0]
    assert len(bad) == 0, f"host core differs from the reference on docs {bad[:8]}"
    check_keep(z, name, st.dump)


@pytest.mark.parametrize("name", sorted(SETS))
def test_host_core_incr_without_value_kinds_latches(name):
    z, b, pre, first, caps, c = load(name)
    _, err, st = core_host.replay_batch(b, caps)
    incr_docs = [d for d in range(b.ndocs) if d % 2 == 0]  # combine_inject: a late incr in every other document
    assert all(err[d] in (0, E_UNSUPPORTED) for d in range(b.ndocs))
    assert (err[incr_docs] == E_UNSUPPORTED).any()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SETS))
def test_gpu_combining_ops_match_reference(name):
    from fluidframework_amd.engine import Engine
    z, b, pre, first, caps, c = load(name)
    eng = Engine(b.ndocs, **c)
    eng.set_value_kinds(KINDS)
    eng.start_collab(pre.local_long_id)
    eng.replay(pre)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert np.array_equal(eng.digests(), z[f"{name}_prefix_digests"])
    for waves in ((1, 4, 8) if c["ncap"] <= 192 else (None,)):
        eng2 = Engine(b.ndocs, waves=waves, **c)
        eng2.set_value_kinds(KINDS)
        eng2.start_collab(b.local_long_id)
        eng2.replay(b)
        err, err_op = eng2.errors()
        assert (err == 0).all(), (err[err != 0][:4], err_op[err != 0][:4])
        bad = np.nonzero(eng2.digests() != z[f"{name}_final_digests"])[0]
        assert len(bad) == 0, f"HIP engine differs from the reference on docs {bad[:8]}"
        check_keep(z, name, eng2.dump)
        eng2.close()
