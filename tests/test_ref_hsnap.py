"""SharedMatrix vectors loaded from summaries with allocated handles, against the REFERENCE (VERDICT r4 #5;
tests/golden/refhsnap_c5_perm.npz from tools/make_ref_goldens.py --hsnap).

The refhandles logs (config-5 PermutationVector replicas + getAllocatedHandle records) ran under the reference
with PermutationVector's bookkeeping; at a cut with nothing pending each replica was summarized as
PermutationVector.snapshot does (permutationvector.ts:256-268: the merge-tree's SnapshotV1 with PermutationSegment
specs [length, start], plus the HandleTable blob), and a fresh replica loaded it as PermutationVector.load does
(270-275: HandleTable.load, then Client.load with the vector's delta hooks installed, so loadBody's inserts reset
their segments' starts, 297-309) and applied the rest of the log. Here snapshot.load_records turns the same summary
and blob into load records (MT_NOOP_HTLOAD records, starts in the segments' records) ahead of the tail, and the
host core and the HIP engine must end with the reference's digests (dumps that carry allocated starts) and its
HandleTable.snapshot()."""
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
from fluidframework_amd import snapshot as sn
import core_host
import handles_inject
from make_goldens_sha import log_sha
from test_ref_goldens import caps_for
from test_snapshot_ref import client_index, long_name

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PCAP = 1 << 12


def load():
    z = np.load(os.path.join(GOLDEN, "refhsnap_c5_perm.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    c = caps_for(w)
    caps = (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"])
    b = handles_inject.inject(gen.generate(w, ids=z["doc_ids"], threads=8), caps)
    assert log_sha(b) == str(z["log_sha256"]), "the injected logs differ from the fixture's"
    trees = json.loads(str(z["trees"]))
    return z, c, caps, b, trees


def part(z, name, d):
    return z[name][z[name[:-1] + "_off"][d]: z[name[:-1] + "_off"][d + 1]]


def loaded_batch(z, b, trees) -> ol.Batch:
    """every document's loading replica: the summary's load records, then the log from the cut"""
    logs = []
    for d in range(b.ndocs):
        log = ol.DocLog(gen.generator_interner(), local_long_id=int(b.local_long_id[d]))
        sn.load_records(trees[d], log, client_index, long_name(int(b.local_long_id[d])),
                        handle_table=part(z, "blobs", d), perm_vector=True)
        ops, text, props, kv = b.doc_arrays(d)
        logs.append(ol.concat_records(log.arrays(), (ops[int(z["cuts"][d]):], text, props, kv)))
    return ol.Batch.from_arrays(logs, np.full(b.ndocs, -1, np.int32))  # detached: the COLLAB record starts collaboration


def test_fixture_summaries_hold_allocated_handles():
    z, c, caps, b, trees = load()
    assert not z["load_error"].any() and (z["tail_error"] < 0).all()
    starts = 0
    for d in range(b.ndocs):
        for spec in sn.segment_specs(trees[d]):
            if isinstance(spec, dict) and "json" in spec:
                spec = spec["json"]
            if isinstance(spec, list) and len(spec) > 1 and spec[1] is not None and spec[1] >= 1:
                starts += 1
    assert starts > 500
    assert sum(len(part(z, "blobs", d)) > 1 for d in range(b.ndocs)) > b.ndocs // 2


def test_host_core_loads_summaries_with_handles():
    z, c, caps, b, trees = load()
    lb = loaded_batch(z, b, trees)
    dig, err, st = core_host.replay_batch(lb, caps, pcap=PCAP)
    assert (err == 0).all(), np.nonzero(err)[0][:8]
    assert np.array_equal(dig, z["loaded_digests"])
    for d in range(b.ndocs):
        assert np.array_equal(st.handle_table(d), part(z, "finals", d)), f"doc {d}"


@pytest.mark.gpu
def test_gpu_loads_summaries_with_handles():
    from fluidframework_amd.engine import Engine
    z, c, caps, b, trees = load()
    lb = loaded_batch(z, b, trees)
    eng = Engine(lb.ndocs, **dict(c, pcap=PCAP))  # no start_collab: each loaded replica starts detached
    eng.replay(lb)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
    assert np.array_equal(eng.digests(), z["loaded_digests"])
    for d in range(lb.ndocs):
        assert np.array_equal(eng.handle_table(d), part(z, "finals", d)), f"doc {d}"
