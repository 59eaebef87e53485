"""Snapshot emit + load pinned to the REFERENCE (tests/golden/ref_*.npz, snap_* fields).

tools/make_ref_goldens.py ran, for every document of every fixture set, the reference's own
SnapshotV1 (extractSync + emit, snapshotV1.ts:82-234) on the replica after records [0, cut) — cut is
a point where the replica has no unacked op — then Client.load (SnapshotLoader, snapshotLoader.ts)
of that tree into a fresh client with the same long id, which applied records [cut, end). The fixture
keeps a hash of each emitted tree (blob JSON with sorted keys: property-set key order is insertion
order in the reference and key-id order here), the FNV-1a-64 digest of each loaded client's final
canonical dump, the record at which a loaded client threw (the v1 format drops overlapping-remove
client lists, so a few loaded replicas cannot apply their tail — the engine must fail on the same
record), and the trees of the first documents.

Here the same is done with the product path (fluidframework_amd/snapshot.py over the oracle, the host
build of the engine core, or the HIP engine): emit from the dump after [0, cut) must hash equal to
the reference's tree; loading OUR tree (and, for the stored documents, the REFERENCE's tree) plus the
tail must reproduce the reference's loaded digests and its failures.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
from fluidframework_amd import snapshot as sn
import core_host
import oracle_client as oc
from test_ref_goldens import NAMES, caps_for, regenerate

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def canonical_tree(tree: dict) -> str:
    """Same canonical form as tools/make_ref_goldens.py canonical_tree."""
    blobs = sn._blobs(tree)
    return json.dumps({k: json.loads(v) for k, v in blobs.items()}, sort_keys=True, separators=(",", ":"))


def sha(tree) -> str:
    return hashlib.sha256(canonical_tree(tree).encode()).hexdigest()


def long_name(i: int) -> str:
    return f"c{i}" if i >= 0 else "original"


def client_index(name: str) -> int:
    return int(name[1:])


SETS = NAMES + ["snap_body"]


def fixture(name):
    """(fixture, batch, interner, caps): the generator's sets regenerate their logs; the synthetic
    body-window set (tools/make_ref_goldens.py snap_body_logs) stores them."""
    if name != "snap_body":
        z, w, b = regenerate(name)
        return z, b, gen.generator_interner(), caps_for(w)
    z = np.load(os.path.join(GOLDEN, "refsnap_body.npz"), allow_pickle=False)
    b = ol.Batch(z["ops"], z["op_off"], z["text"], z["text_off"], z["props"], z["props_off"], z["kv"], z["kv_off"],
                 z["local"])
    t = json.loads(str(z["interner"]))
    it = ol.Interner()
    for k in t["keys"][1:]:
        it.key(k)
    for v in t["values"][1:]:
        it.value(json.loads(v))
    assert it.keys == t["keys"] and it.values == t["values"]
    return z, b, it, dict(ncap=16384, hcap=32768, acap=1 << 18, mcap=4096, gcap=1024, ccap=64)


def load_arrays(tree, b: ol.Batch, d: int, cut: int, it=None):
    """The loaded replica's record stream: the snapshot's load records, then records [cut, end)."""
    log = ol.DocLog(it or gen.generator_interner())
    sn.load_records(tree, log, client_index, long_name(int(b.local_long_id[d])))
    ops, text, props, kv = b.doc_arrays(d)
    return ol.concat_records(log.arrays(), (ops[cut:], text, props, kv)), len(log.ops)


def prefix_arrays(b: ol.Batch, d: int, cut: int):
    ops, text, props, kv = b.doc_arrays(d)
    return ops[:cut], text, props, kv


def has_snapshots(z) -> bool:
    return "snap_cut" in z.files


def oracle_dump(arrays, local, it=None):
    c = oc.OracleClient(it or gen.generator_interner())
    c.start_collab(local)
    err = c.replay_arrays(*arrays)
    return err, c


def oracle_error_index(arrays, it=None) -> int:
    """The record at which the oracle fails (replaying record by record)."""
    ops, text, props, kv = arrays
    c = oc.OracleClient(it or gen.generator_interner())
    for i in range(len(ops)):
        if c.replay_arrays(ops[i: i + 1], text, props, kv):
            return i
    return -1


def check_loaded(z, d, err, err_at, digest, nload, ops):
    if "snap_load_error" in z.files and z["snap_load_error"][d]:
        # the reference cannot load its own snapshot of this document: loadBody's insertSegments at
        # root.cachedLength under the (UniversalSequenceNumber, segment client) perspective
        # (snapshotLoader.ts:200-213) finds no such position when a window segment of another client
        # precedes it; the engine must fail during the load records too
        assert err == 1 and 0 <= err_at < nload, f"doc {d}: the reference fails to load; here err {err} at {err_at}"
        return
    want_at = int(z["snap_tail_error"][d])
    if err and 0 <= err_at < len(ops):  # the reference applies a group message at its last record
        while ops[err_at]["kind"] & ol.OPF_GROUPED and err_at + 1 < len(ops):
            err_at += 1
    if want_at >= 0:
        assert err != 0, f"doc {d}: the reference's loaded client threw at tail record {want_at}; no error here"
        assert err_at - nload == want_at, f"doc {d}: error at tail record {err_at - nload}, reference {want_at}"
    else:
        assert err == 0, f"doc {d}: error {err} at record {err_at}"
        assert digest == int(z["snap_loaded_digests"][d]), f"doc {d}: loaded digest differs from the reference"


@pytest.mark.parametrize("name", SETS)
def test_oracle_snapshot_emit_and_load_match_reference(name):
    z, b, it, _ = fixture(name)
    if not has_snapshots(z):
        pytest.skip("fixture predates snapshots")
    for d in range(b.ndocs):
        cut = int(z["snap_cut"][d])
        local = int(b.local_long_id[d])
        err, c = oracle_dump(prefix_arrays(b, d, cut), local, it)
        assert err == 0
        tree = sn.emit_from_dump(c.dump(), it, long_name)
        assert sha(tree) == str(z["snap_sha256"][d]), f"doc {d}: emitted snapshot differs from the reference's"
        arrays, nload = load_arrays(tree, b, d, cut, it)
        err, c2 = oracle_dump(arrays, -1, it)
        at = oracle_error_index(arrays, it) if err else -1
        check_loaded(z, d, err, at, c2.digest() if err == 0 else 0, nload, arrays[0])


@pytest.mark.parametrize("name", SETS)
def test_host_core_snapshot_emit_and_load_match_reference(name):
    z, b, it, c = fixture(name)
    if not has_snapshots(z):
        pytest.skip("fixture predates snapshots")
    caps = (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"])
    st = core_host.HostStore(b.ndocs, caps)
    ld = core_host.HostStore(b.ndocs, caps)
    for d in range(b.ndocs):
        cut = int(z["snap_cut"][d])
        st.start_collab(d, int(b.local_long_id[d]))
        assert st.replay(d, *prefix_arrays(b, d, cut)) == 0
        tree = sn.emit_from_dump(st.dump(d), it, long_name)
        assert sha(tree) == str(z["snap_sha256"][d]), f"doc {d}: emitted snapshot differs from the reference's"
        arrays, nload = load_arrays(tree, b, d, cut, it)
        err = ld.replay(d, *arrays)
        check_loaded(z, d, err, ld.error_op(d) if err else -1, ld.digest(d) if err == 0 else 0, nload, arrays[0])


@pytest.mark.parametrize("name", SETS)
def test_reference_trees_load(name):
    """The stored documents: the REFERENCE's emitted tree itself (not ours) loads and replays."""
    z, b, it, _ = fixture(name)
    if not has_snapshots(z):
        pytest.skip("fixture predates snapshots")
    trees = json.loads(str(z["snap_trees" if name == "snap_body" else "keep_snap_trees"]))
    for d, tree in enumerate(trees):
        assert sha(tree) == str(z["snap_sha256"][d])
        arrays, nload = load_arrays(tree, b, d, int(z["snap_cut"][d]), it)
        err, c = oracle_dump(arrays, -1, it)
        at = oracle_error_index(arrays, it) if err else -1
        check_loaded(z, d, err, at, c.digest() if err == 0 else 0, nload, arrays[0])


def test_body_window_set_shape():
    """The synthetic set really has body chunks with window merge info, and both outcomes."""
    z, b, it, _ = fixture("snap_body")
    trees = json.loads(str(z["snap_trees"]))
    for tree in trees:
        blobs = sn._blobs(tree)
        assert len(blobs) >= 2
        body = json.loads(blobs["body_0"])["segments"]
        assert any(isinstance(x, dict) and "json" in x for x in body)
    assert z["snap_load_error"].any() and not z["snap_load_error"].all()


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])  # the prefix replay on both config-2/3 kernel builds
@pytest.mark.parametrize("name", [n for n in SETS if n != "c4_large"])
def test_gpu_snapshot_emit_and_load_match_reference(name, waves):
    """Both halves on the HIP engine: the prefix replays on the GPU and its dumps are emitted; the
    loaded replicas (load records + tail) replay on the GPU as one batch. (c4_large, two 300k-message
    documents, runs on the CPU tier only: its load records alone are minutes of one wave's work.)"""
    from fluidframework_amd.engine import Engine
    z, b, it, caps = fixture(name)
    if not has_snapshots(z):
        pytest.skip("fixture predates snapshots")
    cuts = [int(x) for x in z["snap_cut"]]
    pre = Engine(b.ndocs, waves=waves, **caps)
    pre.start_collab(b.local_long_id)
    pre.replay(ol.Batch.from_arrays([prefix_arrays(b, d, cuts[d]) for d in range(b.ndocs)], b.local_long_id))
    err, _ = pre.errors()
    assert (err == 0).all()
    loads, nloads = [], []
    for d in range(b.ndocs):
        tree = sn.emit_from_dump(pre.dump(d), it, long_name)
        assert sha(tree) == str(z["snap_sha256"][d]), f"doc {d}: emitted snapshot differs from the reference's"
        a, n = load_arrays(tree, b, d, cuts[d], it)
        loads.append(a)
        nloads.append(n)
    pre.close()
    eng = Engine(b.ndocs, **caps)  # no start_collab: each loaded replica starts detached
    eng.replay(ol.Batch.from_arrays(loads, np.full(b.ndocs, -1, np.int32)))
    err, err_op = eng.errors()
    dig = eng.digests()
    for d in range(b.ndocs):
        check_loaded(z, d, int(err[d]), int(err_op[d]), int(dig[d]), nloads[d], loads[d][0])
