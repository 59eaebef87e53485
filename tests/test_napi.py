"""The Node-API addon (fluidframework_amd/napi/mt_napi.cc -> build/mt_napi.node) and its JavaScript
facade (fluidframework_amd/js/mergetree_gpu.js), under node 12.

CPU tier: node loads the addon (and through it libmtreplay.so), which exports the engine's entry
points; the facade loads; creating an engine without a GPU fails loudly (no CPU fallback).
GPU tier: known-answer scenarios of the reference's specs driven from JavaScript (tests/napi_kat.js)
through facade -> addon -> HIP engine, with the facade's group ops, local edits + acks and segment
queries.
"""
import json
import os
import shutil
import subprocess

import pytest

from fluidframework_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")

EXPORTS = ["create", "startCollab", "submit", "run", "sync", "reset", "errors", "digests", "getLength", "getText",
           "getContainingSegment", "getPosition", "ndocs", "lastRunMs", "deltas", "refPositions", "submitDocs",
           "docError"]


def _node(script: str) -> str:
    r = subprocess.run([NODE, "-e", script], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_addon_loads_and_exports_entry_points():
    addon = native.build_napi()
    out = json.loads(_node(f"const a = require({json.dumps(addon)}); "
                           "console.log(JSON.stringify({keys: Object.keys(a), rec: a.OP_RECORD_BYTES}))"))
    assert set(EXPORTS) <= set(out["keys"])
    assert out["rec"] == 32


def test_facade_loads():
    native.build_napi()
    out = _node("const f = require('./fluidframework_amd/js/mergetree_gpu.js'); "
                "console.log([typeof f.ReplayEngine, typeof f.GpuClient, Object.keys(f.OP).join()].join(' '))")
    assert out == "function function INSERT,REMOVE,ANNOTATE,GROUP,NOOP"


def test_delta_stream_decoder():
    """decodeDeltas on a hand-written stream (include/mt_oplog.h): an annotate with one property delta
    and one blocked segment, then an UNLINK."""
    native.build_napi()
    E = -(1 << 31)
    words = [2, 7, 3, 4, 1, (1 << 16) | 2, 9, 1, -1, E, 2, -3, 8, -1, 6, 0, E, 1]
    out = json.loads(_node(
        "const f = require('./fluidframework_amd/js/mergetree_gpu.js'); const it = new f.Interner(); "
        "it.key('bold'); it.value(true); it.value(false); "
        f"console.log(JSON.stringify(f.decodeDeltas(Int32Array.from({json.dumps(words)}), it)))"))
    assert out == [{"operation": "ANNOTATE", "seq": 7, "deltaSegments": [
                        {"position": 3, "length": 4, "propertyDeltas": {"bold": False}},
                        {"position": 9, "length": 1}]},
                   {"operation": "UNLINK", "seq": 8, "deltaSegments": [{"length": 6}]}]


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    native.build_napi()
    out = _node("const f = require('./fluidframework_amd/js/mergetree_gpu.js'); "
                "try { new f.ReplayEngine(2); console.log('created'); } catch (e) { console.log(e.message); }")
    assert "mt_engine_create failed" in out


@pytest.mark.gpu
def test_known_answers_through_node():
    native.build_napi()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "napi_kat.js")], capture_output=True, text=True,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # client.applyMsg.spec.ts:88-98: the local insert is unacked (-1) until its message (seq 17)
    assert out["insertBeforeAck"] == "abchello world"
    assert out["insertSeqBeforeAck"] == -1 and out["insertSeqAfterAck"] == 17
    assert out["positionOfSecond"] == 3
    # client.applyMsg.spec.ts:100-110
    assert out["removeBeforeAck"] == "ello world" and out["removeAfterAck"] == "ello world"
    # concurrent inserts around a locally deleted segment (oracle-pinned answer)
    assert out["intersecting"] == "bc"
    # a remote replaceRange group (sequence.ts:455-469): insert "!" at 11, remove [5, 11)
    assert out["groupReplace"] == "hello!" and out["groupLength"] == 6
    assert len(out["digests"]) == 4
    # delta events: the insert; the annotate's boundary split then the annotate (bold was absent: null);
    # the remove's boundary split then the remove of " " (sequence.ts:136-150 listener view)
    ev = [(e["operation"], e["seq"], [(s.get("position"), s["length"], s.get("propertyDeltas"))
                                      for s in e["deltaSegments"]]) for e in out["deltas"]]
    assert ev == [("INSERT", 1, [(0, 11, None)]),
                  ("SPLIT", 2, [(None, 5, None), (None, 6, None)]),
                  ("ANNOTATE", 2, [(0, 5, {"bold": None})]),
                  ("SPLIT", 3, [(None, 1, None), (None, 5, None)]),
                  ("REMOVE", 3, [(5, 1, None)])]
    # local reference at "w"; the remove of " wo" slides it to "rld" (position 5); an insert at it goes
    # before "rld" and after the tombstone; reconnect regenerates that insert at 5
    # (localReference.ts, mergeTree.ts:2033-2130, client.ts:675-762); the same scenario on the
    # type-erased reference gives these values
    assert (out["refBefore"], out["refSlid"], out["refText"], out["refAfterInsert"]) == (6, 5, "helloXrld", 6)
    assert out["regen"] == [{"type": 0, "pos1": 5, "length": 1}]


@pytest.mark.gpu
def test_merge_tree_calls_text_ranges_and_per_doc_seqs_through_node():
    """tests/napi_kat2.js: MergeTree-level calls with explicit (refSeq, clientId, seq), per-document minSeq /
    currentSeq at collaboration start and getText with placeholder / start / end, through node -> addon ->
    GPU; the answers are the type-erased reference's for the same steps (tools/make_napi_kat2.mjs)"""
    native.build_napi()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "napi_kat2.js")], capture_output=True, text=True,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "napi_kat2_expected.json")))
    assert out["answers"] == want
    assert out["starUnsupported"]  # the "*" placeholder (Marker.toString()) is not modelled


@pytest.mark.gpu
def test_client_surface_through_node():
    """tests/napi_kat3.js: the rest of the Client surface SharedString / SharedSegmentSequence / SharedMatrix call
    (walkSegments with splitRange, getPropertiesAtPosition, getRangeExtentsOfPosition, resolveRemoteClientPosition,
    localTransaction, insertSegmentLocal, findTile, getMarkerFromId, annotateMarker, removeLocalReference,
    PermutationVector adjustPosition / handleToPosition) through node -> addon -> GPU; the answers are the
    type-erased reference's for the same steps (tools/make_napi_kat3.mjs)"""
    native.build_napi()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "napi_kat3.js")], capture_output=True, text=True,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "napi_kat3_expected.json")))
    assert len(out["answers"]) == len(want)
    for i, (g, w) in enumerate(zip(out["answers"], want)):
        assert g == w, (i, g, w)
    assert out["refused"]  # a perspective the reference's partial lengths answer differently is refused


@pytest.mark.gpu
def test_subsequence_through_node():
    """tests/napi_subseq.js: a SharedObjectSequence replica through node -> addon -> GPU (insertItemsLocal, {items}
    messages, an ack, getItems / getItemCount, getText with and without placeholder, segments either side of MaxRun);
    the answers are the type-erased reference's for the same steps (tools/make_napi_subseq.mjs)"""
    native.build_napi()
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "napi_subseq.js")], capture_output=True, text=True,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "napi_subseq_expected.json")))
    assert len(out["answers"]) == len(want)
    for i, (g, w) in enumerate(zip(out["answers"], want)):
        assert g == w, (i, g, w)


def test_typings_declare_every_export_and_method():
    """fluidframework_amd/js/mergetree_gpu.d.ts declares every name the facade exports and every public method
    of its classes (no TypeScript compiler in this image: a textual check)"""
    import re
    js = open(os.path.join(ROOT, "fluidframework_amd", "js", "mergetree_gpu.js")).read()
    dts = open(os.path.join(ROOT, "fluidframework_amd", "js", "mergetree_gpu.d.ts")).read()
    exports = re.search(r"module\.exports = \{([^}]*)\}", js, re.S).group(1)
    names = [n.strip() for n in exports.replace("\n", " ").split(",") if n.strip()]
    for n in names:
        assert re.search(rf"\b(class|const|function) {n}\b", dts), f"{n} is not declared in the typings"
    for cls in ("ReplayEngine", "GpuClient", "GpuMergeTree"):
        body = js[js.index(f"class {cls} "):]
        body = body[: body.index("\n}\n")]
        methods = set(re.findall(r"^    (?:get )?([a-zA-Z]\w*)\(", body, re.M)) - {"constructor", "if", "for"}
        dbody = dts[dts.index(f"class {cls} "):]
        dbody = dbody[: dbody.index("\n}\n")]
        internal = {"enqueue", "propsRecord", "checkDoc", "fields", "sent", "read"}
        for m in methods - internal:
            assert re.search(rf"\b{m}\b", dbody), f"{cls}.{m} is not declared in the typings"


@pytest.mark.gpu
def test_interactive_reads_flush_only_dirty_documents():
    """tools/facade_latency.js on a 4,096-document engine: local edits, remote sequenced inserts and reads, each read
    flushing only the documents with queued records (mt_engine_submit_docs) and reading one document's error
    (mt_engine_doc_error); every answer is checked by the script against the text it expects."""
    native.build_napi()
    r = subprocess.run([NODE, os.path.join(ROOT, "tools", "facade_latency.js"), "4096", "40"], capture_output=True,
                       text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["answers_checked"] and out["docs_touched"] > 40
