"""Golden vectors from the reference's own fixtures: the SharedString v1 snapshot files
(tests/golden/sequence_snapshots_v1, see tests/golden/README.md).

The edit scripts are restated from packages/dds/sequence/src/test/generateSharedStrings.ts:24-98;
each is replayed as LOCAL edits of a non-collaborating replica (a detached SharedString), the
canonical segment dump is coalesced as SnapshotV1.extractSync does (snapshotV1.ts:181-215), and the
resulting JSON segment specs (TextSegment.toJSONObject textSegment.ts:48-54, Marker.toJSONObject
mergeTree.ts:690-694) must equal the fixture's segments, chunk by chunk concatenated
(getSeqLengthSegs never splits a segment, snapshotV1.ts:59-81)."""
import json
import os

import numpy as np
import pytest

from fluidframework_amd import oplog as ol
from fluidframework_amd import snapshot as sn
import oracle_client as oc
from replicas import parse_dump

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sequence_snapshots_v1")
SIZE_OF_FIRST_CHUNK = 10000  # SnapshotLegacy.sizeOfFirstChunk (snapshotlegacy.ts:57)
TEXT_GRANULARITY = 256       # MergeTree.TextSegmentGranularity (mergeTree.ts:1093)
TILE = 1                     # ReferenceType.Tile (ops.ts:6-15)


class _Doc:
    """A detached SharedString's client: every edit is a local op applied at once; positions for
    later edits are computed from the running local length, as the generator script does."""

    def __init__(self):
        self.it = ol.Interner()
        self.log = ol.DocLog(self.it)
        self.length = 0

    def insert_text(self, pos, text):
        self.log.add(ol.OP_INSERT | ol.OPF_LOCAL, pos1=pos, text=text)
        self.length += len(text)

    def insert_marker(self, pos, ref_type, props):
        self.log.add(ol.OP_INSERT | ol.OPF_LOCAL, pos1=pos, marker=ref_type, props=props)
        self.length += 1

    def annotate(self, start, end, props):
        self.log.add(ol.OP_ANNOTATE | ol.OPF_LOCAL, pos1=start, pos2=end, props=props)


def _script(name):
    """generateSharedStrings.ts:24-98 (insertText = "text")."""
    d = _Doc()
    if name == "headerOnly":
        for i in range(SIZE_OF_FIRST_CHUNK // 4 // 2):
            d.insert_text(0, f"text{i}")
    elif name == "headerAndBody":
        for i in range(SIZE_OF_FIRST_CHUNK // 4 * 2):
            d.insert_text(0, f"text{i}")
    elif name == "largeBody":
        for i in range(SIZE_OF_FIRST_CHUNK):
            d.insert_text(0, f"text-{i}")
    elif name == "withMarkers":
        for i in range(SIZE_OF_FIRST_CHUNK // 4 * 2):
            d.insert_text(0, f"text{i}")
        i = 0
        while i < d.length:  # the bound is re-read after every marker (sharedString.getLength())
            d.insert_marker(i, TILE, {"ItemType": "Paragraph", "Properties": {"Bold": False},
                                      "markerId": f"marker{i}", "referenceTileLabels": ["Eop"]})
            i += 70
    elif name == "withAnnotations":
        for i in range(SIZE_OF_FIRST_CHUNK // 4 * 2):
            d.insert_text(0, f"text{i}")
        for i in range(0, d.length, 70):
            d.annotate(i, i + 10, {"bold": True})
    else:
        raise ValueError(name)
    return d


def _golden_segments(name):
    tree = json.load(open(os.path.join(GOLD, name + ".json")))
    content = next(e for e in tree["entries"] if e["path"] == "content")["value"]["entries"]
    order = ["header"] + sorted((e["path"] for e in content if e["path"] != "header"),
                                key=lambda p: int(p.split("_")[1]))
    by = {e["path"]: json.loads(e["value"]["contents"]) for e in content}
    segs = []
    for p in order:
        segs.extend(by[p]["segments"])
    return segs


def _snapshot_segments(dump: bytes, it: ol.Interner):
    """The product's SnapshotV1.extractSync (fluidframework_amd/snapshot.py) over a dump, as specs."""
    hdr, segs = parse_dump(dump)
    return [spec for spec, _ in sn.extract_segments(hdr, segs, it, _long_name)]


def _long_name(i):
    return f"c{i}"


def _contents(tree):
    return {k: v for k, v in sn._blobs(tree).items()}


def _replay(kind, d: _Doc, local: int = 0) -> bytes:
    return _replay_arrays(kind, d.it, d.log.arrays(), local)


def _replay_arrays(kind, it, arrays, local):
    ops, text, props, kv = arrays
    if kind == "oracle":
        c = oc.OracleClient(it)
        assert c.replay_arrays(ops, text, props, kv) == 0
        return c.dump()
    if kind == "host":
        import core_host
        st = core_host.HostStore(1, (16384, 32768, 1 << 18, 1024, 64, 64))
        st.start_collab(0, local)
        assert st.replay(0, ops, text, props, kv) == 0
        return st.dump(0)
    from fluidframework_amd.engine import Engine
    eng = Engine(1, ncap=16384, hcap=32768, acap=1 << 18, mcap=1024, gcap=64, ccap=64)
    eng.start_collab([local])
    eng.replay(ol.Batch.from_arrays([(ops, text, props, kv)], [local]))
    err, _ = eng.errors()
    assert err[0] == 0
    return eng.dump(0)


NAMES = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"]


@pytest.mark.parametrize("kind", ["oracle", "host", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("name", NAMES)
def test_snapshot_golden(name, kind):
    d = _script(name)
    dump = _replay(kind, d, local=-1)  # a detached SharedString: no collaboration
    got = _snapshot_segments(dump, d.it)
    want = _golden_segments(name)
    assert len(got) == len(want)
    assert got == want
    # the whole emitted tree (SnapshotV1.emit: chunking, header metadata, JSON text) byte for byte
    tree = json.load(open(os.path.join(GOLD, name + ".json")))
    assert _contents(sn.emit_from_dump(dump, d.it, _long_name)) == _contents(tree)


@pytest.mark.parametrize("kind", ["oracle", "host", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("name", NAMES)
def test_snapshot_golden_load_roundtrip(name, kind):
    """SnapshotLoader (snapshotLoader.ts:86-228) of the fixture as load records: header reload
    (7-child blocks bottom-up), startOrUpdateCollaboration("snapshot"), body appends; the loaded
    replica's text is the fixture's, and emitting it again reproduces the fixture exactly."""
    tree = json.load(open(os.path.join(GOLD, name + ".json")))
    it = ol.Interner()
    log = ol.DocLog(it)
    md = sn.load_records(tree, log, lambda n: {"snapshot": 0}[n], "snapshot")
    dump = _replay_arrays(kind, it, log.arrays(), -1)
    hdr, segs = parse_dump(dump)
    assert hdr["length"] == md["totalLength"] and hdr["currentSeq"] == md["sequenceNumber"]
    text = "".join(s["text"] if s["kind"] == ol.SEG_TEXT else "" for s in segs)
    want = "".join(x if isinstance(x, str) else x.get("text", "") for x in sn.segment_specs(tree))
    assert text == want
    nhead = json.loads(sn._blobs(tree)["header"])["segmentCount"]
    assert hdr["nleaf"] >= -(-nhead // 7)  # reloadFromSegments' leaf blocks hold <= 7 segments
    assert _contents(sn.emit_from_dump(dump, it, lambda i: "snapshot")) == _contents(tree)


LEGACY = {"legacy": os.path.join(os.path.dirname(GOLD), "sequence_snapshots_legacy"),
          "legacyWithCatchUp": os.path.join(os.path.dirname(GOLD), "sequence_snapshots_legacy_catchup")}


@pytest.mark.parametrize("kind", ["oracle", "host", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("fmt", sorted(LEGACY))
@pytest.mark.parametrize("name", NAMES)
def test_legacy_snapshot_loads(name, fmt, kind):
    """The reference's legacy-format fixtures (packages/dds/sequence/src/test/snapshots/legacy*,
    snapshotVersion.spec.ts): chunks converted by toLatestVersion (snapshotChunks.ts:136-185), the
    catch-up ops blob applied after the body; the loaded document emits as the v1 fixture of the
    same content, byte for byte."""
    tree = json.load(open(os.path.join(LEGACY[fmt], name + ".json")))
    it = ol.Interner()
    log = ol.DocLog(it)
    sn.load_records(tree, log, lambda n: {"snapshot": 0}[n], "snapshot")
    dump = _replay_arrays(kind, it, log.arrays(), -1)
    v1 = json.load(open(os.path.join(GOLD, name + ".json")))
    assert _contents(sn.emit_from_dump(dump, it, lambda i: "snapshot")) == _contents(v1)


@pytest.mark.parametrize("kind", ["oracle", "host", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("fmt", sorted(LEGACY))
@pytest.mark.parametrize("name", NAMES)
def test_legacy_snapshot_emit_roundtrip(name, fmt, kind):
    """SnapshotLegacy emit (snapshotlegacy.ts:104-242, SharedString's default summary): the legacy
    fixture loaded into a replica is summarized again in the legacy format, with the fixture's
    catch-up blob name (options.catchUpBlobName) and its (empty) catch-up messages; every blob is the
    fixture's byte for byte. The same holds for the document built by the generator script."""
    tree = json.load(open(os.path.join(LEGACY[fmt], name + ".json")))
    want = _contents(tree)
    blob = [p for p in want if p not in (sn.HEADER, sn.BODY)]
    assert len(blob) == 1
    it = ol.Interner()
    log = ol.DocLog(it)
    sn.load_records(tree, log, lambda n: {"snapshot": 0}[n], "snapshot")
    dump = _replay_arrays(kind, it, log.arrays(), -1)
    assert _contents(sn.emit_legacy_from_dump(dump, it, [], catchup_blob=blob[0])) == want
    d = _script(name)
    dump = _replay(kind, d, local=-1)
    assert _contents(sn.emit_legacy_from_dump(dump, d.it, [], catchup_blob=blob[0])) == want
