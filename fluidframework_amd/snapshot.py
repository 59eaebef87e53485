"""Merge-tree snapshots: the v1 summary format <-> the engine.

Emit (SnapshotV1.extractSync + emit, packages/dds/merge-tree/src/snapshotV1.ts:156-234, 82-154):
the engine's canonical segment dump (mt_engine_dump, include/mt_oplog.h — read back from HBM) is
walked in document order; unacked segments and segments removed at or below the MSN are elided;
settled segments are coalesced (canAppend + matchProperties, as the reference's clone/append);
window segments keep their merge info ({json, seq, client, removedSeq, removedClient}); segments are
cut into chunks of ~chunkSize characters (getSeqLengthSegs, 59-81) and serialized as the v1 chunk
JSON (serializeAsMaxSupportedVersion). The result is the ITree of blobs the reference produces.

Load (SnapshotLoader, snapshotLoader.ts:86-228): the header chunk's segments become MT_OP_RELOAD
records (the engine rebuilds them as reloadFromSegments does, 7 children per block bottom-up,
mergeTree.ts:1229-1284), then MT_OP_COLLAB (startOrUpdateCollaboration with the header's
minSeq/currentSeq), then the body chunks' segments as MT_OP_APPEND records (loadBody's
insertSegments at the end of the local view). The records go through the normal replay path
(mt_engine_submit / mt_engine_run), so a batch of documents loads and then keeps replaying on the GPU.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from . import oplog as ol

HEADER = "header"           # SnapshotLegacy.header (snapshotlegacy.ts:55)
BODY = "body"               # SnapshotLegacy.body
CHUNK_SIZE = 10000          # SnapshotV1.chunkSize (snapshotV1.ts:40)
TEXT_GRANULARITY = 256      # TextSegmentGranularity (mergeTree.ts:1093)
MAX_RUN = 128               # SubSequence MaxRun (sequence sharedSequence.ts:12)
UNALLOCATED = -0x80000000   # Handle.unallocated (matrix handletable.ts:11)


def _js(v: Any) -> str:
    """JSON.stringify for the JSON-shaped values of a snapshot."""
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)


# ---- emit -------------------------------------------------------------------------------------
def _props(seg, interner: ol.Interner) -> Optional[Dict[str, Any]]:
    if not seg["flags"] & 1:  # MT_DF_HAS_PROPS: properties !== undefined
        return None
    return {interner.key_str(k): ol.derived_json(v, interner) if isinstance(v, ol.Derived) else interner.value_obj(v)
            for k, v in seg["props"]}


def _json_spec(seg, props, interner: Optional[ol.Interner] = None):
    """ISegment.toJSONObject: TextSegment (textSegment.ts:48-54), Marker (mergeTree.ts:690-694),
    PermutationSegment (permutationvector.ts:77-79), SubSequence (sequence sharedSequence.ts:43-47: {items} and
    addSerializedProps' props; the item ids map back through the interner's items)."""
    if seg["kind"] == ol.SEG_TEXT:
        return {"text": seg["text"], "props": props} if props is not None else seg["text"]
    if seg["kind"] == ol.SEG_RUN:
        j = {"items": [interner.item_obj(u) for u in seg["items"]]}
        if props is not None:
            j["props"] = props
        return j
    if seg["kind"] == ol.SEG_MARKER:
        j = {"marker": {"refType": seg["refType"]}}
        if props is not None:
            j["props"] = props
        return j
    return [seg["len"], seg.get("start", UNALLOCATED)]


def _can_append(a, b) -> bool:
    if a["kind"] == ol.SEG_PERM or b["kind"] == ol.SEG_PERM:  # PermutationSegment.canAppend (87-93)
        if a["kind"] != b["kind"]:
            return False
        sa, sb = a.get("start", UNALLOCATED), b.get("start", UNALLOCATED)
        return sb == UNALLOCATED if sa == UNALLOCATED else sb == sa + a["len"]
    if a["kind"] == ol.SEG_RUN:  # SubSequence.canAppend (sharedSequence.ts:57-60): no newline rule
        return b["kind"] == ol.SEG_RUN and (a["len"] <= MAX_RUN or b["len"] <= MAX_RUN)
    if a["kind"] != ol.SEG_TEXT or b["kind"] != ol.SEG_TEXT:  # Marker.canAppend is false
        return False
    return not a["text"].endswith("\n") and (a["len"] <= TEXT_GRANULARITY or b["len"] <= TEXT_GRANULARITY)


def _appended(prev, cur):
    """prev.append(cur) (TextSegment / SubSequence / PermutationSegment): the merged segment"""
    return dict(prev, len=prev["len"] + cur["len"],
                text=(prev["text"] + cur["text"]) if prev["kind"] == ol.SEG_TEXT else None,
                items=(prev["items"] + cur["items"]) if prev["kind"] == ol.SEG_RUN else None)


def extract_segments(hdr, segs, interner: ol.Interner, long_name) -> List[tuple]:
    """SnapshotV1.extractSync (snapshotV1.ts:156-234) over a parsed canonical dump: a list of
    (json spec, length). `long_name(i)` gives the long client id string of long-client index i."""
    min_seq = hdr["minSeq"]
    out: List[tuple] = []
    prev = None

    def push(p):
        if p is not None:
            out.append((_json_spec(p, p["_props"], interner), p["len"]))

    for s in segs:
        removed = s["removedSeq"] is not None
        if s["seq"] == -1 or (removed and s["removedSeq"] <= min_seq):
            continue  # unacked, or removed at/below the MSN (a pending removal, -1, is elided too)
        props = _props(s, interner)
        if s["seq"] <= min_seq and not removed:
            cur = dict(s, _props=props)
            if prev is None:
                prev = cur
            elif _can_append(prev, cur) and prev["_props"] == cur["_props"]:
                prev = _appended(prev, cur)
            else:
                push(prev)
                prev = cur
        else:
            push(prev)
            prev = None
            raw: Dict[str, Any] = {"json": _json_spec(s, props, interner)}
            if s["seq"] > min_seq:
                raw["seq"] = s["seq"]
                raw["client"] = long_name(s["client"])
            if removed:
                raw["removedSeq"] = s["removedSeq"]
                raw["removedClient"] = long_name(s["removedClient"])
            out.append((raw, s["len"]))
    push(prev)
    return out


def emit_v1(hdr, segs, interner: ol.Interner, long_name, chunk_size: int = CHUNK_SIZE) -> dict:
    """SnapshotV1.emit (snapshotV1.ts:82-154): the ITree of a merge-tree snapshot (header blob, then
    body_<i> blobs), contents serialized like serializeAsMaxSupportedVersion with JSON.stringify."""
    specs = extract_segments(hdr, segs, interner, long_name)
    chunks = []
    start = 0
    while True:
        seg_list, length, count = [], 0, 0
        while length < chunk_size and start + count < len(specs):  # getSeqLengthSegs (59-81)
            seg_list.append(specs[start + count][0])
            length += specs[start + count][1]
            count += 1
        chunks.append({"version": "1", "segmentCount": count, "length": length, "segments": seg_list,
                       "startIndex": start})
        start += count
        if start >= len(specs):
            break
    meta = {"minSequenceNumber": hdr["minSeq"], "sequenceNumber": hdr["currentSeq"],
            "orderedChunkMetadata": [{"id": HEADER}], "totalLength": sum(c["length"] for c in chunks),
            "totalSegmentCount": sum(c["segmentCount"] for c in chunks)}
    body = []
    for i, c in enumerate(chunks[1:]):
        cid = f"{BODY}_{i}"
        meta["orderedChunkMetadata"].append({"id": cid})
        body.append(_blob(cid, c))
    # the header is serialized last, so it lists every body chunk id (snapshotV1.ts:111-151)
    return {"entries": [_blob(HEADER, dict(chunks[0], headerMetadata=meta))] + body, "id": None}


def _blob(path: str, chunk: dict) -> dict:
    return {"mode": "100644", "path": path, "type": "Blob", "value": {"contents": _js(chunk), "encoding": "utf-8"}}


# ---- emit, legacy format (SharedString's default summary) -------------------------------------
CATCHUP = "catchupOps"      # SnapshotLegacy.catchupOps (snapshotlegacy.ts:56); options.catchUpBlobName


def extract_segments_legacy(hdr, segs, interner: ol.Interner) -> List[tuple]:
    """SnapshotLegacy.extractSync (snapshotlegacy.ts:179-242) over a parsed canonical dump: a list of
    (json spec, length). mergeTree.map(..., minSeq, NonCollabClient) visits the segments of nonzero
    length in that perspective (nodeMap, mergeTree.ts:2936-2998), and extractSegment keeps those
    sequenced at or below the MSN and not removed at or below it (a pending removal, -1, is kept);
    consecutive ones merge while prev.canAppend(segment) and their properties match (prev grows)."""
    min_seq = hdr["minSeq"]
    out: List[tuple] = []
    prev = None
    for s in segs:
        if s["len"] <= 0 or s["seq"] == -1 or s["seq"] > min_seq:
            continue
        rs = s["removedSeq"]
        if rs is not None and rs != -1 and rs <= min_seq:
            continue
        cur = dict(s, _props=_props(s, interner))
        if prev is not None and _can_append(prev, cur) and prev["_props"] == cur["_props"]:
            prev = _appended(prev, cur)
        else:
            if prev is not None:
                out.append((_json_spec(prev, prev["_props"], interner), prev["len"]))
            prev = cur
    if prev is not None:
        out.append((_json_spec(prev, prev["_props"], interner), prev["len"]))
    return out


def emit_legacy(hdr, segs, interner: ol.Interner, catchup: Optional[List[dict]] = None,
                chunk_size: int = CHUNK_SIZE, catchup_blob: str = CATCHUP) -> dict:
    """SnapshotLegacy.extractSync + emit (snapshotlegacy.ts:104-242), what Client.snapshot writes unless
    newMergeTreeSnapshotFormat is set (client.ts:895-935): a header chunk of the first segments up to
    ~chunk_size characters, one body chunk with the rest, and the caller's catch-up messages
    (SharedString's messagesSinceMSNChange: see catchup_messages) as JSON. The chunks are the legacy
    chunk object serialized by serializeAsMinSupportedVersion (snapshotChunks.ts:76-122), key order
    included (`version` is undefined and JSON.stringify drops it)."""
    specs = extract_segments_legacy(hdr, segs, interner)
    total = sum(n for _, n in specs)  # segmentsTotalLength (the extracted total wins a mismatch, 232-240)
    seq = hdr["minSeq"]

    def chunk(approx, start):  # getSeqLengthSegs (75-100)
        seg_list, length, count = [], 0, 0
        while length < approx and start + count < len(specs):
            seg_list.append(specs[start + count][0])
            length += specs[start + count][1]
            count += 1
        return {"chunkStartSegmentIndex": start, "chunkSegmentCount": count, "chunkLengthChars": length,
                "totalLengthChars": total, "totalSegmentCount": len(specs), "chunkSequenceNumber": seq,
                "segmentTexts": seg_list}

    c1 = chunk(chunk_size, 0)
    ids = [{"id": HEADER}] + ([{"id": BODY}] if c1["chunkLengthChars"] < total else [])
    # buildHeaderMetadataForLegecyChunk (snapshotChunks.ts:165-185): minSequenceNumber is undefined
    c1["headerMetadata"] = {"orderedChunkMetadata": ids, "sequenceNumber": seq, "totalLength": total,
                            "totalSegmentCount": len(specs)}
    entries = [_blob(HEADER, c1)]
    if c1["chunkSegmentCount"] < len(specs):
        entries.append(_blob(BODY, chunk(total, c1["chunkSegmentCount"])))
    entries.append({"mode": "100644", "path": catchup_blob, "type": "Blob",
                    "value": {"contents": _js(catchup or []), "encoding": "utf-8"}})
    return {"entries": entries, "id": None}


def _insert_spec(op: Dict[str, Any]):
    """TextSegment / Marker .toJSONObject() of the segment an insert op made, as a delta callback sees it:
    its properties are the op's with the null-valued keys deleted (addProperties, segmentPropertiesManager.ts
    100-106), present (possibly empty) whenever the op carried props."""
    seg = op["seg"]
    if isinstance(seg, dict) and "props" in seg:
        seg = dict(seg, props={k: v for k, v in seg["props"].items() if v is not None})
    return seg


def _same_props(a, b) -> bool:
    """matchProperties (properties.ts:61-92) of two JSON property sets (None: undefined)."""
    if a is None or b is None:
        return a is None and b is None
    return a == b


def ops_from_deltas(msg: Dict[str, Any], events, interner: ol.Interner) -> List[Dict[str, Any]]:
    """SharedSegmentSequence.createOpsFromDelta (sequence.ts:62-110) over the sequenceDelta events one
    message fired (delta words decoded by oplog.decode_deltas), ops accumulating across the events of a
    group: insert ranges become insert ops of the segment's JSON; remove ranges extend the last op when it
    starts at the range's position (its pos2 becomes NaN, JSON null, when it has none) or add
    [pos, pos + length); annotate ranges carry the segment's value (null if absent) of each changed key and
    extend the last op when it ends at the range and has the same props. A remote annotate that pending local
    rewrites blocked has no property deltas, and the reference's Object.keys(undefined) throws there."""
    members = msg["contents"]["ops"] if msg["contents"]["type"] == 3 else [msg["contents"]]
    inserts = [m for m in members if m["type"] == ol.OP_INSERT]
    annot = [m for m in members if m["type"] == ol.OP_ANNOTATE]
    out: List[Dict[str, Any]] = []
    nan = float("nan")
    for op, _seq, segs in events:
        if op == ol.OP_INSERT:
            ins = inserts.pop(0)
            for pos, _ln, _nd, _pd in segs:
                out.append({"pos1": pos, "seg": _insert_spec(ins), "type": ol.OP_INSERT})
        elif op == ol.OP_REMOVE:
            for pos, ln, _nd, _pd in segs:
                last = out[-1] if out else None
                if last is not None and last.get("pos1") == pos:
                    p2 = last.get("pos2", nan)
                    last["pos2"] = nan if p2 is None or p2 != p2 else p2 + ln
                else:
                    out.append({"pos1": pos, "pos2": pos + ln, "type": ol.OP_REMOVE})
        elif op == ol.OP_ANNOTATE:
            new = annot.pop(0)["props"]
            for pos, ln, nd, pd in segs:
                if pd is None:
                    raise ValueError("createOpsFromDelta: an annotate range without property deltas (its "
                                     "addProperties was blocked by pending local rewrites); the reference throws")
                props = {}
                for k, _v in pd:
                    key = interner.key_str(k)
                    props[key] = new.get(key)  # the key's value after the op: written from the op, or deleted
                last = out[-1] if out else None
                if last is not None and last.get("pos2") == pos and _same_props(last.get("props"), props):
                    last["pos2"] += ln
                else:
                    out.append({"pos1": pos, "pos2": pos + ln, "props": props, "type": ol.OP_ANNOTATE})
    for o in out:  # JSON.stringify(NaN) is null
        if "pos2" in o and o["pos2"] is not None and o["pos2"] != o["pos2"]:
            o["pos2"] = None
    return out


def catchup_messages(ops, text, props, kv, deltas, interner: ol.Interner, long_name, min_seq: int):
    """SharedString's messagesSinceMSNChange when it summarizes (sequence.ts:566-616): every sequenced op
    message the replica applied, those with referenceSequenceNumber != sequenceNumber - 1 rebased
    (refSeq = seq - 1, contents = createOpsFromDelta of the sequenceDelta events the message fired; one op,
    else a group of them: an ack fires none), then those above the MSN, with the MSN as their
    minimumSequenceNumber. `ops/text/props/kv`: the replica's records so far; `deltas`: its delta-stream
    words over the same records (an engine created with caps.dcap > 0)."""
    from . import wire
    by_seq: Dict[int, list] = {}
    for ev in ol.decode_deltas(deltas):
        if ev[0] in (ol.OP_INSERT, ol.OP_REMOVE, ol.OP_ANNOTATE) and ev[1] >= 0:
            by_seq.setdefault(ev[1], []).append(ev)
    stash = []
    for msg, _last in wire.record_messages(ops, text, props, kv, interner, long_name):
        if msg["type"] != wire.MSG_OP:
            continue
        if msg["referenceSequenceNumber"] != msg["sequenceNumber"] - 1:
            got = ops_from_deltas(msg, by_seq.get(msg["sequenceNumber"], []), interner)
            msg = dict(msg, referenceSequenceNumber=msg["sequenceNumber"] - 1,
                       contents=got[0] if len(got) == 1 else {"ops": got, "type": 3})
        stash.append(msg)
    return [dict(m, minimumSequenceNumber=min_seq) for m in stash if m["sequenceNumber"] > min_seq]


def emit_legacy_from_dump(dump: bytes, interner: ol.Interner, catchup: Optional[List[dict]] = None,
                          chunk_size: int = CHUNK_SIZE, catchup_blob: str = CATCHUP) -> dict:
    """emit_legacy over an engine / oracle canonical dump (bytes)."""
    hdr, segs = ol.parse_dump(dump)
    return emit_legacy(hdr, segs, interner, catchup, chunk_size, catchup_blob)


def emit_from_dump(dump: bytes, interner: ol.Interner, long_name, chunk_size: int = CHUNK_SIZE) -> dict:
    """emit_v1 over an engine / oracle canonical dump (bytes)."""
    hdr, segs = ol.parse_dump(dump)
    return emit_v1(hdr, segs, interner, long_name, chunk_size)


# ---- load -------------------------------------------------------------------------------------
def _blobs(tree: dict) -> Dict[str, str]:
    """path -> contents of a merge-tree snapshot tree; a SharedString's tree holds it under `content`."""
    out = {}
    for e in tree["entries"]:
        if e["type"] == "Tree" and e["path"] == "content":
            return _blobs(e["value"])
        if e["type"] == "Blob":
            out[e["path"]] = e["value"]["contents"]
    return out


def _latest(path: str, chunk: dict) -> dict:
    """toLatestVersion (snapshotChunks.ts:136-163): a legacy chunk (no version) in the v1 shape; a
    legacy header without headerMetadata gets buildHeaderMetadataForLegecyChunk's (165-185)."""
    if chunk.get("version") == "1":
        return chunk
    if chunk.get("version") is not None:
        raise ValueError(f"Unsupported chunk path: {path} version: {chunk['version']}")
    md = None
    if path == HEADER:
        md = chunk.get("headerMetadata")
        if md is None:
            ids = [{"id": HEADER}]
            if chunk["chunkLengthChars"] < chunk["totalLengthChars"]:
                ids.append({"id": BODY})
            md = {"orderedChunkMetadata": ids, "minSequenceNumber": chunk.get("chunkMinSequenceNumber"),
                  "sequenceNumber": chunk.get("chunkSequenceNumber"), "totalLength": chunk["totalLengthChars"],
                  "totalSegmentCount": chunk["totalSegmentCount"]}
    return {"version": "1", "segmentCount": chunk["chunkSegmentCount"], "length": chunk["chunkLengthChars"],
            "segments": chunk["segmentTexts"], "startIndex": chunk["chunkStartSegmentIndex"], "headerMetadata": md}


def _chunks(tree: dict):
    """(header chunk, body chunks in orderedChunkMetadata order, catch-up messages) of a snapshot
    (SnapshotLoader.initialize / loadBodyAndCatchupOps, snapshotLoader.ts:36-84)."""
    blobs = _blobs(tree)
    head = _latest(HEADER, json.loads(blobs[HEADER]))
    md = head["headerMetadata"]
    ids = [c["id"] for c in md["orderedChunkMetadata"]]
    body = [_latest(i, json.loads(blobs[i])) for i in ids[1:]]
    rest = [p for p in blobs if p not in ids]
    if len(rest) > 1:
        raise ValueError("Unexpected blobs in snapshot")
    catchup = json.loads(blobs[rest[0]]) if rest else []  # the legacy catch-up ops blob (loadCatchupOps)
    return head, body, catchup


NOOP_HTLOAD = 2  # seg_kind of a local NOOP record loading PermutationVector's HandleTable (mt_oplog.h MT_NOOP_HTLOAD)


def handle_table_records(log: ol.DocLog, handles) -> None:
    """PermutationVector.load's HandleTable.load(handleTableData) (permutationvector.ts:270-275, handletable.ts:84-86):
    the summary's `handles` array (handles[0] = the free-list head, then 0 for an allocated handle or the next
    free one) as MT_NOOP_HTLOAD records, each entry two text-pool units (low, high), up to 16,383 entries a
    record (text_len is 16 bits)."""
    h = [int(x) for x in handles]
    step = 16383
    for first in range(0, len(h), step):
        part = h[first: first + step]
        toff = len(log.text)
        for v in part:
            v &= 0xFFFFFFFF
            log.text.extend((v & 0xFFFF, v >> 16))
        log.add(ol.OP_NOOP | ol.OPF_LOCAL, pos1=first, pos2=len(h))
        r = list(log.ops[-1])
        r[1], r[8], r[9] = NOOP_HTLOAD, toff, 2 * len(part)  # seg_kind, text_off, text_len
        log.ops[-1] = tuple(r)


def load_records(tree: dict, log: ol.DocLog, client_index, local_client: Optional[str] = "snapshot",
                 catchup: bool = True, handle_table=None, perm_vector: bool = False) -> dict:
    """Append a snapshot's load records to `log` (one document's event stream); returns the header
    metadata. `client_index(name)` maps a long client id to the batch's long-client index;
    `local_client` is the id startOrUpdateCollaboration gets (None: a detached load, no collaboration,
    snapshotLoader.ts:135-151). `catchup` False leaves out the catch-up messages a legacy summary carries (what
    TestClient.createFromSnapshot does: it awaits them but applies none, testClient.ts:57-73).
    SharedMatrix vectors: `handle_table` = the summary's handleTable blob (loaded first, as PermutationVector.load
    does); PermutationSegment specs keep their allocated start ([length, start]), except that with `perm_vector`
    a body segment's start is reset as PermutationVector's onDelta INSERT resets every inserted segment's
    (permutationvector.ts:297-309: loadBody inserts through insertSegments, whose delta callback fires)."""
    head, chunks, ops = _chunks(tree)
    if handle_table is not None:
        handle_table_records(log, handle_table)
    catchup = ops if catchup else []
    md = head["headerMetadata"]
    body = [spec for c in chunks for spec in c["segments"]]

    batch = [False, False]  # an open loadBody batch; a batchable segment seen (snapshotLoader.ts:207-226)

    def add(kind, spec, countdown=0):
        info = {}
        if isinstance(spec, dict) and "json" in spec:  # IJSONSegmentWithMergeInfo (snapshotChunks.ts:60-73)
            info, spec = spec, spec["json"]
        if kind == ol.OP_APPEND:
            # loadBody batches a segment whose clientId is NonCollabClient and seq UniversalSequenceNumber
            # (specToSegment: no `client`, and `seq` absent or 0; snapshotLoader.ts:93-100, 219) into one
            # insertSegments call: members after the first continue at the previous member's position
            # (MT_OPF_GROUPED, mt_oplog.h)
            seq0 = "seq" not in info or (type(info["seq"]) is int and info["seq"] == 0)
            batchable = "client" not in info and seq0
            # The reference's flushBatch never empties `batch` (208-211): every later flush and the final
            # one pass the already inserted segments to insertSegments again. Each such re-insert is a
            # no-op (the walk cannot reach root.cachedLength: the segment that forced the earlier flush
            # has seq > 0 and another client, so it is invisible under (UniversalSequenceNumber,
            # NonCollabClient), and the segment keeps its parent, so blockInsert does not throw,
            # mergeTree.ts:2236-2249); a segment batched after such a flush is placed past that point and
            # throws "MergeTree insert failed", as the engine's insert of it does. A segment with a
            # client but seq 0 would be visible there, and the re-insert would duplicate the batch.
            if not batchable and batch[1] and seq0:
                raise ValueError("snapshot body: a segment with a client and seq 0 after batched segments; the "
                                 "reference's loadBody inserts the batch twice (snapshotLoader.ts:208-226)")
            if batchable and batch[0]:
                kind |= ol.OPF_GROUPED
            batch[0] = batchable
            batch[1] = batch[1] or batchable
        seq = info.get("seq", 0)
        client = client_index(info["client"]) if info.get("client") is not None else ol.CLIENT_NONCOLLAB
        rseq = info.get("removedSeq", 0) or 0
        rcl = client_index(info["removedClient"]) if info.get("removedClient") is not None else 0
        common = dict(client=client, seq=seq, ref_seq=rseq, min_seq=rcl, pos1=countdown)
        if isinstance(spec, str):
            log.add(kind, text=spec, **common)
        elif isinstance(spec, list):  # PermutationSegment [length, start] (permutationvector.ts:40-43, 75-77)
            start = spec[1] if len(spec) > 1 and spec[1] is not None and spec[1] >= 1 else 0
            if perm_vector and (kind & 7) == ol.OP_APPEND:
                start = 0
            log.add(kind, perm=spec[0], **common)
            if start:
                r = list(log.ops[-1])
                r[8] = int(start)  # text_off: the loaded segment's start handle (mt_oplog.h)
                log.ops[-1] = tuple(r)
        elif "marker" in spec:
            log.add(kind, marker=spec["marker"]["refType"], props=spec.get("props"), **common)
        elif "items" in spec:  # SubSequence.fromJSONObject (sharedSequence.ts:23-32)
            log.add(kind, items=spec["items"], props=spec.get("props"), **common)
        else:
            log.add(kind, text=spec["text"], props=spec.get("props"), **common)

    hs = head["segments"]
    for i, spec in enumerate(hs):
        add(ol.OP_RELOAD, spec, countdown=len(hs) - i)
    if local_client is not None:
        msn = md.get("minSequenceNumber")
        log.add(ol.OP_COLLAB, client=client_index(local_client), seq=md["sequenceNumber"],
                min_seq=msn if msn is not None else md["sequenceNumber"])
    for spec in body:
        add(ol.OP_APPEND, spec)
    if catchup:  # the messages SharedString applies after loading (sequence.ts loadContent)
        from . import wire
        wire.add_messages(log, catchup, client_index)
    return md


def segment_specs(tree: dict) -> List[Any]:
    """Every segment spec of a snapshot in order (header chunk, then the body chunks)."""
    head, chunks, _ = _chunks(tree)
    return list(head["segments"]) + [spec for c in chunks for spec in c["segments"]]
