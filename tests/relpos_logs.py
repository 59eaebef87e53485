"""Logs with relative positions (test infrastructure; mt_oplog.h MT_SEG_RELPOS): remote clients insert text
and markers (most with a unique "markerId" property, reservedMarkerIdKey), remove and annotate ranges, and a
third of the ops name a position relative to a live marker (IRelativePosition {id, before, offset}, ops.ts:
56-61): text inserted before / after a marker with offsets, SharedString.annotateMarker's
{id, before: true} .. {id} range (opBuilder.ts:30-40), removes that start or end at a marker. Every message
has refSeq = seq - 1 and MSN = seq - 1 (each op sees the whole document), so a plain list models the
document while the log is drawn. The replica (long id 0) only observes."""
import random

import numpy as np

from fluidframework_amd import oplog as ol

RELPOS_UNITS = ol.RELPOS_UNITS
SEG_RELPOS = ol.SEG_RELPOS
MARKER_KEY = ol.MARKER_ID_KEY


def add_rel(L: ol.DocLog, kind, rel1=None, rel2=None, **kw):
    L.add_relative(kind, rel1, rel2, **kw)


def build(ndocs: int, nmsg: int, seed: int, interner=None):
    """(batch, interner, the live marker ids of each document at the end, in document order)"""
    interner = interner or ol.Interner()
    logs = []
    live = []
    for d in range(ndocs):
        rng = random.Random(seed * 1000 + d)
        L = ol.DocLog(interner, local_long_id=0)
        doc = []  # per position: ("t", char) or ("m", marker id or None)
        nid = 0
        for i in range(nmsg):
            seq = i + 1
            cl = 1 + rng.randrange(4)
            base = dict(client=cl, seq=seq, ref_seq=seq - 1, min_seq=seq - 1)
            ids = [(k, x[1]) for k, x in enumerate(doc) if x[0] == "m" and x[1] is not None]
            n = len(doc)
            r = rng.random()
            rel = ids and rng.random() < 0.35
            if r < 0.45 or n < 8:  # insert text
                t = "".join(rng.choice("abcdefgh") for _ in range(1 + rng.randrange(6)))
                if rel:
                    k, mid = rng.choice(ids)
                    before = rng.random() < 0.5
                    off = None if rng.random() < 0.4 else rng.randrange(0, 4)
                    pos = k - (off or 0) if before else k + 1 + (off or 0)
                    if 0 <= pos <= n:
                        add_rel(L, ol.OP_INSERT, (mid, before, off), None, pos1=0, text=t, **base)
                        doc[pos:pos] = [("t", c) for c in t]
                        continue
                pos = rng.randrange(n + 1)
                L.add(ol.OP_INSERT, pos1=pos, text=t, **base)
                doc[pos:pos] = [("t", c) for c in t]
            elif r < 0.6:  # insert a marker
                pos = rng.randrange(n + 1)
                mid = None
                props = None
                if rng.random() < 0.85:
                    mid = f"id{d}_{nid}"
                    nid += 1
                    props = {MARKER_KEY: mid}
                L.add(ol.OP_INSERT, pos1=pos, marker=rng.choice((0, 1)), props=props, **base)
                doc.insert(pos, ("m", mid))
            elif r < 0.8:  # remove
                if rel:
                    k, mid = rng.choice(ids)
                    if rng.random() < 0.5:  # from the marker (incl.) to a later position
                        end = min(n, k + 1 + rng.randrange(5))
                        add_rel(L, ol.OP_REMOVE, (mid, True, None), None, pos1=0, pos2=end, **base)
                        del doc[k:end]
                    else:  # from an earlier position to just before the marker
                        a = max(0, k - 1 - rng.randrange(5))
                        if a < k:
                            add_rel(L, ol.OP_REMOVE, None, (mid, True, None), pos1=a, pos2=0, **base)
                            del doc[a:k]
                    continue
                a = rng.randrange(n)
                b = min(n, a + 1 + rng.randrange(6))
                L.add(ol.OP_REMOVE, pos1=a, pos2=b, **base)
                del doc[a:b]
            else:  # annotate
                props = {"k": rng.randrange(3)}
                if rel:  # annotateMarker: exactly the marker (createAnnotateMarkerOp, opBuilder.ts:30-40)
                    k, mid = rng.choice(ids)
                    add_rel(L, ol.OP_ANNOTATE, (mid, True, None), (mid, False, None), pos1=0, pos2=0, props=props,
                            **base)
                    continue
                a = rng.randrange(n)
                b = min(n, a + 1 + rng.randrange(6))
                L.add(ol.OP_ANNOTATE, pos1=a, pos2=b, props=props, **base)
        logs.append(L)
        live.append([x[1] for x in doc if x[0] == "m" and x[1] is not None])
    return ol.Batch.from_logs(logs), interner, live


def text_of(doc_model) -> str:
    return "".join(c for k, c in doc_model if k == "t")
