"""Logs for the refsByOffset-entry KATs (a removed reference's entry keeps its shape) — test
infrastructure for tests/test_ref_entries.py and tools/make_ref_goldens.py --refentry.

The reference's LocalReferenceCollection.removeLocalRef (localReference.ts:225-264) only splices a reference out
of its entry's before / at / after list: refsByOffset[offset] stays defined, with its shape, moves with the
collection's splits and appends while the collection holds other references (split / append run only on a
non-empty collection, 126-133, 211-241), and goes away with the collection (a removed segment's localRefs =
undefined, mergeTree.ts:2673-2676; an unlinked or appended-away segment). What is observable is the entry's
kind: addLocalRef on an entry that a tombstone slide created (no `at` list) throws (195-201), and a slide onto
an entry keeps its `at` list. The handcrafted documents hit each case once; the fuzzed ones put many
references, removals and slides on a few segments of a short document with zamboni merging (minSeq lag 3).

Records: sequenced inserts / removes of client 1 or 2 (refSeq = seq - 1), and local MT_OP_REF records of the
observer replica (long id 0): pos1 = position, pos2 = ReferenceType (add), or seg_kind MT_REF_REMOVE with
pos1 = the reference's index (remove)."""
from __future__ import annotations

import numpy as np

from fluidframework_amd import oplog as ol

SLIDE = 0x40  # ReferenceType.SlideOnRemove (ops.ts)
REF_REMOVE = 1  # mt_oplog.h MT_REF_REMOVE


class _Doc:
    def __init__(self, interner, lag: int = 0):
        self.log = ol.DocLog(interner, local_long_id=0)
        self.seq = 0
        self.lag = lag
        self.length = 0
        self.nref = 0

    def _seq(self):
        self.seq += 1
        return dict(seq=self.seq, ref_seq=self.seq - 1, min_seq=max(0, self.seq - 1 - self.lag))

    def ins(self, pos: int, text: str, client: int = 1):
        self.log.add(ol.OP_INSERT, client=client, pos1=pos, text=text, **self._seq())
        self.length += len(text)

    def rem(self, a: int, b: int, client: int = 1):
        self.log.add(ol.OP_REMOVE, client=client, pos1=a, pos2=b, **self._seq())
        self.length -= b - a

    def ref(self, pos: int, slide: bool = True) -> int:
        self.log.add(ol.OP_REF | ol.OPF_LOCAL, pos1=pos, pos2=SLIDE if slide else 0)
        self.nref += 1
        return self.nref - 1

    def unref(self, i: int):
        self.log.add(ol.OP_REF | ol.OPF_LOCAL, pos1=i)
        r = list(self.log.ops[-1])
        r[1] = REF_REMOVE  # seg_kind
        self.log.ops[-1] = tuple(r)


def handcrafted(it) -> list:
    docs = []
    # (a) a slid reference (its entry: `before` only) removed, then a reference added at that offset: throws
    d = _Doc(it)
    d.ins(0, "abc"), d.ins(3, "XYZ")
    r0 = d.ref(1)
    d.rem(0, 3)          # r0 slides to "XYZ" offset 0 (addBeforeTombstones)
    d.unref(r0)
    d.ref(0)             # refsByOffset[0] has no `at`: addLocalRef throws
    d.ref(1)
    docs.append(d)
    # (b) an `at` reference removed, then a slide onto its offset, then an add there: the entry keeps `at`
    d = _Doc(it)
    d.ins(0, "abc"), d.ins(3, "XYZ")
    r0 = d.ref(3)        # "XYZ" offset 0: {at: [r0]}
    d.unref(r0)
    d.ref(1)             # in "abc"
    d.rem(0, 3)          # slides onto "XYZ" offset 0: the entry has `at`, gets `before`
    d.ref(0)             # at.push: fine
    docs.append(d)
    # (c) a slid entry moves with a split of a non-empty collection, then an add at its new offset throws
    d = _Doc(it)
    d.ins(0, "XYZW"), d.ins(4, "abc")
    d.ref(1)             # keeps "XYZW"'s collection non-empty
    r1 = d.ref(5)        # in "abc"
    d.rem(4, 7)          # past the end: r1 goes after "XYZW" offset 3 (addAfterTombstones)
    d.unref(r1)
    d.ins(2, "Q")        # splits "XYZW" at 2: the entry at 3 rides to "ZW" offset 1
    d.ref(4)             # "ZW" offset 1: no `at` there, throws
    d.ref(3)
    docs.append(d)
    # (d) the same with an empty collection: the split leaves the entry behind, the add succeeds
    d = _Doc(it)
    d.ins(0, "XYZW"), d.ins(4, "abc")
    r1 = d.ref(5)
    d.rem(4, 7)
    d.unref(r1)
    d.ins(2, "Q")
    d.ref(4)
    docs.append(d)
    # (e) a slid entry in a removed segment goes with the segment's collection; the next slide makes a new one
    d = _Doc(it)
    d.ins(0, "abc"), d.ins(3, "XYZ"), d.ins(6, "uvw")
    r0 = d.ref(1)
    d.rem(0, 3)          # r0 -> "XYZ" offset 0
    d.unref(r0)
    d.ref(4)             # "XYZ" offset 1 (keeps it non-empty)
    d.ref(1)             # "XYZ" offset 1 again
    d.rem(0, 3)          # "XYZ" removed: its collection (and the empty entry) goes; both refs slide to "uvw"
    d.ref(0)             # "uvw" offset 0 holds a fresh `before` entry: throws
    docs.append(d)
    return docs


def fuzzed(it, ndocs: int, nrec: int = 400, seed: int = 90210) -> list:
    docs = []
    for k in range(ndocs):
        rng = np.random.default_rng(seed + k)
        d = _Doc(it, lag=3)
        letters = "abcdefghij"
        for _ in range(nrec):
            u = rng.random()
            if d.length < 8 or u < 0.25:
                p = int(rng.integers(0, d.length + 1))
                n = int(rng.integers(1, 4))
                txt = "".join(letters[int(x)] for x in rng.integers(0, len(letters), n))
                if rng.random() < 0.15:
                    txt = txt[:-1] + "\n"  # a newline ends appends: more segment boundaries survive zamboni
                d.ins(p, txt, client=1 + int(rng.integers(0, 2)))
            elif u < 0.40:
                a = int(rng.integers(0, d.length))
                b = min(d.length, a + int(rng.integers(1, 4)))
                d.rem(a, b, client=1 + int(rng.integers(0, 2)))
            elif u < 0.75 and d.length > 0:
                d.ref(int(rng.integers(0, d.length)), slide=rng.random() < 0.8)
            elif d.nref > 0:
                d.unref(int(rng.integers(0, d.nref)))
        docs.append(d)
    return docs


def batch(nfuzz: int = 48) -> ol.Batch:
    it = ol.Interner()
    docs = handcrafted(it) + fuzzed(it, nfuzz)
    return ol.Batch.from_logs([d.log for d in docs])


RCAP = 256  # references per document (the fuzzed documents make ~140)
