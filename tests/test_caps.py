"""Per-document capacities past the round-1 caps, oracle vs host core vs GPU:

- removedClientOverlap longer than the 8 entries a cold row holds inline (mergeTree.ts:2700-2711
  pushes one entry per concurrent remover): 12 clients remove the same range concurrently, a
  lagging client splits the removed segment (splitAt copies the list, mergeTree.ts:523-567), and
  zamboni unlinks old rows so the per-document overflow pool is swept and reused;
- 20 distinct property keys in one document (the larger profiles hold 24 key slots);
- 250 distinct client ids are in tests/test_gpu_parity.py / test_core_host.py (byte short ids).
"""
import numpy as np
import pytest

from fluidframework_amd import oplog as ol
import core_host
import oracle_client as oc

CAPS = dict(ncap=2048, hcap=4096, acap=1 << 16, mcap=2048, gcap=256, ccap=64)
NREMOVERS = 12


def overlap_log(rounds: int = 120) -> ol.DocLog:
    """Observer replica (long id 0). Each round: NREMOVERS clients remove [p, p+3) concurrently at
    refSeq = base; client 20 (same refSeq) inserts "X" inside the range it still sees."""
    it = ol.Interner()
    log = ol.DocLog(it, local_long_id=0)
    seq = 1
    log.add(ol.OP_INSERT, client=1, seq=seq, ref_seq=0, min_seq=0, pos1=0, text="abcdefghijklmnopqrstuvwxyz" * 12)
    L = 312  # >= 120 rounds each allocate an overflow block: the 64-block pool is swept and reused
    for r in range(rounds):
        base = seq
        p = (7 * r) % (L - 4)
        for c in range(1, NREMOVERS + 1):
            seq += 1
            log.add(ol.OP_REMOVE, client=c, seq=seq, ref_seq=base, min_seq=base, pos1=p, pos2=p + 3)
        seq += 1
        log.add(ol.OP_INSERT, client=20, seq=seq, ref_seq=base, min_seq=base, pos1=p + 1, text="X")
        L = L - 3 + 1
    seq += 1  # the last rounds' rows stay in the window (removedSeq > minSeq)
    log.add(ol.OP_NOOP, client=1, seq=seq, ref_seq=seq - 1, min_seq=base)
    return log


def keys_log(nkeys: int = 20) -> ol.DocLog:
    it = ol.Interner()
    log = ol.DocLog(it, local_long_id=0)
    log.add(ol.OP_INSERT, client=1, seq=1, ref_seq=0, min_seq=0, pos1=0, text="0123456789" * 10,
            props={"a": 1, "b": "x", "c": [1, 2]})
    seq = 1
    for i in range(3 * nkeys):
        seq += 1
        log.add(ol.OP_ANNOTATE, client=1 + i % 3, seq=seq, ref_seq=seq - 1 - i % 2, min_seq=max(0, seq - 4),
                pos1=(5 * i) % 90, pos2=(5 * i) % 90 + 7, props={f"k{i % nkeys}": i, "a": None if i % 5 == 0 else i})
    return log


def _oracle(log):
    c = oc.OracleClient(log.interner)
    c.start_collab(log.local_long_id)
    assert c.replay_arrays(*log.arrays()) == 0
    return c


def _host(log):
    st = core_host.HostStore(1, tuple(CAPS[k] for k in ("ncap", "hcap", "acap", "mcap", "gcap", "ccap")))
    st.start_collab(0, log.local_long_id)
    err = st.replay(0, *log.arrays())
    return st, err


def test_long_overlap_lists_oracle_and_host():
    log = overlap_log()
    c = _oracle(log)
    _, segs = ol.parse_dump(c.dump())
    assert max(len(s["overlap"]) for s in segs) == NREMOVERS - 1  # more than the 8 held inline
    st, err = _host(log)
    assert err == 0
    assert st.dump(0) == c.dump()


def test_twenty_property_keys_oracle_and_host():
    log = keys_log()
    c = _oracle(log)
    _, segs = ol.parse_dump(c.dump())
    assert len({k for s in segs for k, _ in s["props"]}) >= 20
    st, err = _host(log)
    assert err == 0
    assert st.dump(0) == c.dump()


@pytest.mark.gpu
def test_caps_on_gpu():
    from fluidframework_amd.engine import Engine
    logs = [overlap_log(), keys_log()]
    want = [_oracle(lg).dump() for lg in logs]
    eng = Engine(len(logs), **CAPS)
    eng.start_collab([0, 0])
    # both documents share one interner only through their own tables: replay one engine per log
    for d, lg in enumerate(logs):
        e = Engine(1, **CAPS)
        e.start_collab([0])
        e.replay(ol.Batch.from_logs([lg]))
        err, _ = e.errors()
        assert err[0] == 0
        assert e.dump(0) == want[d]
        e.close()
    eng.close()


@pytest.mark.gpu
def test_capacity_promotion_mixed_batch():
    """One engine of the small profile (192 nodes / 1,536 row slots, 8 property key slots) over a mixed
    batch: config-3 documents that fit, one with 20 property keys and two coalescing-defeated documents
    with thousands of rows. The ones that overflow latch E_CAPACITY, mt_engine_sync replays them again in
    the next profiles, and every document's digest and dump equal the oracle's."""
    from fluidframework_amd import gen
    from fluidframework_amd.engine import Engine, default_caps
    small = gen.generate(gen.config3(512), 12)
    big = gen.generate(gen.config4(12000), 2)  # ~5k rows each
    docs = [small.doc_arrays(d) for d in range(small.ndocs)]
    local = [int(x) for x in small.local_long_id]
    kl = keys_log()
    docs.insert(5, kl.arrays())
    local.insert(5, kl.local_long_id)
    for d in range(big.ndocs):
        docs.append(big.doc_arrays(d))
        local.append(int(big.local_long_id[d]))
    batch = ol.Batch.from_arrays(docs, np.asarray(local, np.int32))
    want = []
    for d, arrays in enumerate(docs):
        c = oc.OracleClient()
        c.start_collab(local[d])
        assert c.replay_arrays(*arrays) == 0
        want.append(c)
    eng = Engine(batch.ndocs, **default_caps(512))
    eng.start_collab(batch.local_long_id)
    eng.replay(batch)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err, err_op)
    promoted = set(eng.promoted().tolist())
    assert {5, batch.ndocs - 2, batch.ndocs - 1} <= promoted  # 20 keys; > 1,536 rows
    assert len(promoted) < batch.ndocs // 2
    dig = eng.digests()
    for d in range(batch.ndocs):
        assert dig[d] == want[d].digest(), f"doc {d}"
        assert eng.dump(d) == want[d].dump(), f"doc {d}"
    assert eng.get_text(batch.ndocs - 1) == want[-1].get_text()
    # a second replay of the same staged batch promotes the same documents again
    eng.reset()
    eng.run()
    eng.sync()
    assert set(eng.promoted().tolist()) == promoted
    assert (eng.digests() == dig).all()


@pytest.mark.gpu
def test_capacity_promotion_incremental_batches():
    """Two submit / run / sync rounds without a reset (what GpuClient's flush does on every read): the
    coalescing-defeated documents overflow the small profile in the first round and are promoted; the
    second round's records for them replay in the promoted engine on top of the state they hold. Every
    document ends equal to the oracle over its whole log (a re-promotion from the second batch
    alone used to drop the first batch's records)."""
    from fluidframework_amd import gen
    from fluidframework_amd.engine import Engine, default_caps
    small = gen.generate(gen.config3(512), 6)
    big = gen.generate(gen.config4(12000), 2)
    docs = [small.doc_arrays(d) for d in range(small.ndocs)] + [big.doc_arrays(d) for d in range(big.ndocs)]
    local = [int(x) for x in small.local_long_id] + [int(x) for x in big.local_long_id]
    local = np.asarray(local, np.int32)

    def cut(ops):  # a record boundary that does not split a group
        i = len(ops) // 2
        while i < len(ops) and ops["kind"][i] & 0x40:
            i += 1
        return i

    halves = []
    for part in (0, 1):
        arr = []
        for o, t, p, k in docs:
            c = cut(o)
            arr.append((o[:c] if part == 0 else o[c:], t, p, k))
        halves.append(ol.Batch.from_arrays(arr, local))
    want = []
    for d, arrays in enumerate(docs):
        c = oc.OracleClient()
        c.start_collab(int(local[d]))
        assert c.replay_arrays(*arrays) == 0
        want.append(c)
    eng = Engine(len(docs), **default_caps(512))
    eng.start_collab(local)
    eng.replay(halves[0])
    first = set(eng.promoted().tolist())
    assert {len(docs) - 2, len(docs) - 1} <= first
    eng.replay(halves[1])  # no reset: the promoted documents continue in the promoted engine
    err, err_op = eng.errors()
    assert (err == 0).all(), (err, err_op)
    assert set(eng.promoted().tolist()) == first
    dig = eng.digests()
    for d in range(len(docs)):
        assert dig[d] == want[d].digest(), f"doc {d}"
    assert eng.get_text(len(docs) - 1) == want[-1].get_text()
    eng.close()
