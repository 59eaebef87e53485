"""GPU parity: the HIP replay engine (libmtreplay.so, through the C ABI) against the CPU oracle
on the same generated op logs — per-doc canonical-dump digests must be bit-identical, and full
dumps / perspective texts / lengths are compared for a sample of docs."""
import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd import oplog as ol
import oracle_client as oc
import persp_logs
from fluidframework_amd.engine import EngineError
from replicas import parse_dump

pytestmark = pytest.mark.gpu


def _engine(ndocs, ops_per_doc, **caps):
    from fluidframework_amd.engine import Engine, default_caps
    c = default_caps(ops_per_doc)
    c.update(caps)
    return Engine(ndocs, **c)


def fnv1a64(bs: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in bs:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _check_every_doc(eng, b: ol.Batch, gdig: np.ndarray):
    """For EVERY document: the device digest (k_digest) is FNV-1a-64 of the device's own canonical
    dump (k_dump), and the device text and local length equal the oracle's."""
    for d in range(b.ndocs):
        dump = eng.dump(d)
        assert fnv1a64(dump) == int(gdig[d]), f"doc {d}: k_digest != FNV-1a(k_dump)"
        c = oc.OracleClient()
        c.start_collab(int(b.local_long_id[d]))
        c.replay_arrays(*b.doc(d))
        assert eng.get_text(d) == c.get_text(), f"doc {d}: text"
        assert eng.get_length(d) == c.get_length(), f"doc {d}: length"


def _check_batch(b: ol.Batch, ops_per_doc: int, ndump: int = 4, every: bool = False, **caps):
    secs, odig, oerr = oc.replay_batch(b, threads=8)
    assert (oerr == 0).all()
    eng = _engine(b.ndocs, ops_per_doc, **caps)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, err_op = eng.errors()
    assert (err == 0).all(), (np.nonzero(err)[0][:8], err[err != 0][:8], err_op[err != 0][:8])
    gdig = eng.digests()
    bad = np.nonzero(gdig != odig)[0]
    if len(bad):
        d = int(bad[0])
        ops, text, props, kv = b.doc(d)
        c = oc.OracleClient()
        c.start_collab(int(b.local_long_id[d]))
        c.replay_arrays(ops, text, props, kv)
        ho, so = parse_dump(c.dump())
        hg, sg = parse_dump(eng.dump(d))
        raise AssertionError(f"{len(bad)} docs differ; doc {d}: oracle hdr {ho} gpu hdr {hg}")
    if every:
        _check_every_doc(eng, b, gdig)
    for d in range(min(ndump, b.ndocs)):
        ops, text, props, kv = b.doc(d)
        c = oc.OracleClient()
        c.start_collab(int(b.local_long_id[d]))
        c.replay_arrays(ops, text, props, kv)
        assert eng.dump(d) == c.dump()
        assert eng.get_text(d) == c.get_text()
        assert eng.get_length(d) == c.get_length()
    return eng


def test_observer_config2_small():
    b = gen.generate(gen.config2(2000), 96)
    _check_batch(b, 2000, every=True)


def test_lagged_local_config3_small():
    b = gen.generate(gen.config3(2048), 128)
    eng = _check_batch(b, 2048, every=True)
    # perspective lengths for a few remote clients at the current seq
    for d in range(4):
        ops, text, props, kv = b.doc(d)
        c = oc.OracleClient()
        c.start_collab(int(b.local_long_id[d]))
        c.replay_arrays(ops, text, props, kv)
        cur = c.current_seq
        for k in (0, 2, 5):
            assert eng.get_length(d, cur, k) == c.get_length_at(cur, k)
            assert eng.get_text(d, cur, k) == c.get_text_at(cur, k)


def test_farm_config1():
    """Config 1: the reference's conflict farm (8 replicas of one document, rounds of 100 local
    edits then sequencing); every replica matches the oracle and all replicas converge."""
    b = gen.generate(gen.config1(10000), 16)
    eng = _check_batch(b, 10000, every=True)
    for f in range(2):
        texts = {eng.get_text(8 * f + c) for c in range(8)}
        assert len(texts) == 1


def test_incremental_submits_match_one_shot():
    """Replaying a log in several submits gives the same state as one submit (state persists
    in HBM between runs, like a long-lived Client)."""
    b = gen.generate(gen.config3(1024), 32)
    one = _engine(32, 1024)
    one.start_collab(b.local_long_id)
    one.replay(b)
    inc = _engine(32, 1024)
    inc.start_collab(b.local_long_id)
    cuts = [0, 100, 517, 1024 * 2]
    for a, z in zip(cuts[:-1], cuts[1:]):
        per = []
        for d in range(32):
            ops, text, props, kv = b.doc(d)
            per.append((ops[a:z], text, props, kv))
        inc.replay(ol.Batch.from_arrays(per, b.local_long_id))
    assert (inc.digests() == one.digests()).all()


def test_large_doc_props_newlines():
    """Coalescing defeated (distinct props + trailing newlines, config 4 shape) at test size."""
    w = gen.config4(6000)
    b = gen.generate(w, 4)
    _check_batch(b, 6000, ndump=2, ncap=4096, hcap=8192, acap=1 << 17)


def test_large_doc_flat_profile_20k():
    """Config-4 shape at 20k ops/doc in the flat 16,384-node profile (~8.5k rows, ~1.8k leaves)."""
    w = gen.config4(20000)
    b = gen.generate(w, 2)
    _check_batch(b, 20000, ndump=2, ncap=16384, hcap=16384, acap=1 << 20)


def test_config4_tiled_over_100k_live_rows():
    """Config 4 on the tiled large-document profile (chunk rope + STABLE summaries + window set, one
    workgroup per document): two documents of 300k sequenced messages end with >100k live rows
    each, and replay bit-exact against the oracle."""
    from fluidframework_amd.engine import default_caps
    b = gen.generate(gen.config4(300_000), 2)
    for d in range(2):
        c = oc.OracleClient()
        c.start_collab(1)
        c.replay_arrays(*b.doc(d))
        assert c.stats()["nlive"] > 100_000
    _check_batch(b, 300_000, ndump=1, **default_caps(300_000, config=4))


def test_config4_full_length_documents():
    """Two config-4 documents at the bench's full length (1,000,000 sequenced messages each, ~400k live
    rows) on the tiled profile, bit-exact against the oracle."""
    from fluidframework_amd.engine import default_caps
    b = gen.generate(gen.config4(1_000_000), 2)
    _check_batch(b, 1_000_000, ndump=1, **default_caps(1_000_000, config=4))


def test_tiled_profile_local_pending_config3():
    """The tiled profile on config-3 documents (local-pending edits, acks, lag): same digests."""
    from fluidframework_amd.engine import default_caps
    b = gen.generate(gen.config3(2048), 16)
    _check_batch(b, 2048, ndump=2, every=True, **default_caps(2048, config=4))


def test_matrix_permutation_vectors_config5():
    """Config 5: SharedMatrix rows/cols PermutationVector replicas (PermutationSegment rows,
    annotate-heavy) in the 640-node profile; perspective lengths of remote clients agree too."""
    from fluidframework_amd.engine import default_caps
    b = gen.generate(gen.config5(4096), 64)
    eng = _check_batch(b, 4096, every=True, **default_caps(4096, config=5))
    for d in range(3):
        ops, text, props, kv = b.doc(d)
        c = oc.OracleClient()
        c.start_collab(int(b.local_long_id[d]))
        c.replay_arrays(ops, text, props, kv)
        cur = c.current_seq
        for k in (0, 3):
            # a perspective past every refSeq client k has sent an op under is answered (and equals the
            # oracle); an earlier one is refused (tests/test_ref_persp.py, mt_kernels.h persp_refused)
            if persp_logs.answered(ops, int(b.local_long_id[d]), cur - 5, k):
                assert eng.get_length(d, cur - 5, k) == c.get_length_at(cur - 5, k)
            else:
                with pytest.raises(EngineError) as ex:
                    eng.get_length(d, cur - 5, k)
                assert ex.value.code == 4
            assert eng.get_length(d, cur, k) == c.get_length_at(cur, k)


def test_containing_segment_and_position():
    """getContainingSegment / getPosition through the C ABI (mt_engine_get_containing_segment /
    mt_engine_get_position) against the oracle, flat and tiled profiles, local and current views;
    a handle round-trips: getPosition(handle) + offset == pos."""
    from fluidframework_amd.engine import default_caps
    b = gen.generate(gen.config3(2048), 3)
    rng = np.random.default_rng(9)
    for caps in (default_caps(2048), default_caps(2048, config=4)):
        eng = Engine_(b, caps)
        for d in range(3):
            c = oc.OracleClient()
            c.start_collab(int(b.local_long_id[d]))
            c.replay_arrays(*b.doc(d))
            cur = c.current_seq
            for k in (None, 0, 2, 5):
                n = c.get_length() if k is None else c.get_length_at(cur, k)
                for pos in list(rng.integers(0, max(n, 1), 8)) + [0, n - 1, n]:
                    want = c.containing(int(pos), cur, k)
                    lc = -1 if k is None else k
                    seg = eng.get_containing_segment(d, int(pos), cur, lc)
                    if not want[0]:
                        assert seg is None
                        continue
                    got = (1, seg.offset, seg.length, seg.seq, seg.client, eng.get_position(d, seg, cur, lc))
                    assert got == want, (d, k, pos, got, want)
                    assert got[5] + got[1] == pos


def Engine_(b, caps):
    from fluidframework_amd.engine import Engine
    eng = Engine(b.ndocs, **caps)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    return eng


def test_250_client_ids():
    """Documents edited by 250 distinct client ids (short ids are bytes: up to 254 per document)."""
    from test_core_host import many_clients_batch
    b = many_clients_batch()
    _check_batch(b, 3000, ndump=2, every=True)


def stalled_window_log(nbase: int = 30000, nwin: int = 3800) -> ol.DocLog:
    """A settled document of `nbase` rows (single "c\\n" segments: a newline ends every append), then a
    collaboration window of `nwin` sequenced inserts scattered over it under a minSeq that stays put (a
    client that does not advance its refSeq), then the minSeq catches up. The zamboni heap (one entry per
    leaf with rows in the window) grows to ~2,900 entries,
    with ~3,800 rows in the window set (its capacity is 4,096), and drains again."""
    it = ol.Interner()
    log = ol.DocLog(it, local_long_id=0)
    seq = 0
    rng = np.random.default_rng(7)
    length = 0
    for i in range(nbase + nwin):
        seq += 1
        ms = seq - 1 if i < nbase else nbase
        p = int(rng.integers(0, length // 2 + 1)) * 2
        log.add(ol.OP_INSERT, client=1 + i % 3, seq=seq, ref_seq=seq - 1, min_seq=ms, pos1=p, text="c\n")
        length += 2
    for i in range(600):  # the minSeq catches up in steps; each zamboni call pops two heap entries
        seq += 1
        log.add(ol.OP_NOOP, client=1, seq=seq, ref_seq=seq - 1, min_seq=min(seq - 1, nbase + (i + 1) * nwin // 300))
    return log


def test_tiled_deep_collaboration_window():
    from fluidframework_amd.engine import Engine, default_caps
    log = stalled_window_log()
    c = oc.OracleClient(log.interner)
    c.start_collab(log.local_long_id)
    assert c.replay_arrays(*log.arrays()) == 0
    eng = Engine(1, **default_caps(40_000, config=4))
    eng.start_collab([0])
    eng.replay(ol.Batch.from_logs([log]))
    err, _ = eng.errors()
    assert err[0] == 0
    assert eng.dump(0) == c.dump()
    assert eng.get_text(0) == c.get_text()
