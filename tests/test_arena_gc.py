"""Text-arena compaction (arena_gc) in the middle of replay, on the GPU against the host core.

With the text arena a few times smaller than a document writes over its life, the replay compacts the arena many
times, including inside scour's append walk (the GPU plans its appends on scalars and copies them after the walk;
a walk that needs a compaction makes its planned copies first and goes on through the serial append, mt_core.h
scour_par). Every document must replay without error to the host core's digests (the host core is the CPU spec,
pinned to the oracle and the reference's fixtures elsewhere). CPU half: the host core itself compacts and matches
the large-arena digests (arena placement is not observable)."""
import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
from test_ref_goldens import caps_for


def _batch(config, ops, n):
    w = {2: gen.config2, 3: gen.config3}[config](ops)
    return w, gen.generate(w, ids=np.arange(n), threads=8)


def _caps(w, acap):
    c = caps_for(w)
    return (c["ncap"], c["hcap"], acap, c["mcap"], c["gcap"], c["ccap"]), dict(c, acap=acap)


@pytest.mark.parametrize("config,ops,acap", [(3, 4096, 6144), (2, 4000, 4096)])
def test_host_core_compacting_arena_matches_large_arena(config, ops, acap):
    w, b = _batch(config, ops, 24)
    small, _ = _caps(w, acap)
    large, _ = _caps(w, 1 << 17)
    d1, e1, _ = core_host.replay_batch(b, small)
    d2, e2, _ = core_host.replay_batch(b, large)
    assert (e1 == 0).all() and (e2 == 0).all()
    assert np.array_equal(d1, d2)


@pytest.mark.gpu
@pytest.mark.parametrize("config,ops,acap", [(3, 4096, 6144), (3, 4096, 8192), (2, 4000, 4096)])
def test_gpu_compacting_arena_matches_host_core(config, ops, acap):
    from fluidframework_amd.engine import Engine
    w, b = _batch(config, ops, 64)
    tup, kw = _caps(w, acap)
    hd, he, _ = core_host.replay_batch(b, tup)
    assert (he == 0).all()
    eng = Engine(b.ndocs, **kw)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert len(eng.promoted()) == 0, "the compacting arena must suffice without a larger profile"
    assert np.array_equal(eng.digests(), hd)


def _wide_batch():
    import dataclasses
    # refSeq lags up to 18,000 of 36,000 ops: both documents outgrow the narrow 2,048 entries (probed on the GPU,
    # tools/probe_promote.py: lag 10,000 promotes none, 14,000 one of two, 18,000 and up both)
    w = dataclasses.replace(gen.config4(36000), max_lag=18000)
    return gen.generate(w, ids=np.arange(2), threads=2)


def _tiled_caps():
    from fluidframework_amd.engine import default_caps
    c = default_caps(36000, config=4)
    return c, tuple(c[k] for k in ("ncap", "hcap", "acap", "mcap", "gcap", "ccap"))


def test_host_tiled_large_window_replays():
    b = _wide_batch()
    _, tup = _tiled_caps()
    _, err, _ = core_host.replay_batch(b, tup)
    assert (err == 0).all()


@pytest.mark.gpu
def test_gpu_tiled_narrow_to_wide_promotion_matches_host_core():
    """the narrow tiled kernel (window set and heap in LDS, 2,048 entries each) latches E_CAPACITY on a document whose
    window set outgrows it; the engine replays that document again in the wide variant (mt_replay.hip promote)"""
    from fluidframework_amd.engine import Engine
    b = _wide_batch()
    kw, tup = _tiled_caps()
    hd, he, _ = core_host.replay_batch(b, tup)
    assert (he == 0).all()
    eng = Engine(b.ndocs, **kw)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert len(eng.promoted()) == b.ndocs, "every document's window set should outgrow the narrow kernel's"
    assert np.array_equal(eng.digests(), hd)


@pytest.mark.gpu
def test_gpu_tiled_incremental_batch_crossing_narrow_capacity():
    """A replay on top of earlier batches cannot be redone from the staged log, so promotion cannot rescue it: the
    engine runs such a batch on the wide tiled kernel (mt_prof_huge.hip). The first batch (600 events per document)
    fits the narrow kernel; the second takes every document's window set past its 2,048 entries. Both documents
    must replay to the end, unpromoted, to the host core's digests of the whole log."""
    from fluidframework_amd import oplog as ol
    from fluidframework_amd.engine import Engine
    b = _wide_batch()
    kw, tup = _tiled_caps()
    hd, he, _ = core_host.replay_batch(b, tup)
    assert (he == 0).all()
    cut = 600
    head, tail = [], []
    for d in range(b.ndocs):
        ops, text, props, kv = b.doc_arrays(d)
        head.append((ops[:cut], text, props, kv))
        tail.append((ops[cut:], text, props, kv))
    eng = Engine(b.ndocs, **kw)
    eng.start_collab(b.local_long_id)
    eng.replay(ol.Batch.from_arrays(head, b.local_long_id))
    err, _ = eng.errors()
    assert (err == 0).all() and len(eng.promoted()) == 0
    eng.replay(ol.Batch.from_arrays(tail, b.local_long_id))
    err, err_op = eng.errors()
    assert (err == 0).all(), (err, err_op)
    assert len(eng.promoted()) == 0
    assert np.array_equal(eng.digests(), hd)
