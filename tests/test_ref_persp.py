"""Reads at past (refSeq, clientId) perspectives against the REFERENCE (tests/golden/refpersp_*.npz,
tools/make_ref_goldens.py --persp; VERDICT r3 "What's weak" #1).

tests/persp_logs.py replays config-3 and config-5 logs (whole, and cut at a random record), then asks the
reference MergeTree.getLength, getContainingSegment + getPosition and MergeTreeTextHelper.getText at refSeqs
from 24 below minSeq up to currentSeq, for every long client. The reference answers remote perspectives from
its block PartialSequenceLengths (partialLengths.ts:432-486); the engine sums the leaf visibility predicate.
The engine answers a remote perspective only when refSeq >= minSeq and refSeq >= every refSeq that client has
sent an op under (mt_kernels.h persp_refused) and returns MT_E_UNSUPPORTED otherwise. Checked here:
  - every answered query equals the reference (host core on CPU; the HIP engine through the C ABI on GPU);
  - the GPU engine refuses exactly the queries the rule names, and never answers silently differently;
  - the rule is not vacuous: among the refused perspectives, the leaf sum differs from the reference's
    answer on hundreds of queries (what the engine would have returned silently before).
"""
import os

import numpy as np
import pytest

import core_host
import persp_logs as pl
from make_goldens_sha import log_sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MT_E_UNSUPPORTED = 4


def fnv(units: str) -> int:
    h = 0xcbf29ce484222325
    for x in units.encode("utf-16-le"):
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return int(np.uint64(h).view(np.int64))


def load(name):
    z = np.load(os.path.join(GOLDEN, f"refpersp_{name}.npz"), allow_pickle=False)
    b, _ = pl.batch(name, z["cuts"])
    assert log_sha(b) == str(z["log_sha256"]), "the logs differ from the fixture's"
    return z, b


def rule(b, q):
    return np.asarray([pl.answered(b.doc(int(x[1]))[0], int(b.local_long_id[int(x[1])]), int(x[2]), int(x[3]))
                       for x in q])


def host_answer(st, x):
    kind, d, ref, cl, a, e = (int(v) for v in x)
    if kind == pl.Q_LEN:
        return [st.L.mth_length(st.h, d, ref, cl), 0, 0, 0, 0, 0]
    if kind == pl.Q_SEG:
        return list(st.containing(d, a, ref, cl))
    t = st.text_range(d, ref, cl, "", None if a == -(1 << 31) else a, None if e == -(1 << 31) else e)
    return [len(t), fnv(t), 0, 0, 0, 0]


@pytest.mark.parametrize("name", list(pl.SETS))
def test_host_core_answers_match_reference_where_the_engine_answers(name):
    import ctypes
    z, b = load(name)
    _, err, st = core_host.replay_batch(b, pl.CAPS[name])
    assert (err == 0).all()
    st.L.mth_length.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
    q, want = z["queries"], z["answers"]
    ok = rule(b, q)
    same = np.asarray([host_answer(st, x) == [int(v) for v in w] for x, w in zip(q, want)])
    assert same[ok].all(), [(q[i].tolist(), want[i].tolist()) for i in np.nonzero(ok & ~same)[0][:5]]
    assert ok.sum() >= 1000
    # the refused perspectives are where the leaf sum and the partial lengths part
    assert (~same[~ok]).sum() >= 100
    for k in (pl.Q_LEN, pl.Q_SEG, pl.Q_TEXT):
        assert (ok & (q[:, 0] == k)).sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])  # both config-2/3 kernel builds (mt_engine_set_variant)
@pytest.mark.parametrize("name", list(pl.SETS))
def test_gpu_answers_match_reference_or_refuse(name, waves):
    from fluidframework_amd.engine import Engine, EngineError, SegRef
    z, b = load(name)
    c = pl.CAPS[name]
    eng = Engine(b.ndocs, waves=waves, ncap=c[0], hcap=c[1], acap=c[2], mcap=c[3], gcap=c[4], ccap=c[5])
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    assert (eng.errors()[0] == 0).all()
    q, want = z["queries"], z["answers"]
    ok = rule(b, q)
    answered = 0
    for x, w, legal in zip(q, want, ok):
        kind, d, ref, cl, a, e = (int(v) for v in x)
        try:
            if kind == pl.Q_LEN:
                got = [eng.get_length(d, ref, cl), 0, 0, 0, 0, 0]
            elif kind == pl.Q_SEG:
                s = eng.get_containing_segment(d, a, ref, cl)
                got = [0] * 6 if s is None else [1, s.offset, s.length, s.seq, s.client,
                                                 eng.get_position(d, s, ref, cl)]
            else:
                t = eng.get_text(d, ref, cl, "", None if a == -(1 << 31) else a, None if e == -(1 << 31) else e)
                got = [len(t), fnv(t), 0, 0, 0, 0]
        except EngineError as ex:
            assert ex.code == MT_E_UNSUPPORTED, ex
            assert not legal, f"refused an answerable perspective {x.tolist()}"
            continue
        assert legal, f"answered a refused perspective {x.tolist()}"
        assert got == [int(v) for v in w], (x.tolist(), got, w.tolist())
        answered += 1
    assert answered == int(ok.sum()) and answered >= 1000
    eng.close()
