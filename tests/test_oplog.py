"""Host-side op-log logic: batch subsetting keeps per-document pools exact (bench.py's CPU
baseline replays a subset of the GPU batch and compares digests)."""
import numpy as np

from fluidframework_amd import gen
import oracle_client as oc


def test_subset_matches_full_batch():
    b = gen.generate(gen.config3(512), 64)
    _, d_full, e_full = oc.replay_batch(b, threads=4)
    assert (e_full == 0).all()
    sb = b.subset(range(10, 30))
    assert sb.ndocs == 20
    assert int(sb.text_off[-1]) <= len(sb.text)
    assert len(sb.text) < len(b.text)  # per-doc text pools are sliced, not copied whole
    _, d_sub, e_sub = oc.replay_batch(sb, threads=4)
    assert (e_sub == 0).all()
    assert (d_full[10:30] == d_sub).all()


def test_generator_is_deterministic():
    a = gen.generate(gen.config3(300), 8)
    b = gen.generate(gen.config3(300), 8, threads=3)
    assert (a.ops == b.ops).all() and (a.op_off == b.op_off).all() and (a.text == b.text).all()
    c = gen.generate(gen.config3(300), 4, doc_base=4)
    assert (c.ops == a.subset(range(4, 8)).ops).all()
