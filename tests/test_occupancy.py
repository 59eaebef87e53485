"""The config-2/3 profile's three k_replay builds (mt_prof_small.hip): 8 waves per SIMD (mt_small_w8.hip), 4 waves
per SIMD without VGPR spills (mt_small_w4.hip), which mt_engine_create picks when the batch's documents fit 4 per SIMD,
and the LDS-image build (mt_small_lds.hip, MT_SMALL_WAVES=1: three documents per CU). All replay the same batches to
the host core's digests (MT_SMALL_WAVES forces one build; the engine reads it at creation)."""
import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
from test_ref_goldens import caps_for


@pytest.mark.gpu
@pytest.mark.parametrize("config,ops", [(2, 3000), (3, 2048)])
@pytest.mark.parametrize("waves", ["1", "4", "8"])
def test_gpu_small_profile_builds_match_host_core(monkeypatch, config, ops, waves):
    from fluidframework_amd.engine import Engine
    w = {2: gen.config2, 3: gen.config3}[config](ops)
    b = gen.generate(w, ids=np.arange(96), threads=8)
    c = caps_for(w)
    hd, he, _ = core_host.replay_batch(b, tuple(c[k] for k in ("ncap", "hcap", "acap", "mcap", "gcap", "ccap")))
    assert (he == 0).all()
    monkeypatch.setenv("MT_SMALL_WAVES", waves)
    eng = Engine(b.ndocs, **c)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    assert (err == 0).all()
    assert np.array_equal(eng.digests(), hd)
