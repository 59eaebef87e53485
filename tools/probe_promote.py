"""Which config-4 refSeq lag outgrows the narrow tiled kernel's window set / heap (2,048 entries each)?
Replays a few large-lag documents per lag on the GPU and on the host core; prints promotions and digest parity."""
import dataclasses
import sys
import time

import numpy as np

sys.path[:0] = [".", "tests"]
from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.engine import Engine, default_caps  # noqa: E402
import core_host  # noqa: E402

OPS = 36000
c = default_caps(OPS, config=4)
tup = tuple(c[k] for k in ("ncap", "hcap", "acap", "mcap", "gcap", "ccap"))
for lag in (10000, 14000, 18000, 24000, 30000):
    t0 = time.time()
    w = dataclasses.replace(gen.config4(OPS), max_lag=lag)
    b = gen.generate(w, ids=np.arange(2), threads=2)
    hd, he, _ = core_host.replay_batch(b, tup)
    eng = Engine(b.ndocs, **c)
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    err, _ = eng.errors()
    print(f"lag {lag}: host err {list(he)} gpu err {list(err)} promoted {list(eng.promoted())} "
          f"digests equal {np.array_equal(eng.digests(), hd)} ({time.time() - t0:.1f} s)", flush=True)
