"""Count documents whose GPU replay digest differs from the oracle (debug tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np

from fluidframework_amd import gen
from fluidframework_amd.engine import Engine, default_caps
import oracle_client as oc

cfg, n, ndocs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
b = gen.generate(getattr(gen, cfg)(n), ndocs)
_, odig, _ = oc.replay_batch(b, threads=8)
eng = Engine(b.ndocs, **default_caps(n))
for rep in range(2):
    eng.reset()
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    bad = np.nonzero(eng.digests() != odig)[0]
    print(os.environ.get("MT_REPLAY_LDS"), os.environ.get("MT_REPLAY_WAVES"), "rep", rep, "bad", len(bad), bad[:12], flush=True)

# dumps of the bad docs against the oracle, and the host FNV-1a-64 of the GPU dump vs its digest
def fnv(bs):
    h = 0xcbf29ce484222325
    for x in bs:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


gd = eng.digests()
for d in bad[:4]:
    d = int(d)
    c = oc.OracleClient()
    c.start_collab(int(b.local_long_id[d]))
    c.replay_arrays(*b.doc(d))
    g = eng.dump(d)
    print("doc", d, "dump==oracle", g == c.dump(), "fnv(gpu dump)==gpu digest", fnv(g) == int(gd[d]),
          "oracle digest==fnv(oracle dump)", fnv(c.dump()) == c.digest(), len(g), len(c.dump()), flush=True)
