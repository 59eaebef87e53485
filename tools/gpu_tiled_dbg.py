"""Tiled-profile failure triage (GPU): does the failure follow the documents' data or their slot
position in the engine (byte offset of the document block)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd.engine import Engine, default_caps  # noqa: E402
import oracle_client as oc  # noqa: E402

b = gen.generate(gen.config3(2048), 16)
_, odig, _ = oc.replay_batch(b, threads=8)
caps = default_caps(2048, config=4)
for name, order in (("natural", list(range(16))), ("reversed", list(range(15, -1, -1))), ("last4", [12, 13, 14, 15]),
                    ("first4", [0, 1, 2, 3])):
    sb = b.subset(order)
    eng = Engine(sb.ndocs, **caps)
    eng.start_collab(sb.local_long_id)
    eng.replay(sb)
    err, eo = eng.errors()
    dig = eng.digests()
    ok = dig == odig[order]
    print(name, "slot errors", [(i, int(err[i]), int(eo[i])) for i in range(sb.ndocs) if err[i]],
          "digest mismatches at slots", [i for i in range(sb.ndocs) if not ok[i]], flush=True)
    del eng
