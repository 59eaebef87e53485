"""Reconnect — Client.regeneratePendingOp — against the REFERENCE merge-tree
(tests/golden/refregen_*.npz).

Each fixture document reconnects once (tests/regen_inject.py): at a seeded point every op in flight is
regenerated (MT_OPF_REGEN records, one per pending segment group, in queue order), and the acks of the
resubmitted messages carry one member per regenerated op. The reference (tools/ref_replay.mjs --deltas,
via tools/make_ref_goldens.py --regen) runs Client.regeneratePendingOp with each pending message and its
segment group and records the ops it returns (MT_DELTA_REGEN events: findReconnectionPostition, length,
op type) inside the delta stream, beside the callbacks. Compared: every document's digest (pending-group
counts per segment included) and its whole delta stream.
"""
import glob
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
import core_host
import regen_inject
from test_ref_goldens import caps_for
from make_goldens_sha import log_sha

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = [os.path.basename(f)[9:-4] for f in sorted(glob.glob(os.path.join(GOLDEN, "refregen_*.npz")))]


def load(name):
    z = np.load(os.path.join(GOLDEN, f"refregen_{name}.npz"), allow_pickle=False)
    w = gen.Workload(**json.loads(str(z["workload"])))
    b = gen.generate(w, ids=z["doc_ids"], threads=8)
    c = caps_for(w)
    rb = regen_inject.inject(b, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]))
    assert log_sha(rb) == str(z["log_sha256"]), "the injected logs differ from the fixture's"
    return z, w, rb, c


def test_regen_fixture_set_complete():
    assert set(NAMES) >= {"c1_farm", "c3_lagged", "c3_lagged_long", "c5_perm"}
    assert sum(int(np.load(os.path.join(GOLDEN, f"refregen_{n}.npz"))["nregen"].sum()) for n in NAMES) > 1000


@pytest.mark.parametrize("name", NAMES)
def test_host_core_reconnect_matches_reference(name):
    z, w, rb, c = load(name)
    dig, err, st = core_host.replay_batch(rb, (c["ncap"], c["hcap"], c["acap"], c["mcap"], c["gcap"], c["ccap"]),
                                          dcap=1 << 12)
    assert (err == 0).all()
    bad = np.nonzero(dig != z["digests"])[0]
    assert len(bad) == 0, f"replicas differ from the reference's after reconnect on docs {bad[:8]}"
    bad = [d for d in range(rb.ndocs) if st.deltas(d)[:2] != (int(z["nwords"][d]), int(z["hashes"][d]))]
    assert not bad, f"regenerated ops / callbacks differ from the reference's on docs {bad[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reconnect_matches_reference(name):
    from fluidframework_amd.engine import Engine
    z, w, rb, c = load(name)
    eng = Engine(rb.ndocs, dcap=1 << 12, **c)
    eng.start_collab(rb.local_long_id)
    eng.replay(rb)
    err, err_op = eng.errors()
    assert (err == 0).all(), (err[err != 0][:8], err_op[err != 0][:8])
    bad = np.nonzero(eng.digests() != z["digests"])[0]
    assert len(bad) == 0, f"HIP engine differs from the reference after reconnect on docs {bad[:8]}"
    n, h = eng.delta_state()
    bad = np.nonzero((n != z["nwords"]) | (h != z["hashes"]))[0]
    assert len(bad) == 0, f"HIP engine's regenerated ops / callbacks differ from the reference's on docs {bad[:8]}"
