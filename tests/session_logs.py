"""Documents with many clients (test infrastructure): a generated batch whose remote clients reconnect under new long
ids ("sessions"), as a long-lived document's writers do — every reconnect is a new clientId the reference registers
in clientNameToIds (client.ts:637-661). A remote client starts a new session (probability `p`) only at a message
whose refSeq covers the client's previous message, so the renamed client has seen everything its earlier session
sent and the log's positions keep their meaning. The local replica's own id and its acks stay. With `p` = 0.5 a
1,500-message config-3 document sees several hundred distinct clients: more than the 253 short-id slots, so the
engine recycles slots (mt_core.h reclaim_shorts) while the reference keeps numbering."""
import dataclasses

import numpy as np

from fluidframework_amd import oplog as ol

FIRST_SESSION = 1000  # long ids of the sessions: past the generator's own client indices


def with_sessions(b: ol.Batch, p: float = 0.5, seed: int = 7) -> ol.Batch:
    ops = b.ops.copy()
    rng = np.random.default_rng(seed)
    nclients = []
    for d in range(b.ndocs):
        lo, hi = int(b.op_off[d]), int(b.op_off[d + 1])
        local = int(b.local_long_id[d])
        cur, last = {}, {}
        nxt = FIRST_SESSION
        in_group = False
        for i in range(lo, hi):
            r = ops[i]
            k = int(r["kind"])
            if k & ol.OPF_LOCAL or k & ol.OPF_TREE or (k & 7) >= ol.OP_RELOAD:
                continue
            c = int(r["client"])
            if c == local or c >= 0xFFFE:
                continue
            if not in_group:  # one decision per message (a group's members share it)
                if c in last and int(r["ref_seq"]) >= last[c] and rng.random() < p:
                    cur[c] = nxt
                    nxt += 1
                last[c] = int(r["seq"])
            ops["client"][i] = cur.get(c, c)
            in_group = bool(k & ol.OPF_GROUPED)
        nclients.append(len(set(int(x) for x in ops["client"][lo:hi])))
    out = dataclasses.replace(b, ops=ops)
    out.nclients = nclients  # distinct long ids per document (informational)
    return out
