"""MergeTree-level records in generated logs (test infrastructure, mt_oplog.h MT_OPF_TREE): every third
plain remote op message becomes MergeTree.insertSegments / markRangeRemoved / annotateRange with the
message's (refSeq, clientId, seq) followed by a NOOP message of the same seq (the Client's
updateSeqNumbers), and every fourth plain local edit becomes the MergeTree-level call with the replica's
own client id, seq UnassignedSequenceNumber and refSeq = the replica's currentSeq — what applyRemoteOp and
insertSegmentLocal / removeRangeLocal / annotateRangeLocal themselves call (client.ts:164-211, 768-795).
Group messages, acks and records with other flags stay as they are."""
import numpy as np

from fluidframework_amd import oplog as ol

OPF_TREE = 0x20
OPF_GROUPED = 0x40
CLIENT_LOCAL = 0xFFFE


def to_tree_ops(b: ol.Batch) -> ol.Batch:
    per = []
    for d in range(b.ndocs):
        ops, text, props, kv = b.doc(d)
        local = int(b.local_long_id[d])
        out = []
        cur = 0
        nrem = nloc = 0
        prev_grouped = False
        for r in ops:
            k = int(r["kind"])
            base = k & 7
            plain = base <= 2 and (k & ~0x87) == 0
            if plain and not (k & ol.OPF_LOCAL) and not prev_grouped and int(r["client"]) != local:
                nrem += 1
                if nrem % 3 == 0:
                    t = r.copy()
                    t["kind"] = base | OPF_TREE
                    out.append(t)
                    n = r.copy()
                    n["kind"] = ol.OP_NOOP
                    n["text_len"] = 0
                    n["props"] = 0
                    out.append(n)
                    cur = int(r["seq"])
                    prev_grouped = False
                    continue
            if plain and (k & ol.OPF_LOCAL) and local >= 0:
                nloc += 1
                if nloc % 4 == 0:
                    t = r.copy()
                    t["kind"] = base | OPF_TREE
                    t["client"] = local
                    t["seq"] = -1
                    t["ref_seq"] = cur
                    out.append(t)
                    continue
            out.append(r)
            if not (k & ol.OPF_LOCAL) and not (k & OPF_GROUPED):
                cur = int(r["seq"])
            prev_grouped = bool(k & OPF_GROUPED) and not (k & ol.OPF_LOCAL)
        per.append((np.asarray(out, dtype=ops.dtype), text, props, kv))
    return ol.Batch.from_arrays(per, b.local_long_id)
