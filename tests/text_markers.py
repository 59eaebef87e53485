"""Marker segments in generated logs (test infrastructure): every second length-1 text insert of a remote
client becomes a Marker insert (length 1 too, so every later position of the log stays valid), refType
alternating Simple (0) / Tile (1). Used by the getText fixtures (tests/test_ref_text.py): the generator
itself emits no markers."""
import numpy as np

from fluidframework_amd import oplog as ol


def with_markers(b: ol.Batch) -> ol.Batch:
    ops = b.ops.copy()
    for d in range(b.ndocs):
        lo, hi = int(b.op_off[d]), int(b.op_off[d + 1])
        o = ops[lo:hi]
        cand = np.nonzero(((o["kind"] & 0x87) == ol.OP_INSERT) & (o["seg_kind"] == ol.SEG_TEXT) &
                          (o["text_len"] == 1) & (o["client"] != int(b.local_long_id[d])))[0]
        pick = cand[::2]
        o["seg_kind"][pick] = ol.SEG_MARKER
        o["text_len"][pick] = 0
        o["text_off"][pick] = 0
        o["pos2"][pick] = np.arange(len(pick)) & 1
        ops[lo:hi] = o
    return ol.Batch(ops=ops, op_off=b.op_off, text=b.text, text_off=b.text_off, props=b.props,
                    props_off=b.props_off, kv=b.kv, kv_off=b.kv_off, local_long_id=b.local_long_id)
