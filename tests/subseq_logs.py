"""SubSequence logs (test infrastructure, mt_oplog.h MT_SEG_RUN): a generated batch whose TextSegment inserts become
SubSequence inserts of the same units, each unit an item — the log a SharedNumberSequence replica would see
(sequence sharedSequence.ts:18-101, SharedSequence.insert 116-125: `new SubSequence(items)` + addProperties). The
positions, removes, annotates and acks are unchanged; what differs is zamboni's canAppend (MaxRun 128 instead of the
text granularity 256, no newline rule), so the trees coalesce differently and the dump carries kind 3 rows."""
import dataclasses

from fluidframework_amd import oplog as ol


def to_run(b: ol.Batch) -> ol.Batch:
    ops = b.ops.copy()
    ins = ((ops["kind"] & 7) == ol.OP_INSERT) & ((ops["seg_kind"] & 0x7F) == ol.SEG_TEXT)
    ops["seg_kind"][ins] = (ops["seg_kind"][ins] & 0x80) | ol.SEG_RUN
    return dataclasses.replace(b, ops=ops)
