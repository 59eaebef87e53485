"""One `TestClient`-shaped surface (packages/dds/merge-tree/src/test/testClient.ts:42-261) over
three implementations, so the reference's known-answer scenarios run unchanged against:
  - "oracle": the CPU restatement (oracle/),
  - "host":   the serial host build of the engine core,
  - "gpu":    the HIP engine (libmtreplay.so) on cuda:0.
"""
from __future__ import annotations

import numpy as np

from fluidframework_amd import oplog as ol
from fluidframework_amd.oplog import parse_dump  # noqa: F401 (re-exported for the tests)
from oracle_client import Msg, OracleClient


class _LogReplica:
    """Shared TestClient surface for the log-driven implementations (host core, GPU)."""

    def __init__(self, interner=None):
        self.interner = interner or ol.Interner()
        self.long_client_id = None

    def _apply(self, m: Msg, local: bool) -> int:
        log = ol.DocLog(self.interner)
        m.add_to(log, local)
        return self._replay_log(log)

    def apply_msg(self, m: Msg) -> int:
        return self._apply(m, False)

    def insert_text_local(self, pos, text, props=None):
        if len(text) == 0:
            return None
        m = Msg(ol.OP_INSERT, pos1=pos, text=text, props=props)
        return m if self._apply(m, True) == 0 else None

    def remove_range_local(self, start, end):
        m = Msg(ol.OP_REMOVE, pos1=start, pos2=end)
        return m if self._apply(m, True) == 0 else None

    def annotate_range_local(self, start, end, props, combining=ol.COMBINE_NONE):
        m = Msg(ol.OP_ANNOTATE, pos1=start, pos2=end, props=props, combining=combining)
        return m if self._apply(m, True) == 0 else None

    def make_op_message(self, op, seq, ref_seq=None, long_client=None, min_seq=0):
        if ref_seq is None:
            ref_seq = self.current_seq
        if long_client is None:
            long_client = self.long_client_id
        return op.sequenced(seq, ref_seq, long_client, min_seq)

    @property
    def current_seq(self):
        return parse_dump(self.dump())[0]["currentSeq"]

    def get_length(self):
        return parse_dump(self.dump())[0]["length"]


class HostReplica(_LogReplica):
    def __init__(self, interner=None):
        super().__init__(interner)
        import core_host
        self.st = core_host.HostStore(1)

    def start_collab(self, long_id, min_seq=0, cur_seq=0):
        self.long_client_id = long_id
        self.st.start_collab(0, long_id, min_seq, cur_seq)

    def _replay_log(self, log):
        ops, text, props, kv = log.arrays()
        return self.st.replay(0, ops, text, props, kv)

    @property
    def error(self):
        return self.st.error(0)

    def dump(self):
        return self.st.dump(0)

    def get_text(self):
        return self.st.text(0)


class GpuReplica(_LogReplica):
    def __init__(self, interner=None):
        super().__init__(interner)
        from fluidframework_amd.engine import Engine
        self.eng = Engine(1, ncap=256, hcap=512, acap=1 << 14, mcap=1024, gcap=256, ccap=16)

    def start_collab(self, long_id, min_seq=0, cur_seq=0):
        self.long_client_id = long_id
        self.eng.start_collab([long_id], min_seq, cur_seq)

    def _replay_log(self, log):
        self.eng.replay(ol.Batch.from_logs([log]))
        return int(self.eng.errors()[0][0])

    @property
    def error(self):
        return int(self.eng.errors()[0][0])

    def dump(self):
        return self.eng.dump(0)

    def get_text(self):
        return self.eng.get_text(0)


def make_replica(kind: str, interner=None):
    if kind == "oracle":
        return OracleClient(interner)
    if kind == "host":
        return HostReplica(interner)
    if kind == "gpu":
        return GpuReplica(interner)
    raise ValueError(kind)
