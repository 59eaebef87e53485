"""MI355X-native batched replay engine for the Fluid Framework merge-tree.

The hot path (sequenced-op replay of many documents at once) runs as hand-written CDNA4 HIP
kernels inside ``libmtreplay.so`` behind a C ABI (``include/mt_engine.h``). This package holds
the op-log format (``oplog``), the synthetic workload generator (``gen``) and the ctypes host
facade mirroring the reference ``Client`` surface (``engine``).
"""
