"""Document sharding across ranks (one process per GPU).

Documents are independent: each rank replays its own set of documents with no
data-path collective. The node's documents are split over the ranks by greedy cost bin-packing
(longest-processing-time first on a per-document cost, ties broken by document id), so a world of N
GPUs shares one fixed set of documents ("strong" scaling, the metric's "ops/s per node at 65k
docs"); `weak_ids` gives every rank its own equally sized block instead. The one collective of the
design is the all-gather of per-document 64-bit digests after the replay (verification), plus the
max-over-ranks reduction of the timed interval that bench.py reports.
"""
from __future__ import annotations

import heapq
from typing import List, Sequence

import numpy as np


def doc_range(rank: int, docs_per_rank: int) -> tuple:
    """(first doc, count) of `rank`'s block when every rank holds docs_per_rank docs (weak)."""
    return rank * docs_per_rank, docs_per_rank


def weak_ids(rank: int, docs_per_rank: int) -> np.ndarray:
    base, n = doc_range(rank, docs_per_rank)
    return np.arange(base, base + n, dtype=np.int64)


def assign(costs: Sequence[float], world: int) -> List[np.ndarray]:
    """Greedy LPT bin-packing of documents 0..len(costs)-1 over `world` ranks.

    Documents are taken in decreasing cost (equal costs: increasing id) and each goes to the rank
    with the least total cost so far (equal loads: the lowest rank). Deterministic, so every rank
    computes the same assignment without communicating. Returns each rank's document ids,
    ascending. The LPT bound: the heaviest rank carries at most 4/3 of the optimum."""
    if world < 1:
        raise ValueError("world must be >= 1")
    c = np.asarray(costs, dtype=np.float64)
    order = np.lexsort((np.arange(len(c)), -c))  # cost descending, then id ascending
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    out: List[list] = [[] for _ in range(world)]
    for d in order:
        load, r = heapq.heappop(heap)
        out[r].append(int(d))
        heapq.heappush(heap, (load + float(c[d]), r))
    return [np.asarray(sorted(x), dtype=np.int64) for x in out]


def doc_costs(batch) -> np.ndarray:
    """Replay cost of each document of an op-log batch (oplog.Batch): events x rows. A flat-profile
    event scans the document's rows (BASELINE.md A(op) = 16 B x R + ...), and the rows a log can
    create are bounded by 1 + its insert records (a split adds one row per insert, zamboni only
    merges), so events x (1 + inserts) is the bound the bin-packing balances. Known before any
    replay, from the log alone, so every rank computes the same assignment."""
    kinds = batch.ops["kind"] & 0x07
    doc_of = np.repeat(np.arange(batch.ndocs), np.diff(batch.op_off))
    events = np.diff(batch.op_off).astype(np.float64)
    inserts = np.bincount(doc_of[kinds == 0], minlength=batch.ndocs).astype(np.float64)
    return events * (1.0 + inserts)


def loads(costs: Sequence[float], parts: Sequence[np.ndarray]) -> np.ndarray:
    c = np.asarray(costs, dtype=np.float64)
    return np.asarray([c[p].sum() for p in parts])


def gather_digests(digests: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather every rank's per-document digests (uint64) into one array in rank order.
    Ranks may hold different document counts (bin-packed shards): each rank's digests are padded
    to the largest count for the collective. Over RCCL (backend "nccl") the tensors live on
    `device`; over gloo on the CPU."""
    import torch

    world = dist.get_world_size()
    counts = all_counts(len(digests), dist, device)
    m = int(counts.max()) if len(counts) else 0
    buf = np.zeros(max(m, 1), np.uint64)
    buf[: len(digests)] = digests
    t = torch.from_numpy(buf.view(np.int64))
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([p.cpu().numpy()[: counts[i]] for i, p in enumerate(parts)]).view(np.uint64)


def in_doc_order(gathered: np.ndarray, parts: Sequence[np.ndarray], ndocs: int) -> np.ndarray:
    """Reorder rank-ordered gathered values (gather_digests) into global document order."""
    out = np.zeros(ndocs, gathered.dtype)
    out[np.concatenate(parts)] = gathered
    return out


def all_counts(n: int, dist, device=None) -> np.ndarray:
    import torch

    t = torch.tensor([n], dtype=torch.int64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return np.asarray([int(p.item()) for p in parts], np.int64)


def max_over_ranks(seconds: float, dist, device=None) -> float:
    import torch

    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(n: int, dist, device=None) -> int:
    import torch

    t = torch.tensor([n], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
