"""Document sharding across ranks (one process per GPU).

Documents are independent: rank r of a world of N replays documents
[r * docs_per_rank, (r + 1) * docs_per_rank) with no data-path collective. The one collective of the
design is the all-gather of per-document 64-bit digests after the replay (verification), plus the
max-over-ranks reduction of the timed interval that bench.py reports.
"""
from __future__ import annotations

import numpy as np


def doc_range(rank: int, docs_per_rank: int) -> tuple:
    """(first doc, count) of `rank`'s shard (weak scaling: every rank holds docs_per_rank docs)."""
    return rank * docs_per_rank, docs_per_rank


def gather_digests(digests: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather every rank's per-document digests (uint64) into one array in rank order.
    Over RCCL (backend "nccl") the tensors live on `device`; over gloo on the CPU."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(digests).view(np.int64))
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return np.concatenate([p.cpu().numpy() for p in parts]).view(np.uint64)


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
