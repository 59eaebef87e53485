"""The N > 1 path on CPU (gloo, world size 2).

- Weak form: each rank replays its own block of documents (shard.weak_ids).
- Strong form (bench.py's default for N > 1): one set of documents of UNEQUAL sizes is split over
  the ranks by cost bin-packing (shard.assign), each rank replays only its shard, and the digests
  are all-gathered (shard.gather_digests, ranks holding different counts) and put back in document
  order (shard.in_doc_order).
Either way the gathered digests must equal a single-process replay of all documents. The ranks
replay with the engine's own core (the serial host build of csrc/mt_core.h, libmtcore_host.so: the
same Replica code the HIP kernels run, no GPU in this tier); the single-process reference they are
compared with is the CPU oracle. bench.py runs the same shard/gather code over RCCL with the HIP
engine."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from fluidframework_amd import gen, shard
from fluidframework_amd import oplog as ol

DOCS_PER_RANK = 24
OPS = 400
STRONG_DOCS = 37


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _unequal_batch() -> ol.Batch:
    """STRONG_DOCS config-3 logs cut to very different lengths (a prefix of a replica's event
    stream is itself a valid stream)."""
    full = gen.generate(gen.config3(OPS), STRONG_DOCS, threads=2)
    per = []
    for d in range(STRONG_DOCS):
        ops, text, props, kv = full.doc(d)
        keep = 20 + (d * 97) % (len(ops) - 20)
        per.append((ops[:keep], text, props, kv))
    return ol.Batch.from_arrays(per, full.local_long_id)


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _engine_replay(b):
    """(seconds, digests, errors) of a batch replayed by the engine core's host build"""
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import core_host
    t0 = time.perf_counter()
    dig, err, _ = core_host.replay_batch(b)
    return time.perf_counter() - t0, dig, err


def _weak_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    b = gen.generate(gen.config3(OPS), ids=shard.weak_ids(rank, DOCS_PER_RANK), threads=2)
    secs, dig, err = _engine_replay(b)
    assert (err == 0).all()
    allg = shard.gather_digests(dig, dist)
    tmax = shard.max_over_ranks(secs, dist)
    total = shard.sum_over_ranks(int(b.nops), dist)
    if rank == 0:
        np.save(out, allg)
        with open(out + ".meta", "w") as f:
            f.write(f"{tmax} {total}")
    dist.barrier()
    dist.destroy_process_group()


def _strong_worker(rank, world, port, out):
    dist = _init(rank, world, port)
    full = _unequal_batch()
    parts = shard.assign(shard.doc_costs(full), world)
    mine = full.subset(parts[rank])
    _, dig, err = _engine_replay(mine)
    assert (err == 0).all()
    allg = shard.in_doc_order(shard.gather_digests(dig, dist), parts, full.ndocs)
    if rank == 0:
        np.save(out, allg)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_weak_shards_match_single_process(tmp_path):
    import oracle_client as oc

    out = str(tmp_path / "dig.npy")
    world = 2
    mp.spawn(_weak_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    gathered = np.load(out)
    full = gen.generate(gen.config3(OPS), DOCS_PER_RANK * world, threads=2)
    _, want, err = oc.replay_batch(full, threads=2)
    assert (err == 0).all()
    assert gathered.dtype == np.uint64 and len(gathered) == DOCS_PER_RANK * world
    assert (gathered == want).all()
    tmax, total = open(out + ".meta").read().split()
    assert float(tmax) > 0 and int(total) == full.nops


def test_two_rank_binpacked_unequal_docs_match_single_process(tmp_path):
    import oracle_client as oc

    out = str(tmp_path / "dig.npy")
    world = 2
    mp.spawn(_strong_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    full = _unequal_batch()
    _, want, err = oc.replay_batch(full, threads=2)
    assert (err == 0).all()
    assert (np.load(out) == want).all()


def test_assign_balances_and_covers():
    rng = np.random.default_rng(7)
    for world in (1, 2, 3, 8):
        costs = rng.integers(1, 1000, size=101)
        parts = shard.assign(costs, world)
        ids = np.sort(np.concatenate(parts))
        assert (ids == np.arange(101)).all()  # every document exactly once
        ld = shard.loads(costs, parts)
        lower = max(costs.sum() / world, costs.max())
        assert ld.max() <= 4 / 3 * lower + 1e-9  # LPT bound
        assert shard.assign(costs, world)[0].tolist() == parts[0].tolist()  # deterministic
    # equal costs: an even split
    parts = shard.assign(np.ones(65536), 8)
    assert all(len(p) == 8192 for p in parts)


def test_doc_costs_track_events_times_rows():
    b = _unequal_batch()
    c = shard.doc_costs(b)
    ev = np.diff(b.op_off)
    kinds = b.ops["kind"] & 7
    for d in (0, 5, STRONG_DOCS - 1):
        k = kinds[b.op_off[d]:b.op_off[d + 1]]
        assert c[d] == ev[d] * (1 + (k == 0).sum())
    parts = shard.assign(c, 2)
    ld = shard.loads(c, parts)
    assert ld.max() <= 4 / 3 * max(c.sum() / 2, c.max()) + 1e-9
