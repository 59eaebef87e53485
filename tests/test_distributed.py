"""The N > 1 path on CPU (gloo, world size 2): each rank replays its own shard of documents
(shard.doc_range) with no data-path collective, then the per-document digests are all-gathered
(shard.gather_digests) and must equal a single-process replay of all documents. The replay here is
the CPU oracle (no GPU in this tier); bench.py runs the same shard/gather code over RCCL with the
HIP engine."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from fluidframework_amd import gen, shard

DOCS_PER_RANK = 24
OPS = 400


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch.distributed as dist
    import oracle_client as oc

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base, n = shard.doc_range(rank, DOCS_PER_RANK)
    b = gen.generate(gen.config3(OPS), n, doc_base=base, threads=2)
    secs, dig, err = oc.replay_batch(b, threads=2)
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


def test_two_rank_shards_match_single_process(tmp_path):
    import oracle_client as oc

    out = str(tmp_path / "dig.npy")
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    gathered = np.load(out)
    full = gen.generate(gen.config3(OPS), DOCS_PER_RANK * world, threads=2)
    _, want, err = oc.replay_batch(full, threads=2)
    assert (err == 0).all()
    assert gathered.dtype == np.uint64 and len(gathered) == DOCS_PER_RANK * world
    assert (gathered == want).all()
    tmax, total = open(out + ".meta").read().split()
    assert float(tmax) > 0 and int(total) == full.nops
