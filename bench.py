"""Bench: batched merge-tree replay on MI355X (BASELINE.json metric).

One step = one full replay of this rank's synthetic workload: every document's replica is reset
to an empty collaborating state and its whole event stream (config 3 of BASELINE.json: 8
clients, refSeq lag <= 64, local-pending edits acked <= 64 seqs later, 4,096 sequenced messages
per doc) is applied on the GPU. Inputs are resident in HBM before the timed region. Documents
shard across ranks with no data-path collective ("scaling": "weak": each rank replays its own
65,536 documents); RCCL is used once, after timing, to all-gather per-document digests.

`--config 5` instead measures BASELINE.json's config 5 (SharedMatrix PermutationVector replay:
16,384 matrices x 2 vectors = 32,768 replicas, annotate-heavy PermutationSegment ops); the
default (the line the driver records) is config 3.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--docs D] [--ops-per-doc O] [--config 3|5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


WORKLOADS = {
    3: "config3: docs x {ops} sequenced msgs, 8 clients, lag<=64, local-pending replica",
    5: "config5: SharedMatrix rows+cols PermutationVector replicas x {ops} sequenced msgs each, "
       "8 clients, lag<=64, local-pending, 50% annotate",
}


def log(msg: str) -> None:
    import resource
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6
    print(f"[bench] {msg} (max rss {rss:.1f} GB)", file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=(3, 5))
    ap.add_argument("--docs", type=int, default=0, help="documents per rank (default 65536; config 5: 32768)")
    ap.add_argument("--ops-per-doc", type=int, default=4096, help="sequenced messages per document")
    ap.add_argument("--cpu-sample-docs", type=int, default=8192)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch

    from fluidframework_amd import gen, shard
    from fluidframework_amd.engine import Engine, default_caps

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    device = local_rank

    # ---- synthetic workload (config 3 or 5), this rank's shard of documents ----
    if args.docs <= 0:
        args.docs = 65536 if args.config == 3 else 32768
    w = gen.config3(args.ops_per_doc) if args.config == 3 else gen.config5(args.ops_per_doc)
    t0 = time.time()
    doc_base, ndocs = shard.doc_range(rank, args.docs)
    batch = gen.generate(w, ndocs, doc_base=doc_base, threads=args.cpu_threads)
    log(f"rank {rank}: generated {args.docs} docs, {batch.nops} events in {time.time() - t0:.1f}s")
    local_events = int(((batch.ops["kind"] & 0x80) != 0).sum())

    eng = Engine(args.docs, device=device, **default_caps(args.ops_per_doc, config=args.config))
    log("engine created")
    eng.start_collab(batch.local_long_id)
    eng.submit(batch)  # HtoD once: inputs are resident in HBM for every step
    log("inputs resident in HBM")

    def step() -> float:
        eng.reset()
        eng.run()
        eng.sync()
        return eng.last_run_ms

    for _ in range(args.warmup):
        log(f"warmup step: {step():.1f} ms")
    err, err_op = eng.errors()
    if (err != 0).any():
        bad = np.nonzero(err)[0]
        raise SystemExit(f"replay errors on {len(bad)} docs, e.g. doc {bad[0]} err {err[bad[0]]} at {err_op[bad[0]]}")

    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    t_start = time.perf_counter()
    kernel_ms = []
    for _ in range(args.steps):
        kernel_ms.append(step())
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start

    work = eng.work()  # per doc (sequenced msgs, sum R, sum W) of the last step
    seq_ops = int(work[:, 0].sum())
    alg_bytes = 16 * int(work[:, 1].sum()) + 32 * int(work[:, 2].sum())
    digests = eng.digests()

    if dist:
        dev = f"cuda:{device}"
        elapsed = shard.max_over_ranks(elapsed, dist, dev)
        total_seq_ops = shard.sum_over_ranks(seq_ops, dist, dev)
        # the one collective of the design: all-gather per-document digests (verification)
        shard.gather_digests(digests, dist, dev)
    else:
        total_seq_ops = seq_ops

    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_seq_ops * args.steps / elapsed
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = alg_bytes / (avg_kernel_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_client as oc

        ns = min(args.cpu_sample_docs, args.docs)
        sample = batch.subset(range(ns))
        secs, odig, oerr = oc.replay_batch(sample, threads=args.cpu_threads)
        s_seq = int(((sample.ops["kind"] & 0x80) == 0).sum())
        match = bool((odig == digests[:ns]).all())
        cpu = {"value": s_seq / secs, "unit": "ops/s", "cores": args.cpu_threads, "kind": "port",
               "sample": f"first {ns} of the {args.docs} docs ({s_seq} sequenced msgs), oracle B-tree "
                         f"restatement, {args.cpu_threads} threads, {secs:.1f}s; digests match GPU: {match}"}

    if rank == 0:
        out = {
            "metric": "sequenced merge-tree ops applied/sec (node) at 65k docs; HBM GB/s % of peak",
            "value": value,
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (mt_gen: splitmix64(0x5EED0000+doc) xoshiro256**)",
            "config": {"workload": WORKLOADS[args.config].format(ops=args.ops_per_doc),
                       "docs_per_gpu": args.docs, "ops_per_doc": args.ops_per_doc,
                       "local_edits_per_gpu": local_events, "parallelism": f"docs sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "k_replay", "kernel_ms": avg_kernel_ms,
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
