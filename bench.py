"""Bench: batched merge-tree replay on MI355X (BASELINE.json metric).

One step = one full replay of this rank's synthetic workload: every document's replica is reset to
an empty collaborating state and its whole event stream is applied on the GPU (Client.applyMsg
for sequenced messages, the *Local edits for local ones). Inputs are resident in HBM before the
timed region. `value` = sequenced messages applied per second over all ranks.

Workloads (BASELINE.json configs; --config):
  3 (default, the metric's line): 65,536 documents per node, 8 clients, refSeq lag <= 64,
    local-pending replica with acks, 4,096 sequenced messages per document.
  1: the reference's TestClient conflict farm: 1 document x 8 replicas x 10k ops in rounds of 100.
  2: 4,096 documents x 10k ops, observer replica, refSeq = MSN = seq - 1.
  4: 256 large documents x 1M sequenced messages (>400k live rows each at the end): the tiled
    profile, one workgroup per document.
  5: SharedMatrix PermutationVector replay: 16,384 matrices x 2 vectors = 32,768 replicas.
Multi-GPU (one process per GPU, torchrun): --docs is the NODE total and the documents are split
over the ranks by cost bin-packing (shard.assign; "scaling": "strong", the metric's "ops/s per
node at 65k docs"); --scaling weak gives every rank --docs documents of its own instead. No
data-path collective; RCCL all-gathers per-document digests once, after timing.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5] [--docs D]
                       [--ops-per-doc O] [--scaling strong|weak] [--assign uniform|cost] [--share R/N]
                       [--no-cpu-baseline]
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

# config -> (default node docs, default ops per doc, workload description)
CONFIGS = {
    1: (8, 10_000, "config1: TestClient conflict farm, 1 doc x {docs} replicas (client 0 observes), {ops} ops "
                   "in rounds of 100, MSN = round start"),
    2: (4096, 10_000, "config2: docs x {ops} sequenced msgs, observer replica, refSeq = MSN = seq-1, 60/30/10"),
    3: (65536, 4096, "config3: docs x {ops} sequenced msgs, 8 clients, lag<=64, local-pending replica"),
    4: (256, 1_000_000, "config4: {docs} large docs x {ops} sequenced msgs, lag<=64, 70/25/5, coalescing defeated "
                        "(distinct insert props, 25% trailing newlines): >400k live rows per doc; tiled position "
                        "index, one workgroup per doc"),
    5: (32768, 4096, "config5: SharedMatrix rows+cols PermutationVector replicas x {ops} sequenced msgs each, "
                     "8 clients, lag<=64, local-pending, 50% annotate"),
}


def log(msg: str) -> None:
    import resource
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6
    print(f"[bench] {msg} (max rss {rss:.1f} GB)", file=sys.stderr, flush=True)


def cpu_workers() -> int:
    """Host cores this process may use: its CPU affinity, capped by OMP_NUM_THREADS when set (the
    GPU box sets it to the job's CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def workload(config: int, ops: int):
    from fluidframework_amd import gen
    return {1: gen.config1, 2: gen.config2, 3: gen.config3, 4: gen.config4, 5: gen.config5}[config](ops)


def generate_cached(w, ids, cache: str, key: str):
    """gen.generate, or the same batch memory-mapped from `cache` (written by an earlier run of the
    same workload on this box: profiler passes re-run the bench several times)."""
    import numpy as np
    from fluidframework_amd import gen
    from fluidframework_amd import oplog as ol
    names = [f.name for f in __import__("dataclasses").fields(ol.Batch)]
    d = os.path.join(cache, key) if cache else ""
    if d and os.path.exists(os.path.join(d, "done")):
        return ol.Batch(*[np.load(os.path.join(d, n + ".npy"), mmap_mode="r") for n in names])
    batch = gen.generate(w, ids=ids, threads=cpu_workers())
    if d:
        os.makedirs(d, exist_ok=True)
        for n in names:
            np.save(os.path.join(d, n + ".npy"), getattr(batch, n))
        open(os.path.join(d, "done"), "w").close()
    return batch


def cpu_baseline(batch, gpu_digests, workers: int, target_s: float = 15.0):
    """The oracle (CPU restatement of the reference algorithm, test infrastructure) on `workers`
    host threads over a bounded prefix of this rank's documents, sized for ~target_s seconds."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_client as oc

    nd = batch.ndocs
    probe = min(nd, workers)
    sample = batch.subset(range(probe))
    secs, odig, oerr = oc.replay_batch(sample, threads=workers)
    ns = probe
    if secs > 0 and secs < target_s / 2 and probe < nd:
        ns = int(min(nd, max(probe, probe * target_s / secs)))
        sample = batch.subset(range(ns))
        secs, odig, oerr = oc.replay_batch(sample, threads=workers)
    s_seq = int(((sample.ops["kind"] & 0xC0) == 0).sum())  # sequenced messages (a group counts once)
    match = bool((odig == gpu_digests[:ns]).all()) and bool((oerr == 0).all())
    calib = None
    cpath = os.path.join(ROOT, "profiles", "r02_cpu_calibration.json")
    if os.path.exists(cpath):  # reference (type-erased TS under node) vs this restatement, one thread each
        c = json.load(open(cpath))["cases"]
        calib = {k: round(v["oracle_over_reference"], 2) for k, v in c.items()}
    return {"value": s_seq / secs, "unit": "ops/s", "cores": workers, "kind": "port",
            "restatement_over_reference_speed": calib,
            "sample": f"first {ns} of this rank's {nd} docs ({s_seq} sequenced msgs), oracle/ C restatement "
                      f"of the reference B-tree (PartialSequenceLengths, zamboni), one document per thread, "
                      f"{workers} threads, {secs:.1f}s; digests match GPU: {match}"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="documents per node (strong) or per rank (weak)")
    ap.add_argument("--ops-per-doc", type=int, default=0, help="sequenced messages per document")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU-baseline threads (default: host share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end hand-off runs (profiler passes: their chunked launches would enter the "
                         "replay kernel's average duration)")
    ap.add_argument("--digests-out", default="", help="save the per-document digests (.npy) after the run")
    ap.add_argument("--doc-times-out", default="", help="save each document's replay start / end (.npy, 100 MHz ticks)")
    ap.add_argument("--order", choices=("cost", "doc", "measured"), default="doc",
                    help="replay dispatch order: document order (doc, default: the configs' documents are uniform and "
                         "r05b measured cost order 3 %% slower on config 3), longest-first by shard.doc_costs (cost), or "
                         "longest-first by the replay times the warm-up steps measured (measured; one more untimed step "
                         "runs in that order before timing)")
    ap.add_argument("--assign", choices=("uniform", "cost"), default="uniform",
                    help="strong scaling: bin-pack the node's documents on their message count (uniform: every "
                         "config draws the same number per document, no generation beyond the rank's share) or on "
                         "shard.doc_costs of the generated logs (cost: every rank generates the node's logs first)")
    ap.add_argument("--share", default="",
                    help="R/N: on one GPU, replay the share rank R of an N-rank strong-scaling run would get (the "
                         "per-GPU load of the multi-GPU bench, measured without the other ranks; value = that share)")
    ap.add_argument("--rehearse", action="store_true",
                    help="under torch.distributed.run on a one-GPU box: every rank on device 0, collectives over gloo "
                         "(the multi-rank path of this script end to end on real hardware; not a scaling measurement: "
                         "the ranks share one GPU)")
    ap.add_argument("--gen-cache", default=os.environ.get("MT_GEN_CACHE", ""),
                    help="directory caching generated workloads between runs (profiler passes)")
    args = ap.parse_args()

    import numpy as np
    import torch

    from fluidframework_amd import gen, shard
    from fluidframework_amd.engine import Engine, default_caps

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit(f"--gpus {args.gpus} needs one process per GPU: run under "
                             f"torch.distributed.run --nproc-per-node {args.gpus}")
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    dist = None
    device = 0 if args.rehearse else local_rank
    coll_dev = "cpu" if args.rehearse else f"cuda:{device}"  # where the collectives' tensors live
    if world > 1 or "LOCAL_WORLD_SIZE" in os.environ:  # under torch.distributed.run: RCCL even for one rank
        import torch.distributed as dist

        torch.cuda.set_device(device)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    ndef, odef, desc = CONFIGS[args.config]
    docs = args.docs or ndef
    ops = args.ops_per_doc or odef
    w = workload(args.config, ops)

    # ---- this rank's documents ----
    a_rank, a_world = rank, world  # the share of the assignment this process replays
    if args.share:
        if world != 1 or args.scaling != "strong":
            raise SystemExit("--share simulates one rank's strong-scaling share on a single process")
        a_rank, a_world = (int(x) for x in args.share.split("/"))
        if not 0 <= a_rank < a_world:
            raise SystemExit(f"--share {args.share}: need 0 <= R < N")
    t0 = time.time()
    if args.scaling == "strong":
        # LPT bin-packing (shard.assign) of the node's documents; farms (config 1) stay whole
        unit = w.nclients if args.config == 1 else 1
        if args.assign == "cost" and unit == 1:
            # every rank generates the node's logs and packs on shard.doc_costs (deterministic: no exchange)
            full = generate_cached(w, np.arange(docs), args.gen_cache, f"c{args.config}_d{docs}_o{ops}_all")
            groups = shard.assign(shard.doc_costs(full), a_world)
        else:
            # every document of a config draws the same number of sequenced messages: an even split
            full = None
            groups = shard.assign(np.full(docs // unit, float(ops)), a_world)
        mine = np.concatenate([g[:, None] * unit + np.arange(unit) for g in groups[a_rank:a_rank + 1]]).ravel()
        node_docs = docs
    else:
        full = None
        mine = shard.weak_ids(rank, docs)
        node_docs = docs * world
    key = f"c{args.config}_d{docs}_o{ops}_{args.scaling}_{args.assign}_r{a_rank}of{a_world}"
    batch = full.subset(mine) if full is not None else generate_cached(w, mine, args.gen_cache, key)
    del full
    log(f"rank {rank}: generated {batch.ndocs} docs, {batch.nops} events in {time.time() - t0:.1f}s")
    local_events = int(((batch.ops["kind"] & 0x80) != 0).sum())

    eng = Engine(batch.ndocs, device=device, **default_caps(ops, config=args.config))
    log("engine created")
    costs = shard.doc_costs(batch)
    if args.order == "cost":  # longest-first list schedule of the documents over the GPU's wave slots
        eng.set_order(np.lexsort((np.arange(batch.ndocs), -costs)).astype(np.int32))
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
    if args.order == "measured":  # list scheduling on the measured per-document replay times
        tt = eng.doc_times().astype(np.float64)
        eng.set_order(np.lexsort((np.arange(batch.ndocs), -(tt[:, 1] - tt[:, 0]))).astype(np.int32))
        log(f"reordered step: {step():.1f} ms")
    # documents that outgrow the profile are re-replayed in a larger one inside mt_engine_sync (capacity
    # promotion, include/mt_engine.h); any document still in error is reported, not a reason to stop
    err, err_op = eng.errors()
    bad = np.nonzero(err)[0]
    if len(bad):
        log(f"replay errors on {len(bad)} docs, e.g. doc {bad[0]} err {err[bad[0]]} at {err_op[bad[0]]}")
    promoted = int(len(eng.promoted()))

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

    # per-document replay times of the last timed step (GPU constant clock, 100 MHz): the spread behind the launch's tail
    tt = eng.doc_times().astype(np.float64)
    if args.doc_times_out:
        np.save(args.doc_times_out, tt)
    dur = (tt[:, 1] - tt[:, 0]) / 1e5  # ms
    span = (tt[:, 1].max() - tt[:, 0].min()) / 1e5
    doc_ms = {"mean": float(dur.mean()), "p50": float(np.median(dur)), "p99": float(np.percentile(dur, 99)),
              "max": float(dur.max()), "span": span, "order": args.order,
              "cost_corr": float(np.corrcoef(costs, dur)[0, 1]) if batch.ndocs > 2 and dur.std() > 0 else None,
              "last_start_frac": float((tt[:, 0].max() - tt[:, 0].min()) / max(1.0, tt[:, 1].max() - tt[:, 0].min()))}
    work = eng.work()  # per doc (sequenced msgs, sum R, sum W) of the last step
    seq_ops = int(work[:, 0].sum())
    alg_bytes = 16 * int(work[:, 1].sum()) + 32 * int(work[:, 2].sum())
    # end to end, outside the timed region: the host hand-off of the op logs (bounds checks on the
    # host, H2D) + reset + replay, each once: (1) serial, mt_engine_submit from pageable memory then the replay;
    # (2) overlapped, mt_engine_submit_run from pageable memory (chunk k replays while chunk k+1 is checked and
    # copied through pinned staging buffers); (3) overlapped from pinned memory (a caller that keeps its logs in
    # mt_host_alloc memory: DMA only). Each leaves the same digests as the timed steps.
    ref_digests = eng.digests()
    e2e = {}

    def e2e_run(mode, b):
        torch.cuda.synchronize(device)
        t = time.perf_counter()
        if mode == "serial":
            eng.submit(b)
            eng.reset()
            eng.run()
        else:
            eng.reset()
            eng.submit_run(b)
        eng.sync()
        t = time.perf_counter() - t
        same = bool(np.array_equal(eng.digests(), ref_digests))
        if not same:
            log(f"end-to-end ({mode}) digests differ from the timed steps'")
        return t, same

    from fluidframework_amd.engine import pinned_batch
    for mode in () if args.no_e2e else ("serial", "overlapped", "pinned"):
        if mode == "pinned":
            pb, keep = pinned_batch(batch)
            e2e[mode] = e2e_run(mode, pb)
            del pb, keep
        else:
            e2e[mode] = e2e_run(mode, batch)
        log(f"end to end ({mode}): {e2e[mode][0] * 1e3:.1f} ms")
    t_e2e = e2e["overlapped"][0] if e2e else None

    digests = ref_digests
    if args.digests_out:
        np.save(args.digests_out, digests)

    if dist:
        dev = coll_dev
        elapsed = shard.max_over_ranks(elapsed, dist, dev)
        total_seq_ops = shard.sum_over_ranks(seq_ops, dist, dev)
        total_alg = shard.sum_over_ranks(alg_bytes, dist, dev)
        # the one collective of the design: all-gather per-document digests (verification)
        shard.gather_digests(digests, dist, dev)
    else:
        total_seq_ops = seq_ops
        total_alg = alg_bytes

    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_seq_ops * args.steps / elapsed
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = alg_bytes / (avg_kernel_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(batch, digests, args.cpu_threads or cpu_workers())

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
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (mt_gen: splitmix64(0x5EED0000+doc) xoshiro256**)",
            "config": {"workload": desc.format(ops=ops, docs=docs), "config": args.config,
                       "docs_per_node": node_docs, "docs_rank0": int(batch.ndocs), "ops_per_doc": ops,
                       "local_edits_rank0": local_events,
                       "parallelism": (f"share {a_rank}/{a_world} of the docs bin-packed x{a_world} ({args.assign} "
                                       f"costs), one GPU: value is that share's rate" if args.share else
                                       f"REHEARSAL: {world} ranks on one GPU over gloo, docs bin-packed x{world} "
                                       f"(not a scaling measurement)" if args.rehearse else
                                       f"docs bin-packed x{world} ({args.assign} costs)"),
                       "docs_promoted_rank0": promoted, "docs_in_error_rank0": int(len(bad))},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "traffic_note": "PMC counters cannot be read inside this process; FETCH_SIZE/WRITE_SIZE "
                                         "of k_replay on this command are in profiles/*_traffic.json "
                                         "(tools/gpu.sh traffic:C, tools/roofline_report.py)",
                         "kernel": "k_replay_tiled" if args.config == 4 else "k_replay", "kernel_ms": avg_kernel_ms,
                         "alg_bytes_per_launch": alg_bytes, "alg_bytes_node": total_alg,
                         "alg_formula": ("tile summaries, HBM-resident bytes (BASELINE.md, round 6): A(op) = 32 B x "
                                         "window rows + 640 B + 32 B x rows written" if args.config == 4 else
                                         "flat scan (BASELINE.md): A(op) = 16 B x rows + 32 B x rows written")},
            "cpu_baseline": cpu,
            "doc_time_ms": doc_ms,
            "end_to_end": None if t_e2e is None else {"value": seq_ops / t_e2e, "unit": "ops/s", "ms": t_e2e * 1000.0, "rank": 0,
                           "covers": "reset + mt_engine_submit_run from pageable memory (host bounds checks, pinned "
                                     "staging, H2D of chunk k+1 overlapped with the replay of chunk k) + sync, one "
                                     "step, rank 0",
                           "modes": {m: {"value": seq_ops / t, "ms": t * 1000.0, "digests_equal": same}
                                     for m, (t, same) in e2e.items()},
                           "modes_note": "serial: mt_engine_submit then reset + run (no overlap); overlapped: the "
                                         "value above; pinned: the same from mt_host_alloc memory (DMA only)"},
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
