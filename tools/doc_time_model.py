"""Which per-document statistics of an op log predict its replay time on the GPU (the dispatch-order cost model).

Reads the per-document replay start / end a bench run saved (bench.py --doc-times-out, 100 MHz ticks), regenerates
the same documents' logs (the first N of them), replays them on the host core for the row counts, and prints the
correlation of each candidate statistic with the measured duration, plus a least-squares fit of a few.
usage: python tools/doc_time_model.py TIMES.npy [--config 3] [--ops 4096] [--n 2048]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("times")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ops", type=int, default=4096)
    ap.add_argument("--n", type=int, default=2048)
    a = ap.parse_args()
    from fluidframework_amd import gen, shard
    from fluidframework_amd import oplog as ol
    import core_host
    tt = np.load(a.times).astype(np.float64)
    dur = (tt[:, 1] - tt[:, 0]) / 1e5
    n = min(a.n, len(dur))
    w = {2: gen.config2, 3: gen.config3, 5: gen.config5}[a.config](a.ops)
    b = gen.generate(w, ids=np.arange(n), threads=8)
    dig, err, st = core_host.replay_batch(b)
    kinds = b.ops["kind"] & 7
    doc_of = np.repeat(np.arange(n), np.diff(b.op_off))
    local = (b.ops["kind"] & ol.OPF_LOCAL) != 0

    def per(mask):
        return np.bincount(doc_of[mask], minlength=n).astype(np.float64)

    stats = {
        "events": np.diff(b.op_off).astype(np.float64),
        "local": per(local),
        "inserts": per(kinds == ol.OP_INSERT),
        "removes": per(kinds == ol.OP_REMOVE),
        "annotates": per(kinds == ol.OP_ANNOTATE),
        "ins_units": np.bincount(doc_of, weights=np.where(kinds == ol.OP_INSERT, b.ops["text_len"], 0),
                                 minlength=n),
        "doc_costs": shard.doc_costs(b),
    }
    s8 = [st.stats(d) for d in range(n)]
    stats["nleaf_end"] = np.asarray([x["nleaf"] for x in s8], np.float64)
    stats["hw_slots"] = np.asarray([x["hw_slots"] for x in s8], np.float64)
    stats["arena_top"] = np.asarray([x["arena_top"] for x in s8], np.float64)
    y = dur[:n]
    print(f"{n} documents: duration mean {y.mean():.2f} ms, std {y.std():.2f}, max {y.max():.2f}")
    for k, v in stats.items():
        c = np.corrcoef(v, y)[0, 1] if v.std() > 0 else float("nan")
        print(f"  corr({k:10s}, duration) = {c:+.3f}")
    X = np.stack([np.ones(n), stats["events"], stats["inserts"], stats["hw_slots"], stats["removes"]], 1)
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    pred = X @ coef
    print("  fit 1 + events + inserts + hw_slots + removes: r =", round(float(np.corrcoef(pred, y)[0, 1]), 3),
          "coef", np.round(coef, 5).tolist())


if __name__ == "__main__":
    main()
