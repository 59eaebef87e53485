"""Leaf and node high-water marks of a synthetic config's documents, replayed on the host build of the engine core
(tests/core_host.py): how much of a document's hot image an LDS-resident kernel variant would have to hold.

usage: python tools/leaf_highwater.py [--config 2] [--docs 512] [--ops 10000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from fluidframework_amd import gen  # noqa: E402
import core_host as ch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--docs", type=int, default=512)
    ap.add_argument("--ops", type=int, default=10_000)
    a = ap.parse_args()
    wl = {2: gen.config2, 3: gen.config3, 5: gen.config5}[a.config](a.ops)
    b = gen.generate(wl, a.docs)
    _, err, st = ch.replay_batch(b)
    s = [st.stats(d) for d in range(b.ndocs)]
    leaves = np.array([x["hw_slots"] // 8 for x in s])
    nodes = np.array([x["nodes"] for x in s])
    line = 128  # HotT::Leaf: one 128-byte line per leaf
    print(f"config {a.config}: {b.ndocs} docs x {a.ops} ops, errors {int((err != 0).sum())}")
    print(f"leaf high-water: mean {leaves.mean():.1f} p50 {np.percentile(leaves, 50):.0f} "
          f"p99 {np.percentile(leaves, 99):.0f} max {leaves.max()} -> leaf lines mean {leaves.mean() * line / 1024:.1f} KB, "
          f"max {leaves.max() * line / 1024:.1f} KB")
    print(f"live nodes at the end: mean {nodes.mean():.1f} max {nodes.max()}")


if __name__ == "__main__":
    main()
