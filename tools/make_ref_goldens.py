"""Golden vectors from the REFERENCE merge-tree itself.

TEST INFRASTRUCTURE, dev container only. Steps:
  1. tools/ts_erase.py type-erases packages/dds/merge-tree/src/*.ts into /tmp/mt-oracle (outside the
     repo; the reference never travels, in any form);
  2. for every fixture set below, the in-repo generator (fluidframework_amd/gen.py, deterministic)
     makes the op logs; they are written as raw little-endian files to a scratch dir;
  3. node runs tools/ref_replay.mjs: each replica's log through the reference `Client`
     (applyMsg / insertSegmentLocal / removeRangeLocal / annotateRangeLocal) and its canonical
     segment dump (include/mt_oplog.h);
  4. the fixture `tests/golden/ref_<set>.npz` stores the workload recipe and document ids, a
     SHA-256 of the regenerated op-log bytes (so a generator change is detected, not silently
     re-pinned), the reference's per-document FNV-1a-64 digests, its dumps of the first docs, and
     the full op logs of those first docs (self-contained vectors).
The oracle (oracle/mt_oracle.c) is checked against the same digests here; tests/test_ref_goldens.py
checks the oracle and the host core on CPU and the HIP engine on the GPU.

usage: python tools/make_ref_goldens.py [--sets c2,c3,...] [--node node]
"""
from __future__ import annotations

import argparse
import dataclasses
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from fluidframework_amd import gen  # noqa: E402
from fluidframework_amd import oplog as ol  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
ERASED = "/tmp/mt-oracle"
SCRATCH = "/tmp/mt-ref-batches"
KEEP_LOGS = 4  # documents whose full op logs + reference dumps are stored in the fixture

# fixture sets: (workload, document ids). Sizes keep each fixture well under a megabyte.
SETS = {
    "c1_farm": (gen.config1(2000), list(range(16))),                       # 2 farms x 8 replicas
    "c2_observer": (gen.config2(2000), list(range(96))),
    "c3_lagged": (gen.config3(1500), list(range(128))),
    "c3_lagged_long": (gen.config3(4096), list(range(1000, 1032))),         # the bench's doc length
    "c4_scaled": (gen.config4(20000), list(range(4))),                      # coalescing defeated, MSN advancing
    "c5_perm": (gen.config5(1500), list(range(64))),                        # PermutationSegment rows
}


def write_batch(b: ol.Batch, interner: ol.Interner, d: str) -> None:
    os.makedirs(d, exist_ok=True)
    b.ops.tofile(os.path.join(d, "ops.bin"))
    b.op_off.astype("<i8").tofile(os.path.join(d, "op_off.bin"))
    b.text.astype("<u2").tofile(os.path.join(d, "text.bin"))
    b.text_off.astype("<i8").tofile(os.path.join(d, "text_off.bin"))
    b.props.tofile(os.path.join(d, "props.bin"))
    b.props_off.astype("<i8").tofile(os.path.join(d, "props_off.bin"))
    b.kv.tofile(os.path.join(d, "kv.bin"))
    b.kv_off.astype("<i8").tofile(os.path.join(d, "kv_off.bin"))
    b.local_long_id.astype("<i4").tofile(os.path.join(d, "local.bin"))
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump({"keys": interner.keys, "values": interner.values}, f)


def log_sha(b: ol.Batch) -> str:
    h = hashlib.sha256()
    for d in range(b.ndocs):
        ops, text, props, kv = b.doc(d)
        h.update(ops.tobytes())
        used = ops[(ops["kind"] & 7) == ol.OP_INSERT]
        for o in used:
            h.update(text[o["text_off"]: o["text_off"] + o["text_len"]].tobytes())
    return h.hexdigest()


def fnv1a64(bs: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in bs:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def run_reference(b: ol.Batch, d: str, node: str):
    write_batch(b, gen.generator_interner(), d)
    t0 = time.time()
    r = subprocess.run([node, os.path.join(ROOT, "tools", "ref_replay.mjs"), ERASED, d], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"reference replay failed: {r.stderr[-2000:]}")
    info = json.loads(r.stdout.strip().splitlines()[-1])
    errs = json.load(open(os.path.join(d, "ref_err.json")))["errors"]
    if errs:
        raise RuntimeError(f"reference threw on {len(errs)} docs: {list(errs.items())[:3]}")
    blob = np.fromfile(os.path.join(d, "ref_dumps.bin"), np.uint8)
    off = np.fromfile(os.path.join(d, "ref_dump_off.bin"), "<i8")
    dumps = [blob[off[i]: off[i + 1]].tobytes() for i in range(b.ndocs)]
    return dumps, info, time.time() - t0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default=",".join(SETS))
    ap.add_argument("--node", default="node")
    args = ap.parse_args()
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ts_erase.py"), "--out", ERASED], check=True)
    import oracle_client as oc

    os.makedirs(GOLDEN, exist_ok=True)
    for name in args.sets.split(","):
        w, ids = SETS[name]
        b = gen.generate(w, ids=ids, threads=8)
        dumps, info, secs = run_reference(b, os.path.join(SCRATCH, name), args.node)
        digests = np.asarray([fnv1a64(x) for x in dumps], np.uint64)
        _, odig, oerr = oc.replay_batch(b, threads=8)
        agree = int((odig == digests).sum())
        print(f"{name}: {b.ndocs} docs, {b.nops} events, reference {info['seconds']:.2f}s; "
              f"oracle agrees on {agree}/{b.ndocs} digests", flush=True)
        keep = b.subset(range(min(KEEP_LOGS, b.ndocs)))
        np.savez_compressed(
            os.path.join(GOLDEN, f"ref_{name}.npz"),
            workload=json.dumps(dataclasses.asdict(w)), doc_ids=np.asarray(ids, np.int64), log_sha256=log_sha(b),
            digests=digests, nevents=np.diff(b.op_off),
            keep_ops=keep.ops, keep_op_off=keep.op_off, keep_text=keep.text, keep_text_off=keep.text_off,
            keep_local=keep.local_long_id,
            keep_dumps=np.frombuffer(b"".join(dumps[: keep.ndocs]), np.uint8),
            keep_dump_off=np.concatenate([[0], np.cumsum([len(x) for x in dumps[: keep.ndocs]])]).astype(np.int64),
            source=("packages/dds/merge-tree/src (reference, type-erased by tools/ts_erase.py, run under node "
                    f"{subprocess.run([args.node, '--version'], capture_output=True, text=True).stdout.strip()} by "
                    "tools/ref_replay.mjs)"),
        )


if __name__ == "__main__":
    main()
