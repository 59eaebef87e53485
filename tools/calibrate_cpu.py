"""Calibrate the CPU baseline: the reference merge-tree (type-erased, node 12)
against the oracle restatement (oracle/mt_oracle.c, which bench.py's cpu_baseline times on the GPU
box's cores) on the same op logs, single-threaded, in this container. Dev-container only: the
reference never travels to the GPU box. Writes profiles/r02_cpu_calibration.json.

usage: python tools/calibrate_cpu.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402

from fluidframework_amd import gen  # noqa: E402
import make_ref_goldens as mrg  # noqa: E402
import oracle_client as oc  # noqa: E402


def main():
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ts_erase.py"), "--out", mrg.ERASED], check=True)
    cases = {
        "C1 farm (1 doc x 8 replicas x 10k ops)": (gen.config1(10000), list(range(8))),
        "C2 subset (64 docs x 10k ops)": (gen.config2(10000), list(range(64))),
        "C3 subset (64 docs x 4,096 msgs)": (gen.config3(4096), list(range(64))),
    }
    out = {"note": "single thread each, same op logs, this container (8 x AMD EPYC); "
                   "reference = packages/dds/merge-tree/src type-erased by tools/ts_erase.py under node "
                   + subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
                   + "; restatement = oracle/mt_oracle.c (bench.py cpu_baseline 'port')", "cases": {}}
    for label, (w, ids) in cases.items():
        b = gen.generate(w, ids=ids, threads=8)
        seq = int(((b.ops["kind"] & 0x80) == 0).sum())
        d = os.path.join(mrg.SCRATCH, "calib")
        mrg.write_batch(b, gen.generator_interner(), d)
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "ref_replay.mjs"), mrg.ERASED, d, "--time"],
                           capture_output=True, text=True, check=True)
        ref_s = json.loads(r.stdout.strip().splitlines()[-1])["seconds"]
        t0 = time.time()
        secs, _, err = oc.replay_batch(b, threads=1)
        assert (err == 0).all()
        out["cases"][label] = {"sequenced_msgs": seq, "reference_s": ref_s, "reference_ops_s": seq / ref_s,
                               "oracle_s": secs, "oracle_ops_s": seq / secs, "oracle_over_reference": ref_s / secs}
        print(label, out["cases"][label], flush=True)
    with open(os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
