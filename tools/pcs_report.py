"""Summarize a rocprofv3 host-trap PC-sampling run of the replay kernel (tools/pcsample.sh): where the waves' sampled
program counters sit, by instruction class and by instruction — in particular how many samples land on the SGPR
spill traffic (v_readlane / v_writelane), on scratch (VGPR spill) loads and stores, and on memory waits.

usage: python tools/pcs_report.py gpurun_out/TAG/pcs_cC [N]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    files = [f for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True) if "pc_sampl" in os.path.basename(f)]
    if not files:
        raise SystemExit(f"no pc-sampling csv under {d}: {glob.glob(os.path.join(d, '**', '*'), recursive=True)[:20]}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            rows.extend(csv.DictReader(fh))
    cols = list(rows[0].keys()) if rows else []
    icol = next((c for c in cols if c.lower() == "instruction"), None)
    kcol = next((c for c in cols if "kernel" in c.lower() and "name" in c.lower()), None)
    by_ins, by_cls, by_off = collections.Counter(), collections.Counter(), collections.Counter()
    n = 0
    for r in rows:
        if kcol and "k_replay" not in r.get(kcol, "k_replay"):
            continue
        ins = (r.get(icol) or "?").strip() if icol else "?"
        op = ins.split()[0] if ins else "?"
        n += 1
        by_ins[op] += 1
        if op.startswith(("v_readlane", "v_writelane")):
            cls = "sgpr spill (v_readlane / v_writelane)"
        elif op.startswith("scratch_"):
            cls = "vgpr spill (scratch_*)"
        elif op.startswith("s_waitcnt"):
            cls = "s_waitcnt"
        elif op.startswith(("global_", "buffer_", "flat_")):
            cls = "vector memory"
        elif op.startswith("ds_"):
            cls = "lds"
        elif op.startswith(("s_load", "s_buffer")):
            cls = "scalar memory"
        elif op.startswith("v_"):
            cls = "valu (other)"
        elif op.startswith("s_"):
            cls = "salu / branch"
        else:
            cls = "other"
        by_cls[cls] += 1
        off = r.get("Code_Object_Offset") or r.get("code_object_offset") or r.get("Pc") or ""
        if off:
            by_off[(off, ins)] += 1
    print(f"{n} samples in k_replay ({len(rows)} total), columns: {cols}")
    for c, k in by_cls.most_common():
        print(f"  {c:40s} {k:8d}  {100.0 * k / max(n, 1):5.1f} %")
    print("top instructions:")
    for op, k in by_ins.most_common(top):
        print(f"  {op:32s} {k:8d}  {100.0 * k / max(n, 1):5.1f} %")
    if by_off:
        print("top program counters:")
        for (off, ins), k in by_off.most_common(top):
            print(f"  {off:>12s} {k:7d}  {ins}")


if __name__ == "__main__":
    main()
