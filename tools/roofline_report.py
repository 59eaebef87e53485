"""Roofline report of one config from a tools/gpu.sh output directory.

usage: python tools/roofline_report.py OUTDIR CONFIG [KERNEL_SUBSTR] > summary.json

Reads OUTDIR/bench_cC.json (or trace_cC.json: the bench line printed under the profiler),
OUTDIR/trace_cC_kernel_stats.csv (rocprofv3 --kernel-trace --stats), and whichever PMC passes
exist (pmc_FETCH_SIZE_cC, pmc_WRITE_SIZE_cC, pmc_inst_cC, pmc_wait_cC). For the replay kernel it
states:
  - frac from the committed rocprof average duration: alg_bytes_per_launch / avg_ns / 8 TB/s, and
    its ratio to the bench line's own HIP-event frac;
  - traffic per launch: FETCH_SIZE x 2 (gfx950: 128-byte requests tallied at 64 B,
    /opt/skills/guides/MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KB x 1024, and the raw (x1)
    figure; traffic / alg for both;
  - instructions per event (SQ_INSTS_* / events) and the wave-cycle wait fraction.
The PMC runs are bench.py --steps 1 --warmup 0 --no-e2e (tools/gpu.sh): one replay dispatch per run (two in
rounds before 6, with the end-to-end step), reported per dispatch.
"""
import csv
import glob
import json
import os
import sys

PEAK = 8000.0  # GB/s


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def counters(d, kernel):
    vals, n = {}, {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if kernel not in r["Kernel_Name"]:
                    continue
                k = r["Counter_Name"]
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
                n.setdefault(k, set()).add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return {k: vals[k] / max(1, len(n[k])) for k in vals}, {k: len(v) for k, v in n.items()}


def main():
    out, c = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else ("k_replay_tiled" if c == "4" else "k_replay")
    bpath = os.path.join(out, f"bench_c{c}.json")
    line = last_json(bpath if os.path.exists(bpath) else os.path.join(out, f"trace_c{c}.json"))
    rf = line["roofline"]
    alg = rf["alg_bytes_per_launch"]
    res = {"config": line["config"], "bench_value_ops_s": line["value"], "kernel": kernel,
           "alg_bytes_per_launch": alg, "alg_formula": rf.get("alg_formula"),
           "bench_kernel_ms_hip_events": rf["kernel_ms"], "bench_frac": rf["frac"]}
    ks = os.path.join(out, f"trace_c{c}_kernel_stats.csv")
    if os.path.exists(ks):
        with open(ks) as f:
            rows = [r for r in csv.DictReader(f) if kernel in r["Name"] and (kernel != "k_replay" or "tiled" not in r["Name"])]
        if rows:
            r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            avg = float(r["AverageNs"])
            res["rocprof_kernel"] = r["Name"].split("(")[0]
            res["rocprof_calls"] = int(r["Calls"])
            res["rocprof_avg_ms"] = avg / 1e6
            res["frac_from_rocprof"] = alg / avg / PEAK
            res["frac_rocprof_over_bench"] = res["frac_from_rocprof"] / rf["frac"]
    events = None
    vals = {}
    for p in ("pmc_FETCH_SIZE", "pmc_WRITE_SIZE", "pmc_inst", "pmc_wait"):
        d = os.path.join(out, f"{p}_c{c}")
        if os.path.isdir(d):
            v, n = counters(d, kernel)
            vals.update(v)
            res.setdefault("pmc_dispatches", {}).update(n)
    pl = os.path.join(out, f"pmc_inst_c{c}.json")
    work = line.get("config", {})
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        t2 = 2 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024
        t1 = vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024
        res.update(FETCH_SIZE_kb=vals["FETCH_SIZE"], WRITE_SIZE_kb=vals["WRITE_SIZE"],
                   traffic_bytes_per_launch=int(t2), traffic_over_alg=t2 / alg,
                   traffic_raw_bytes_per_launch=int(t1), traffic_raw_over_alg=t1 / alg)
        if "rocprof_avg_ms" in res:
            res["traffic_GBps"] = t2 / (res["rocprof_avg_ms"] * 1e6)
    seq_ops = line["value"] * line["ms_per_step"] / 1000.0
    events = seq_ops  # sequenced messages per launch (one step = one launch)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
              "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
        if k in vals:
            res[k + "_per_seq_msg"] = vals[k] / events
    if "SQ_WAIT_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
        res["wait_fraction"] = vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]
        res["wait_inst_fraction"] = vals.get("SQ_WAIT_INST_ANY", 0) / vals["SQ_WAVE_CYCLES"]
        res["active_fraction"] = vals.get("SQ_ACTIVE_INST_ANY", 0) / vals["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in vals:
            res["lds_bank_conflict_cycles"] = vals["SQ_LDS_BANK_CONFLICT"]
    res["counters_per_dispatch"] = vals
    res["note"] = ("one rocprofv3 --pmc group per run of bench.py --steps 1 --warmup 0; per-dispatch averages; "
                   "FETCH_SIZE x2 is calibrated for 16 B/lane streaming reads only, so with this kernel's mix of "
                   "16-byte and narrower loads the read bytes lie between the raw (x1) and corrected (x2) figures")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
