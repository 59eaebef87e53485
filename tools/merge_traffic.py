"""Fill roofline.traffic of a bench line from rocprofv3 PMC passes of the same command.

usage: python tools/merge_traffic.py OUTDIR  (OUTDIR from tools/gpu_bench.sh with PMC=1: bench.json,
pmc_fetch/run_counter_collection.csv, pmc_write/run_counter_collection.csv)

traffic = FETCH_SIZE x 2 + WRITE_SIZE of the replay kernel's dispatch, in bytes per launch.
FETCH_SIZE and WRITE_SIZE are reported in KB; gfx950 tallies 128-byte reads as 64 bytes in
FETCH_SIZE, hence the factor 2 (/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3 section).
Prints the bench line with traffic filled and writes OUTDIR/traffic.json."""
import csv
import json
import os
import sys


def counter(path, name, kernel="k_replay"):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == name and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for {kernel} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    out = sys.argv[1]
    fetch_kb, nf = counter(os.path.join(out, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write_kb, nw = counter(os.path.join(out, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    traffic = int(2 * fetch_kb * 1024 + write_kb * 1024)
    line = json.loads(open(os.path.join(out, "bench.json")).read().strip().splitlines()[-1])
    alg = line["roofline"]["alg_bytes_per_launch"]
    line["roofline"]["traffic"] = traffic
    raw = int(fetch_kb * 1024 + write_kb * 1024)
    t = dict(kernel="k_replay", FETCH_SIZE_kb=fetch_kb, WRITE_SIZE_kb=write_kb, dispatches=[nf, nw],
             traffic_bytes_per_launch=traffic, alg_bytes_per_launch=alg, traffic_over_alg=traffic / alg,
             traffic_raw_bytes_per_launch=raw, traffic_raw_over_alg=raw / alg,
             correction_note="the x2 FETCH_SIZE correction is calibrated for 16 B/lane streaming reads only; with "
                             "this kernel's mix of 16-byte and narrower accesses the read bytes lie between the raw "
                             "(x1) and the corrected (x2) figure",
             traffic_GBps=traffic / (line["roofline"]["kernel_ms"] * 1e6),
             config=line["config"],
             note="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate runs of bench.py --steps 1 "
                  "--warmup 0; FETCH_SIZE x2 (gfx950); KB x 1024; traffic_GBps uses the timed bench's "
                  "kernel_ms")
    json.dump(t, open(os.path.join(out, "traffic.json"), "w"), indent=1)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
