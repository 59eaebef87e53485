"""Summarise the PMC passes of tools/gpu_check.sh (PMC=1) for the replay kernel into one JSON.

usage: python tools/pmc_summary.py OUTDIR WORKLOAD_NOTE > summary.json
Reads OUTDIR/pmc*/run_counter_collection.csv, keeps the k_replay dispatch rows and sums each
counter over them (one dispatch per pass: bench.py --steps 1 --warmup 0). traffic_bytes_per_launch
= FETCH_SIZE x 2 (gfx950) + WRITE_SIZE, KB x 1024."""
import csv
import glob
import json
import os
import sys


def main():
    out, note = sys.argv[1], sys.argv[2]
    vals, kernel = {}, None
    for path in sorted(glob.glob(os.path.join(out, "pmc*", "run_counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                if "k_replay" not in r["Kernel_Name"]:
                    continue
                kernel = r["Kernel_Name"].split("(")[0].replace("void ", "")
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {"workload": note, "kernel": kernel,
           "note": "one rocprofv3 --pmc group per run; FETCH_SIZE/WRITE_SIZE in KB"}
    res.update(vals)
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        res["traffic_bytes_per_launch"] = int(2 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024)
    if "SQ_WAIT_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
        res["wait_fraction"] = vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
