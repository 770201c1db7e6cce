"""Summarise rocprofv3 CSV output for the fused integrate kernel.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [<sq_dir>] --out profiles/<name>.json

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch; on gfx950 FETCH_SIZE counts exactly
half of the bytes of a wide coalesced read (MI355X_MICROARCH.md §HBM), so the corrected HBM
bytes per launch are (2*FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = os.environ.get("FETODE_PMC_KERNEL", "fused")


def counters(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KERNEL in row.get("Kernel_Name", "") and "plan_build" not in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--out") + 1]
    args = [a for a in args if a != out]
    res = {"kernel": KERNEL, "passes": {}}
    merged = {}
    for d in args:
        c, n = counters(d)
        res["passes"][d] = {"mean_per_dispatch": c, "dispatches": n}
        merged.update(c)
    if "FETCH_SIZE" in merged and "WRITE_SIZE" in merged:
        res["fetch_kib"] = merged["FETCH_SIZE"]
        res["write_kib"] = merged["WRITE_SIZE"]
        res["hbm_bytes_per_launch"] = (2 * merged["FETCH_SIZE"] + merged["WRITE_SIZE"]) * 1024
        res["correction"] = "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM); KiB -> bytes"
    res["counters"] = merged
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
