"""Per-kernel mean PMC values from rocprofv3 counter_collection CSVs (one or more pass dirs).
usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>_a gpurun_out/pmc_<tag>_b ... [--json out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].replace("(anonymous namespace)::", "")
                k = k.split("(")[0] if not k.startswith("void (") else k
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        # the kernel trace of the same pass: mean launch duration (profiled) per kernel
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].replace("(anonymous namespace)::", "")
                k = k.split("(")[0] if not k.startswith("void (") else k
                acc[k]["dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out:
        args = [a for a in args if a != out]
    res = load(args)
    for k, cs in res.items():
        print(k[:110])
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:.4g}")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
