"""Per-(kernel, grid) PMC summary of rocprofv3 --pmc passes (counter_collection.csv of each pass
directory given): counters averaged per dispatch, plus derived shares (VALU/LDS busy against the
elapsed GRBM cycles, wave-cycle split).  usage: python tools/diag/pmc_by_launch.py DIR [DIR ...]"""
import collections
import csv
import glob
import sys

N_XCD, N_CU, N_SIMD = 8, 256, 1024
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            per[(key, r["Dispatch_Id"])][r["Counter_Name"]] = per[(key, r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (key, _), cs in per.items():
            for n, v in cs.items():
                acc[key][n].append(v)
for key, cs in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    line = f"{key[0][:48]:48s} grid {key[1]:>8s}"
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / N_XCD
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        wc = c["SQ_WAVE_CYCLES"]
        line += f" | wait {c['SQ_WAIT_ANY'] / wc:.2f} stall {c['SQ_WAIT_INST_ANY'] / wc:.2f} active {c['SQ_ACTIVE_INST_ANY'] / wc:.2f}"
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
        line += f" | valu/wave {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}"
    if "SQ_INSTS_LDS" in c:
        line += f" lds {c['SQ_INSTS_LDS']:.3g} salu {c.get('SQ_INSTS_SALU', 0):.3g} trans {c.get('SQ_INSTS_VALU_TRANS_F32', 0):.3g}"
        line += f" conflict/idx {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_LDS_IDX_ACTIVE', 1), 1):.2f}"
        line += f" waitinstlds {c.get('SQ_WAIT_INST_LDS', 0):.3g} activelds {c.get('SQ_ACTIVE_INST_LDS', 0):.3g}"
    if cyc and "SQ_ACTIVE_INST_VALU" in c:
        line += f" | valu_busy {4 * c['SQ_ACTIVE_INST_VALU'] / (N_SIMD * cyc):.2f} waves {c.get('SQ_WAVES', 0):.0f}"
    if cyc:
        line += f" | cycles/xcd {cyc:.3g}"
    print(line)
