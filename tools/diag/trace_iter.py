"""Kernel sequence of the last training iteration from a rocprofv3 kernel-trace CSV."""
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "fused4_kernel" in r["Kernel_Name"]]
a = idx[-2]; b = idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
tot = 0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:9.1f} {d:8.1f} us  {r["Kernel_Name"][:80]}')
print(f"iteration span {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernel time {tot:.1f} us, {b - a} kernels")
