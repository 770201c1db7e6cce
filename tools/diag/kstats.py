"""Print a rocprofv3 run_kernel_stats.csv as calls / mean us / name (top N)."""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    print(f'{r["Calls"]:>6} {float(r["AverageNs"]) / 1e3:10.1f} us  {r["Name"][:90]}')
