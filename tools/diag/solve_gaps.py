"""Back-to-back bench solves (B=4096 LV KAN-FET rk4, 34 steps): host issue time per odeint call and,
under rocprofv3 --kernel-trace, the kernels each solve launches and the gaps between them
(analyse with tools/diag/solve_gaps.py --trace <kernel_trace.csv>)."""
import csv
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--trace":
    rows = list(csv.DictReader(open(sys.argv[2])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = {}
    for r in rows[-400:]:
        names[r["Kernel_Name"][:80]] = names.get(r["Kernel_Name"][:80], 0) + 1
    print("kernels in the last 400 launches:", names)
    fused = [r for r in rows if "fused4_kernel" in r["Kernel_Name"]][-150:]
    st = [int(r["Start_Timestamp"]) for r in fused]
    en = [int(r["End_Timestamp"]) for r in fused]
    dur = sum(e - s for s, e in zip(st, en)) / len(st) / 1e3
    per = (st[-1] - st[0]) / (len(st) - 1) / 1e3
    gaps = sorted((st[i + 1] - en[i]) / 1e3 for i in range(len(st) - 1))
    print(f"fused4: {dur:.1f} us per launch, {per:.1f} us start-to-start, gap median {gaps[len(gaps)//2]:.2f} "
          f"us, p90 {gaps[int(len(gaps) * 0.9)]:.2f} us")
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
g = torch.Generator().manual_seed(0)
y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=g)).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
func = F.autonomous(m)
with torch.no_grad():
    for _ in range(10):
        F.odeint(func, y0, t, method="rk4")
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        F.odeint(func, y0, t, method="rk4")
    issue = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
print(f"host issue {issue * 1e6:.1f} us per odeint call, wall {wall * 1e6:.1f} us per solve", flush=True)
