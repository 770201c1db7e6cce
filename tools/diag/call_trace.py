"""Kernels and inter-kernel gaps of back-to-back inference odeint calls on the bench workload
(B = 4096 LV KAN-FET, 34 rk4 steps): run under rocprofv3 --kernel-trace, then
`python tools/diag/call_trace.py --db <results.db>` prints, per kernel name, count and average
duration, and the average gap between consecutive dispatches of the timed calls."""
import argparse
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--db")
ap.add_argument("--calls", type=int, default=40)
args = ap.parse_args()

if args.db:
    import sqlite3
    c = sqlite3.connect(args.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    rows = rows[-(args.calls * 4):]   # the tail: the timed calls
    from collections import defaultdict
    agg = defaultdict(list)
    for n, s, e in rows:
        agg[n].append(e - s)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):5d} x {sum(v) / len(v) / 1e3:9.2f} us  {n[:100]}")
    f4 = [(s, e) for n, s, e in rows if "fused4_kernel" in n][-args.calls:]
    per = sorted(f4[i + 1][0] - f4[i][0] for i in range(len(f4) - 1))
    dur = sorted(e - s for s, e in f4)
    print("fused4 start-to-start us: median %.2f mean %.2f; duration median %.2f mean %.2f" % (
        per[len(per) // 2] / 1e3, sum(per) / len(per) / 1e3, dur[len(dur) // 2] / 1e3, sum(dur) / len(dur) / 1e3))
    t0 = f4[0][0]
    others = [(n, s, e) for n, s, e in rows if s >= t0 and "fused4_kernel" not in n]
    print("other dispatches within the timed calls:", len(others))
    for n, s, e in others[:10]:
        print("   %.1f us after the first timed call: %s (%.2f us)" % ((s - t0) / 1e3, n[:60], (e - s) / 1e3))
    gaps = [rows[i + 1][1] - rows[i][2] for i in range(len(rows) - 1)]
    gaps.sort()
    print("gaps us: median %.2f  mean %.2f  max %.2f" % (gaps[len(gaps) // 2] / 1e3, sum(gaps) / len(gaps) / 1e3,
                                                          gaps[-1] / 1e3))
    span = (rows[-1][2] - rows[0][1]) / 1e3
    print(f"span of the last {len(rows)} dispatches: {span:.1f} us")
    sys.exit(0)

import torch  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
y0d = y0.to(dev)
func = F.autonomous(model)
with torch.no_grad():
    for _ in range(5):
        F.odeint(func, y0d, t, method="rk4")
    torch.cuda.synchronize(dev)
    for _ in range(args.calls):
        F.odeint(func, y0d, t, method="rk4")
    torch.cuda.synchronize(dev)
print("done")
