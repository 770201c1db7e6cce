"""Kernels and gaps of the bench's captured training iteration (bench.train_rate's CapturedStep,
B = 4096): run under rocprofv3 --kernel-trace; `--db <results.db>` prints the last iteration's
dispatches (name, duration, gap before it) and the per-iteration totals."""
import argparse
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--db")
ap.add_argument("--iters", type=int, default=30)
args = ap.parse_args()

if args.db:
    import sqlite3
    rows = list(sqlite3.connect(args.db).execute("select name, start, end from kernels order by start"))
    marks = [i for i, (n, s, e) in enumerate(rows) if "fused4_kernel" in n or "small6_kernel" in n]
    a, b = marks[-3], marks[-2]   # one whole iteration: from one forward launch to the next
    busy = 0
    for i in range(a, b):
        n, s, e = rows[i]
        gap = (s - rows[i - 1][2]) / 1e3
        busy += e - s
        print(f"{(e - s) / 1e3:9.2f} us  gap {gap:7.2f}  {n[:90]}")
    span = (rows[b][1] - rows[a][1]) / 1e3
    print(f"iteration span {span:.1f} us, kernels {busy / 1e3:.1f} us, gaps {span - busy / 1e3:.1f} us")
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
import fet_ode_amd.dist as D  # noqa: E402
from fet_ode_amd.training import CapturedStep  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
y0d = y0.to(dev)
target = torch.zeros(len(t), y0d.shape[0], 2, device=dev)
func = F.autonomous(model)
opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=True, capturable=True)


def it():
    opt.zero_grad(set_to_none=True)
    sol = F.odeint(func, y0d, t, method="rk4")
    loss = (sol - target).square().mean()
    loss.backward()
    D.allreduce_gradients(list(model.parameters()))
    opt.step()


step = CapturedStep(it, warmup=3, device=dev)
for _ in range(args.iters):
    step()
torch.cuda.synchronize(dev)
print("done")
