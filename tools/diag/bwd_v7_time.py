"""Fixed-grid (rk4, 34 steps) training iteration of the LV KAN-FET field: the one-kernel sweep
(fetode_backward_set_v7(0)) against the lane-group sweep + KAN sums (mode 2), median host wall of
20 synchronised iterations per batch, and the two modes' gradients at the same inputs (max relative
difference per parameter).  --B restricts to one batch (for a rocprofv3 run)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=0)
ap.add_argument("--iters", type=int, default=25)
ap.add_argument("--modes", default="0,2")
args = ap.parse_args()
lib = _lib.load()
dev = torch.device("cuda:0")
t = torch.tensor(np.linspace(0, 3.5, 35))
out = {}
for B in ((args.B,) if args.B else (64, 512, 2048, 4096, 8192)):
    grads = {}
    for mode in (int(m) for m in args.modes.split(",")):
        lib.fetode_backward_set_v7(mode)
        torch.manual_seed(0)
        m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
        y0 = O.lv_y0(B, 0).to(dev)
        ts = []
        for it in range(args.iters):
            m.zero_grad(set_to_none=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sol = F.odeint(F.autonomous(m), y0, t, method="rk4")
            sol.square().mean().backward()
            torch.cuda.synchronize()
            if it >= 5:
                ts.append(time.perf_counter() - t0)
        out[f"B{B}_mode{mode}_ms"] = round(1e3 * float(np.median(ts)), 3)
        grads[mode] = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    if len(grads) == 2:
        g0, g1 = grads.values()
        worst, wn = 0.0, ""
        for n in g0:
            sc = g0[n].abs().max().item()
            d = (g0[n] - g1[n]).abs().max().item() / max(sc, 1e-30)
            if d > worst:
                worst, wn = d, f"{n} scale {sc:.2e}"
        out[f"B{B}_grad_maxrel"] = float(f"{worst:.3e}")
        out[f"B{B}_grad_worst"] = wn
    print(json.dumps(out), flush=True)
