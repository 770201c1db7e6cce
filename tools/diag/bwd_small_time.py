"""Fixed-grid (rk4) training iteration of the LV KAN-FET field at small batches: forward with tape +
the reverse sweep, median of 20 (host wall, synchronised).  FETODE_BWD_TPW1=0 forces the sweep at
two trajectories per wave (A/B)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

dev = torch.device("cuda:0")
t = torch.tensor(np.linspace(0, 3.5, 35))
out = {"tpw1": os.environ.get("FETODE_BWD_TPW1", "1")}
for B in (1, 64, 512, 2048, 4096):
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = O.lv_y0(B, 0).to(dev)
    ts = []
    for it in range(25):
        m.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sol = F.odeint(F.autonomous(m), y0, t, method="rk4")
        sol.square().mean().backward()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(time.perf_counter() - t0)
    out[B] = round(1e3 * float(np.median(ts)), 3)
print(json.dumps(out), flush=True)
