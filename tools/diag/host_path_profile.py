"""Host-side cost of one inference odeint call on the fused path (B = 512, the strong-scaling shard):
wall time per call without synchronisation (the host issue time), and a cProfile of 2000 calls."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
B = int(os.environ.get("B", "512"))
y0 = (0.5 + 2.5 * torch.rand(B, 2, generator=torch.Generator().manual_seed(0))).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
func = F.autonomous(m)
with torch.no_grad():
    for _ in range(20):
        F.odeint(func, y0, t, method="rk4")
    torch.cuda.synchronize()
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        F.odeint(func, y0, t, method="rk4")
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B}: host issue {1e6 * (t1 - t0) / n:.1f} us per call, wall incl. drain {1e6 * (t2 - t0) / n:.1f} us per call",
          flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        F.odeint(func, y0, t, method="rk4")
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
