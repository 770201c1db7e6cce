"""Pipelined odeint loop time per solve at the strong-scaling shard sizes (what bench.py times on
each rank), next to the kernel time and the host-only cost of one call."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
func = F.autonomous(m)
t = torch.tensor(np.linspace(0, 3.5, 35))
for B in (4096, 2048, 1024, 512):
    y0 = bench.lv_y0(B, 0).to(dev)
    with torch.no_grad():
        for _ in range(20):
            F.odeint(func, y0, t, method="rk4")
        torch.cuda.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            F.odeint(func, y0, t, method="rk4")
        torch.cuda.synchronize()
        loop = (time.perf_counter() - t0) / n
        # host cost: the same calls issued behind a long GPU wait (kernel time hidden)
        torch.cuda._sleep(int(2e9 * 0.05))
        t0 = time.perf_counter()
        for _ in range(50):
            F.odeint(func, y0, t, method="rk4")
        host = (time.perf_counter() - t0) / 50
        torch.cuda.synchronize()
    k = bench.kernel_time_ms(m, y0, t)
    print(f"B={B}: loop {loop * 1e3:.3f} ms/solve, kernel {k:.3f} ms, host issue {host * 1e3:.3f} ms/call", flush=True)
