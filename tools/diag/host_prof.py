"""cProfile of the host side of one fused odeint call (B = 512, rk4, 35 points)."""
import cProfile
import os
import pstats
import sys

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
y0 = bench.lv_y0(512, 0).to(dev)
with torch.no_grad():
    for _ in range(20):
        F.odeint(func, y0, t, method="rk4")
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(500):
        F.odeint(func, y0, t, method="rk4")
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
