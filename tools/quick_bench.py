"""Quick timing probe of the fused RK4 solve (not the contract bench; see bench.py)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import fet_ode_amd as F
from oracle import torch_ref as O

dev = torch.device("cuda:0")
for B in (4096, 65536):
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2]).to(dev)
    f = F.autonomous(m)
    y0 = O.lv_y0(B).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        for _ in range(5):
            F.odeint(f, y0, t, method="rk4")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            F.odeint(f, y0, t, method="rk4")
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
    print(f"B={B}: {ms:.3f} ms/solve (34 steps) -> {34/ms*1e3:.0f} RK4 steps/s", flush=True)
