"""Training-iteration timing: fwd (autograd) + bwd + Adam at B (env B, default 4096).
FETODE_FUSED_TRAINING=0 forces the per-stage path (autograd through every stage)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
from oracle import torch_ref as O

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2]).to(dev)
y0 = O.lv_y0(int(os.environ.get("B", "4096"))).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
opt = torch.optim.Adam(m.parameters(), lr=1e-4)
f = F.autonomous(m)
n = int(os.environ.get("ITERS", "6"))
for i in range(n):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    opt.zero_grad()
    sol = F.odeint(f, y0, t, method="rk4")
    torch.cuda.synchronize(); t1 = time.perf_counter()
    sol.square().mean().backward()
    torch.cuda.synchronize(); t2 = time.perf_counter()
    opt.step()
    torch.cuda.synchronize(); t3 = time.perf_counter()
    print(f"iter {i}: fwd {1e3*(t1-t0):.3f} ms  bwd {1e3*(t2-t1):.3f} ms  adam {1e3*(t3-t2):.3f} ms", flush=True)
